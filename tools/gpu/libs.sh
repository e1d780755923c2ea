#!/bin/bash
# Headline config (and the 8-GPU shard size) under several library builds.
# usage: tools/gpu/libs.sh "lib-suffix ..." [bench args]   ("base" = the product library)
cd "$GRAFT_REPO_ROOT" || exit 9
ks=$1; shift
mkdir -p gpurun_out/libs
for n in 100000000 12500000; do
for v in $ks; do
  lib=astro-sph-tools_amd/lib/libasp_hip.so
  [ "$v" != base ] && lib=astro-sph-tools_amd/lib/libasp_hip_$v.so
  ASP_LIB=$PWD/$lib timeout -k 10 200 python bench.py --n $n --steps 10 --warmup 3 --cpu-baseline off --quiet "$@" > gpurun_out/libs/$v.$n.json 2> gpurun_out/libs/$v.$n.err
  rc=$?
  echo "$v n=$n rc=$rc $(python3 -c "import json; d=json.load(open('gpurun_out/libs/$v.$n.json')); print('step', d['ms_per_step'], d['output_ok'], {k: round(x['ms_per_launch'],3) for k,x in d['stages'].items() if x['launches']})" 2>&1 | tail -1)"
  [ $rc -ne 0 ] && [ $rc -ne 3 ] && exit $rc
done
done
exit 0
