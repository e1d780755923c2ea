#!/bin/bash
# diagnostic library variants (tools/ablate.sh) on the headline config
# usage: tools/gpu/ablate.sh MACRO "k1 k2" [bench args]
cd "$GRAFT_REPO_ROOT" || exit 9
m=$1; ks=$2; shift 2
mkdir -p gpurun_out/ablate
for v in base $ks; do
  lib=astro-sph-tools_amd/lib/libasp_hip.so
  [ "$v" != base ] && lib=astro-sph-tools_amd/lib/libasp_hip_$m$v.so
  ASP_LIB=$PWD/$lib timeout -k 10 300 python bench.py --steps 5 --warmup 2 --cpu-baseline off --quiet "$@" > gpurun_out/ablate/$m$v.json 2> gpurun_out/ablate/$m$v.err
  rc=$?
  echo "$m=$v rc=$rc $(python3 -c "import json; d=json.load(open('gpurun_out/ablate/$m$v.json')); print('step', d['ms_per_step'], {k: round(x['ms_per_launch'],3) for k,x in d['stages'].items() if x['launches']})" 2>&1 | tail -1)"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
