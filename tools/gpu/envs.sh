#!/bin/bash
# Library builds x environment settings on the headline config and the 8-GPU shard size.
# usage: tools/gpu/envs.sh "suffix:ENV=val,ENV=val ..."  (suffix "base" = product library)
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out/envs
for n in 100000000 12500000; do
for spec in $1; do
  v=${spec%%:*}; e=${spec#*:}; [ "$e" = "$spec" ] && e=""
  lib=astro-sph-tools_amd/lib/libasp_hip.so
  [ "$v" != base ] && lib=astro-sph-tools_amd/lib/libasp_hip_$v.so
  tag=$(echo "$spec" | tr ':=,' '___')
  env ${e//,/ } ASP_LIB=$PWD/$lib timeout -k 10 200 python bench.py --n $n --steps 10 --warmup 3 --cpu-baseline off --quiet > gpurun_out/envs/$tag.$n.json 2> gpurun_out/envs/$tag.$n.err
  rc=$?
  echo "$spec n=$n rc=$rc $(python3 -c "import json; d=json.load(open('gpurun_out/envs/$tag.$n.json')); print('step', d['ms_per_step'], d['output_ok'], {k: round(x['ms_per_launch'],3) for k,x in d['stages'].items() if x['launches']})" 2>&1 | tail -1)"
  [ $rc -ne 0 ] && exit $rc
done
done
exit 0
