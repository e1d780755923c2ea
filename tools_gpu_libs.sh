#!/bin/bash
# run the headline bench with each given library variant (lib/libasp_hip_<name>.so)
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out/libs
for v in base "$@"; do
  lib=astro-sph-tools_amd/lib/libasp_hip.so
  [ "$v" != base ] && lib=astro-sph-tools_amd/lib/libasp_hip_$v.so
  ASP_LIB=$PWD/$lib timeout -k 10 300 python bench.py --steps 5 --warmup 2 --cpu-baseline off --quiet $BENCH_ARGS > gpurun_out/libs/$v.json 2> gpurun_out/libs/$v.err || { echo "$v failed"; tail -3 gpurun_out/libs/$v.err; exit 1; }
  echo "$v $(python3 -c "import json; d=json.load(open('gpurun_out/libs/$v.json')); print('step', d['ms_per_step'], {k: round(x['ms_per_launch'],3) for k,x in d['stages'].items() if x['launches']})")"
done
