#!/bin/bash
# Same-box A/B of the scatter's batches per iteration: working build (2) vs ab_sb1, ab_sb4,
# ab_base (before the change); parity tests on the working build first.
cd "$GRAFT_REPO_ROOT" || exit 9
export OUT=r05/${TAG:-ab_sb}
R=$GRAFT_REPO_ROOT/astro-sph-tools_amd
bash tools/gpu/run.sh tests tests/test_gpu_parity.py tests/test_gpu_fp64.py tests/test_gpu_configs.py tests/test_gpu_props.py tests/test_gpu_caps.py || exit 1
for rep in 1 2 3; do
  for lib in new sb1 sb4 base; do
    l=""; [ $lib != new ] && l="ASP_LIB=$R/ab_$lib/libasp_hip.so"
    env $l bash tools/gpu/run.sh bench ${lib}_$rep --cpu-baseline off || exit 2
  done
done
for lib in new sb1 sb4 base; do
  l=""; [ $lib != new ] && l="ASP_LIB=$R/ab_$lib/libasp_hip.so"
  env $l bash tools/gpu/run.sh bench shard_$lib --cpu-baseline off --n 12500000 --steps 30 || exit 3
done
