#!/bin/bash
# Same-box A/B of the working build vs ab_base: tests, then the headline and the cube,
# fresh processes alternating.
cd "$GRAFT_REPO_ROOT" || exit 9
export OUT=r05/${TAG:-ab2}
bash tools/gpu/run.sh tests tests/test_gpu_parity.py tests/test_gpu_fp64.py tests/test_gpu_cube.py tests/test_gpu_configs.py tests/test_gpu_caps.py || exit 1
B=$GRAFT_REPO_ROOT/astro-sph-tools_amd/ab_base/libasp_hip.so
for rep in 1 2 3; do
  bash tools/gpu/run.sh bench new_$rep --cpu-baseline off || exit 2
  ASP_LIB=$B bash tools/gpu/run.sh bench base_$rep --cpu-baseline off || exit 3
done
for rep in 1 2; do
  bash tools/gpu/run.sh bench cube_new_$rep --workload cube --steps 5 || exit 4
  ASP_LIB=$B bash tools/gpu/run.sh bench cube_base_$rep --workload cube --steps 5 || exit 5
done
