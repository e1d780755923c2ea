#!/bin/bash
# Cubes on two streams: tests, then one vs two streams (same box).
cd "$GRAFT_REPO_ROOT" || exit 9
export OUT=r05/${TAG:-cube_streams}
bash tools/gpu/run.sh tests tests/test_gpu_streams.py tests/test_gpu_cube.py tests/test_gpu_configs.py || exit 1
for rep in 1 2; do
  bash tools/gpu/run.sh bench cube_s1_$rep --workload cube --streams 1 --cpu-baseline off || exit 2
  bash tools/gpu/run.sh bench cube_s2_$rep --workload cube --streams 2 --cpu-baseline off || exit 3
done
