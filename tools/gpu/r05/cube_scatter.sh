#!/bin/bash
# Compacted, grouped cube scatter: cube tests, then two cube lines.
cd "$GRAFT_REPO_ROOT" || exit 9
export OUT=r05/${TAG:-cube_scatter}
bash tools/gpu/run.sh tests tests/test_gpu_cube.py tests/test_gpu_configs.py tests/test_gpu_streams.py || exit 1
bash tools/gpu/run.sh reps 2 cube --workload cube --cpu-baseline off || exit 2
