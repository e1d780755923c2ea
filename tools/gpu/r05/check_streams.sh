#!/bin/bash
# Stream defaults by world size: multirank bench tests, the default line, the cube lines.
cd "$GRAFT_REPO_ROOT" || exit 9
export OUT=r05/check_streams
bash tools/gpu/run.sh tests tests/test_gpu_bench_multirank.py tests/test_gpu_streams.py || exit 1
bash tools/gpu/run.sh bench bench_n1 --cpu-baseline off || exit 2
bash tools/gpu/run.sh reps 2 cube --workload cube --cpu-baseline off || exit 3
