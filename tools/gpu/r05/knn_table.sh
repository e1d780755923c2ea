#!/bin/bash
# k-NN cell table by starts + suffix minimum: tests, the 10^7 and 10^8 lines.
cd "$GRAFT_REPO_ROOT" || exit 9
export OUT=r05/knn_table
bash tools/gpu/run.sh tests tests/test_gpu_knn.py || exit 1
bash tools/gpu/run.sh bench bench_knn_1e7 --workload knn --n 10000000 --cpu-baseline off || exit 2
LIMIT=400 bash tools/gpu/run.sh bench bench_knn_1e8 --workload knn --n 100000000 --cpu-baseline off || exit 3
