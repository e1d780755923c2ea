#!/bin/bash
# Sequential timed region + overlapped second region: default line, shard line, multirank test.
cd "$GRAFT_REPO_ROOT" || exit 9
export OUT=r05/${TAG:-seq_main}
bash tools/gpu/run.sh bench bench_n1 --cpu-baseline off || exit 1
bash tools/gpu/run.sh bench shard --n 12500000 --cpu-baseline off || exit 2
bash tools/gpu/run.sh tests tests/test_gpu_bench_multirank.py || exit 3
