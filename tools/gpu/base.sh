#!/bin/bash
# Round-2 baseline: GPU parity suite, then the default bench line (no CPU baseline).
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out/base
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/base/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/base/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --cpu-baseline off > gpurun_out/base/bench.json 2> gpurun_out/base/bench.err || { tail -5 gpurun_out/base/bench.err; exit 1; }
cut -c1-600 gpurun_out/base/bench.json
