#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
timeout -k 10 500 python -m pytest tests -m gpu -q -p no:cacheprovider --timeout 200 > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --cpu-baseline off > gpurun_out/bench_full.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_full.log | cut -c1-400
[ $rc -ne 0 ] && exit $rc
bash tools/profile_session.sh r1b
exit 0
