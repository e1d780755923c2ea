#!/bin/bash
# full GPU suite, cube bench line + rocprof summary of the cube bench
cd "$GRAFT_REPO_ROOT" || exit 9
export TMPDIR=/tmp
mkdir -p gpurun_out/cubef
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/cubef/pytest_all.log 2>&1; rc=$?
tail -2 gpurun_out/cubef/pytest_all.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --workload cube --steps 3 --warmup 1 > gpurun_out/cubef/bench_cube.json 2> gpurun_out/cubef/bench_cube.err || { tail -3 gpurun_out/cubef/bench_cube.err; exit 1; }
tail -1 gpurun_out/cubef/bench_cube.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/cubef/prof -o cube -- python3 bench.py --workload cube --steps 3 --warmup 1 --cpu-baseline off > gpurun_out/cubef/prof.log 2>&1 || { tail -3 gpurun_out/cubef/prof.log; exit 1; }
grep -E "Name|k3_" gpurun_out/cubef/prof/cube_kernel_stats.csv
exit 0
