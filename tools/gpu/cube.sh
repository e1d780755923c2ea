#!/bin/bash
# cube parity + a first cube bench + the 2-D suite after the host-runtime split
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out/cube
timeout -k 10 300 python -m pytest tests/test_gpu_cube.py -x -q > gpurun_out/cube/pytest_cube.log 2>&1; rc=$?
tail -5 gpurun_out/cube/pytest_cube.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -m pytest tests -m gpu -x -q > gpurun_out/cube/pytest_all.log 2>&1; rc=$?
tail -3 gpurun_out/cube/pytest_all.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --workload cube --steps 3 --warmup 1 > gpurun_out/cube/bench_cube.json 2> gpurun_out/cube/bench_cube.err; rc=$?
cat gpurun_out/cube/bench_cube.json; exit $rc
