#!/bin/bash
# first GPU session: parity tests, smoke, small + full bench
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
rocm-smi --showproductname > gpurun_out/smi.txt 2>&1 || true
timeout -k 10 500 python -m pytest tests -m gpu -q -p no:cacheprovider --timeout 200 > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after pytest rc=$rc"; tail -30 gpurun_out/pytest_gpu.log; exit $rc; fi
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --n 10000000 --grid 2048 --steps 5 --warmup 2 --cpu-baseline off > gpurun_out/bench_small.log 2>&1
rc=$?; echo "bench small rc=$rc"
if [ $rc -ne 0 ]; then tail -20 gpurun_out/bench_small.log; exit $rc; fi
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --cpu-seconds 10 > gpurun_out/bench_full.log 2>&1
rc=$?; echo "bench full rc=$rc"
tail -3 gpurun_out/bench_full.log
exit 0
