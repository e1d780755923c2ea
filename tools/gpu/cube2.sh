#!/bin/bash
# cube parity, then the cube bench (BASELINE configs[4] on one GPU)
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out/cube
timeout -k 10 300 python -u -m pytest tests/test_gpu_cube.py -x -q --timeout 120 --timeout-method thread > gpurun_out/cube/pytest_cube.log 2>&1; rc=$?
tail -4 gpurun_out/cube/pytest_cube.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --workload cube --steps 3 --warmup 1 "$@" > gpurun_out/cube/bench_cube.json 2> gpurun_out/cube/bench_cube.err; rc=$?
python3 -c "import json; d=json.loads(open('gpurun_out/cube/bench_cube.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], {k: round(x['ms_per_launch'],3) for k,x in d.get('stages',{}).items()})"
exit $rc
