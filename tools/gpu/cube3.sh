#!/bin/bash
# cube parity (both deposit paths forced), then the cube bench over lane/wave thresholds
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out/cube
for lc in 64 0; do
  ASP_CUBE_LANE_COLS=$lc timeout -k 10 300 python -u -m pytest tests/test_gpu_cube.py -x -q --timeout 120 --timeout-method thread > gpurun_out/cube/pytest_cube_$lc.log 2>&1; rc=$?
  echo "lane_cols=$lc: $(tail -1 gpurun_out/cube/pytest_cube_$lc.log)"; [ $rc -ne 0 ] && exit $rc
done
for lc in ${LCS:-64 16 36 128}; do
  ASP_CUBE_LANE_COLS=$lc timeout -k 10 300 python bench.py --workload cube --steps 3 --warmup 1 > gpurun_out/cube/bench_cube_$lc.json 2> gpurun_out/cube/bench_cube_$lc.err || { tail -3 gpurun_out/cube/bench_cube_$lc.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/cube/bench_cube_$lc.json').read().strip().splitlines()[-1]); print('lane_cols=$lc', d['ms_per_step'], {k: round(x['ms_per_launch'],3) for k,x in d.get('stages',{}).items()})"
done
exit 0
