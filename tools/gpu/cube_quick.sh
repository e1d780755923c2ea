# Cube: GPU tests + the 512^3 bench at two lane-path thresholds.
cd "$GRAFT_REPO_ROOT" || exit 9
timeout -k 10 200 python -u -m pytest tests/test_gpu_cube.py -x -q --timeout 150 --timeout-method thread 2>&1 | tail -2 || exit 1
for c in ${CUBE_COLS:-30 40}; do
  ASP_CUBE_LANE_COLS=$c timeout -k 10 200 python bench.py --workload cube --cpu-baseline off --steps 5 --warmup 2 2>/dev/null | python3 -c "import json,sys; d=json.load(sys.stdin); print('$c', d['ms_per_step'], round(d['stages']['cube_deposit']['ms_per_launch'],3))" || exit 1
done
