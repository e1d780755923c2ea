cd "$GRAFT_REPO_ROOT" || exit 9
for c in 0 4 9 16 30 64; do
  ASP_CUBE_LANE_COLS=$c timeout -k 10 200 python bench.py --workload cube --cpu-baseline off --steps 5 --warmup 2 2>/dev/null | python3 -c "import json,sys; d=json.load(sys.stdin); print('$c', d['ms_per_step'], round(d['stages']['cube_deposit']['ms_per_launch'],3))" || exit 1
done
