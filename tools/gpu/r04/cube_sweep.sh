#!/bin/bash
# cube: lane-path threshold sweep (ASP_CUBE_LANE_COLS)
cd "$GRAFT_REPO_ROOT" || exit 9
export TMPDIR=/tmp
o=gpurun_out/r04/${TAG:-cube_sweep}
mkdir -p $o
for v in ${COLS:-30 20 48 64 96}; do
  echo "== $(date +%T) lane_cols=$v"
  ASP_CUBE_LANE_COLS=$v timeout -k 10 300 python bench.py --workload cube --steps 5 --cpu-baseline off > $o/cube_$v.json 2> $o/cube_$v.err || { tail -5 $o/cube_$v.err; exit 1; }
  python -c "import json;d=json.load(open('$o/cube_$v.json'));print('lane_cols $v', d['ms_per_step'], d.get('output_ok'), round(d['stages']['cube_deposit']['ms_per_launch'],3))"
done
