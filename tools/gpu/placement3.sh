#!/bin/bash
# How often the placement trials find the fast record buffer: fresh processes, trials on.
cd "$GRAFT_REPO_ROOT" || exit 9
export TMPDIR=/tmp
for rep in 1 2 3 4 5 6; do
  ASP_PRINT_ALLOC=1 timeout -k 10 200 python bench.py --cpu-baseline off --quiet 2>gpurun_out/pl3_$rep.log | python3 -c "import json,sys; d=json.load(sys.stdin); print('rep $rep', d['ms_per_step'], round(d['stages']['scatter']['ms_per_launch'],3))" || exit 1
  grep -c 'placement trial' gpurun_out/pl3_$rep.log
done
