#!/bin/bash
# Record-buffer placement trials: GPU tests, bench A/B (trials off / on), alloc probe.
cd "$GRAFT_REPO_ROOT" || exit 9
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/placement_tests.log 2>&1; rc=$?; tail -2 gpurun_out/placement_tests.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2 3; do
  ASP_PLACEMENT_TRIALS=0 timeout -k 10 200 python bench.py --cpu-baseline off --quiet | python3 -c "import json,sys; d=json.load(sys.stdin); print('trials0', d['ms_per_step'], round(d['stages']['scatter']['ms_per_launch'],3))" || exit 1
  ASP_PRINT_ALLOC=1 timeout -k 10 200 python bench.py --cpu-baseline off --quiet 2>gpurun_out/placement_alloc_$rep.log | python3 -c "import json,sys; d=json.load(sys.stdin); print('trials6', d['ms_per_step'], round(d['stages']['scatter']['ms_per_launch'],3))" || exit 1
  grep 'placement trial' gpurun_out/placement_alloc_$rep.log | tr '\n' ' '; echo
done
TRIALS=8 timeout -k 10 300 python -u tools/alloc_probe.py > gpurun_out/placement_probe.log 2>&1 || exit 1
grep trial gpurun_out/placement_probe.log
