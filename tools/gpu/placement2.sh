#!/bin/bash
# Placement trials in the 2-D and 3-D scatters: GPU tests, then trials off / on A/B.
cd "$GRAFT_REPO_ROOT" || exit 9
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/placement_tests.log 2>&1; rc=$?; tail -2 gpurun_out/placement_tests.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
  for w in map cube; do
    a=(); [ $w = cube ] && a=(--workload cube)
    for t in 0 8; do
      ASP_PLACEMENT_TRIALS=$t ASP_PRINT_ALLOC=1 timeout -k 10 200 python bench.py --cpu-baseline off --quiet "${a[@]}" 2>gpurun_out/pl_$w$t.log | python3 -c "import json,sys; d=json.load(sys.stdin); print('$w trials$t', d['ms_per_step'], {k: round(v['ms_per_launch'],3) for k,v in d['stages'].items() if 'scatter' in k})" || exit 1
      grep 'placement trial' gpurun_out/pl_$w$t.log | sed 's/asp placement //' | tr '\n' ' '; echo
    done
  done
done
