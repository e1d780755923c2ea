#!/bin/bash
# ASP_GATHER parity tests, full GPU suite, then cfg2 (physical / pixel h) and the headline
# map with and without the gathered large-record path.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out/ga
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k gathered > gpurun_out/ga/pytest_g.log 2>&1
rc=$?; tail -3 gpurun_out/ga/pytest_g.log; [ $rc -ne 0 ] && exit $rc
for g in 0 1; do
  for hl in physical pixel; do
    ASP_GATHER=$g timeout -k 10 200 python bench.py --n 10000000 --grid 2048 --map surface --kernel cubic --h-law $hl --steps 5 --warmup 2 --cpu-baseline off --quiet > gpurun_out/ga/c2_${hl}_$g.json 2> gpurun_out/ga/c2_${hl}_$g.err || exit $?
    python3 -c "import json; d=json.load(open('gpurun_out/ga/c2_${hl}_$g.json')); print('gather=$g cfg2 $hl', d['ms_per_step'], d['output_ok'], {k: round(v['ms_per_launch'],3) for k,v in d['stages'].items()})"
  done
  ASP_GATHER=$g timeout -k 10 200 python bench.py --h-law physical --steps 3 --warmup 1 --cpu-baseline off --quiet > gpurun_out/ga/c3phys_$g.json 2> gpurun_out/ga/c3phys_$g.err || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/ga/c3phys_$g.json')); print('gather=$g cfg3 physical', d['ms_per_step'], d['output_ok'], {k: round(v['ms_per_launch'],3) for k,v in d['stages'].items()})"
done
