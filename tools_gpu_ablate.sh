#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out/ablate
for v in "" 1 2 3; do
  lib=astro-sph-tools_amd/lib/libasp_hip${v:+_ablate$v}.so
  for det in "" "--deterministic"; do
    ASP_LIB=$PWD/$lib timeout -k 10 300 python bench.py --steps 5 --warmup 2 --cpu-baseline off --quiet $det > gpurun_out/ablate/v${v:-0}${det:+_det}.json 2>&1
    rc=$?
    echo "variant=${v:-0} $det rc=$rc $(python3 -c "import json,sys; d=json.load(open('gpurun_out/ablate/v${v:-0}${det:+_det}.json')); print('step', d['ms_per_step'], 'deposit', round(d['stages']['deposit']['ms_per_launch'],3), 'scatter', round(d['stages']['scatter']['ms_per_launch'],3))" 2>&1 | tail -1)"
    [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
