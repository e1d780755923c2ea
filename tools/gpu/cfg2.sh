#!/bin/bash
# BASELINE configs[1]: 10^7 particles -> 2048^2 surface density, cubic spline, both h laws.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out/cfg2
for hl in physical pixel; do
  timeout -k 10 300 python bench.py --n 10000000 --grid 2048 --map surface --kernel cubic --h-law $hl --steps 10 --warmup 3 > gpurun_out/cfg2/$hl.json 2> gpurun_out/cfg2/$hl.err || exit $?
  cut -c1-400 gpurun_out/cfg2/$hl.json
done
