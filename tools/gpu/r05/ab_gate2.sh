#!/bin/bash
# Streams / gate at the per-rank sizes of N = 1, 2, 4 (10^8, 5e7, 2.5e7 particles).
cd "$GRAFT_REPO_ROOT" || exit 9
export OUT=r05/${TAG:-ab_gate2}
for n in 100000000 50000000 25000000; do
  for rep in 1 2; do
    bash tools/gpu/run.sh bench n${n}_s1_$rep --cpu-baseline off --n $n --streams 1 || exit 2
    bash tools/gpu/run.sh bench n${n}_s2_$rep --cpu-baseline off --n $n --streams 2 || exit 3
    ASP_SCATTER_GATE=1 bash tools/gpu/run.sh bench n${n}_s2g_$rep --cpu-baseline off --n $n --streams 2 || exit 4
  done
done
