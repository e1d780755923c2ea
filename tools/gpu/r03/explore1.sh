#!/bin/bash
# Round-3 exploration: single-record vs pair scatter on the bench map (same box), then the
# pair-scatter and LDS-atomic microbenchmarks (uniform and Plummer-skewed tiles).
cd "$GRAFT_REPO_ROOT" || exit 9
export TMPDIR=/tmp
o=gpurun_out/r03/explore1
mkdir -p $o
VARIANTS="order pairs order pairs" bash tools/gpu/r03/ab_map.sh || exit 1
hipcc -O3 --offload-arch=gfx950 -o /tmp/mb_pairs tools/microbench/pairs.hip || exit 2
timeout -k 10 120 /tmp/mb_pairs > $o/mb_pairs.txt 2>&1; rc=$?; cat $o/mb_pairs.txt; [ $rc -eq 0 ] || exit $rc
hipcc -O3 --offload-arch=gfx950 -munsafe-fp-atomics -o /tmp/mb_lds tools/microbench/lds.hip || exit 3
timeout -k 10 120 /tmp/mb_lds > $o/mb_lds.txt 2>&1; rc=$?; cat $o/mb_lds.txt; exit $rc
