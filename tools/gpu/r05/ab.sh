#!/bin/bash
# Same-box A/B: the working build vs astro-sph-tools_amd/ab_base (tools/ab_build.sh), fresh
# processes alternating, bench.py lines (ARGS) -- plus TESTS first if given.
cd "$GRAFT_REPO_ROOT" || exit 9
export OUT=r05/${TAG:-ab}
[ -n "$TESTS" ] && { bash tools/gpu/run.sh tests $TESTS || exit 1; }
for rep in $(seq 1 ${REPS:-3}); do
  bash tools/gpu/run.sh bench new_$rep --cpu-baseline off $ARGS || exit 2
  ASP_LIB=$GRAFT_REPO_ROOT/astro-sph-tools_amd/ab_base/libasp_hip.so bash tools/gpu/run.sh bench base_$rep --cpu-baseline off $ARGS || exit 3
done
