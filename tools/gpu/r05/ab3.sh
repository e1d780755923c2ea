#!/bin/bash
# Same-box A/B of small maps: working build vs ab_base (before the scatter load change) vs
# ab_r4 (the round-4 library): cfg2 pixel and the 1.25e7 shard, fresh processes.
cd "$GRAFT_REPO_ROOT" || exit 9
export OUT=r05/${TAG:-ab3}
R=$GRAFT_REPO_ROOT/astro-sph-tools_amd
for rep in 1 2; do
  for lib in new base r4; do
    l=""; [ $lib != new ] && l="ASP_LIB=$R/ab_$lib/libasp_hip.so"
    env $l bash tools/gpu/run.sh bench cfg2p_${lib}_$rep --cpu-baseline off --n 10000000 --grid 2048 --kernel cubic --map surface || exit 2
    env $l bash tools/gpu/run.sh bench shard_${lib}_$rep --cpu-baseline off --n 12500000 --steps 30 || exit 3
  done
done
