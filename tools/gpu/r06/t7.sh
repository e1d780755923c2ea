#!/bin/bash
# Round 6 A/B: the scatter's stepped batch index (working build) against c0c0feb (ab_base),
# fresh processes alternating; bench timed region with the dominant kernel's events only.
cd "$GRAFT_REPO_ROOT" || exit 9
export OUT=r06/t7
for r in 1 2; do
  ASP_LIB=astro-sph-tools_amd/ab_base/libasp_hip.so bash tools/gpu/run.sh bench base_full_$r --steps 20 --cpu-baseline off --overlap-streams 0 || exit 1
  bash tools/gpu/run.sh bench new_full_$r --steps 20 --cpu-baseline off --overlap-streams 0 || exit 2
  ASP_LIB=astro-sph-tools_amd/ab_base/libasp_hip.so bash tools/gpu/run.sh bench base_shard_$r --n 12500000 --steps 50 --cpu-baseline off --overlap-streams 0 || exit 3
  bash tools/gpu/run.sh bench new_shard_$r --n 12500000 --steps 50 --cpu-baseline off --overlap-streams 0 || exit 4
done
