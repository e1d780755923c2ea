#!/bin/bash
# Three map slots / streams vs two (headline), same box.
cd "$GRAFT_REPO_ROOT" || exit 9
export OUT=r05/${TAG:-ab_slots}
R=$GRAFT_REPO_ROOT/astro-sph-tools_amd
for rep in 1 2; do
  bash tools/gpu/run.sh bench s2_$rep --cpu-baseline off --streams 2 || exit 2
  ASP_LIB=$R/ab_slots3/libasp_hip.so bash tools/gpu/run.sh bench s3_$rep --cpu-baseline off --streams 3 || exit 3
  ASP_LIB=$R/ab_slots3/libasp_hip.so bash tools/gpu/run.sh bench s3n5_$rep --cpu-baseline off --streams 3 --n 50000000 || exit 4
  bash tools/gpu/run.sh bench s2n5_$rep --cpu-baseline off --streams 2 --n 50000000 || exit 5
done
