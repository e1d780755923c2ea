#!/bin/bash
# Global -fno-slp-vectorize (ab_noslp) vs the working library: headline, cfg2 physical, k-NN.
cd "$GRAFT_REPO_ROOT" || exit 9
export OUT=r05/ab_noslp
for rep in 1 2; do
  for v in "" noslp; do
    if [ -n "$v" ]; then export ASP_LIB=astro-sph-tools_amd/ab_$v/libasp_hip.so; else unset ASP_LIB; fi
    bash tools/gpu/run.sh bench cfg3_${v:-work}_$rep --cpu-baseline off --overlap-streams 0 || exit 1
    bash tools/gpu/run.sh bench cfg2p_${v:-work}_$rep --n 10000000 --grid 2048 --kernel cubic --h-law physical --map surface --cpu-baseline off --overlap-streams 0 || exit 2
  done
done
