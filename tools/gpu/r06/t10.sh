#!/bin/bash
# Round 6 A/B: the scatter with two batches of loads in flight (ASP_SCATTER_PREFETCH=2),
# and the same with 1024-thread scatter workgroups, against the production build.
cd "$GRAFT_REPO_ROOT" || exit 9
export OUT=r06/t10
for r in 1 2; do
  for v in prod pf2 pf2b1024; do
    lib=astro-sph-tools_amd/lib/libasp_hip.so; [ $v != prod ] && lib=astro-sph-tools_amd/ab_$v/libasp_hip.so
    ASP_LIB=$lib bash tools/gpu/run.sh bench ${v}_$r --steps 20 --cpu-baseline off --overlap-streams 0 || exit 1
  done
done
