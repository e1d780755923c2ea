#!/bin/bash
# Wave-aggregated count increments: random order (headline) and cell order, vs ab_base.
cd "$GRAFT_REPO_ROOT" || exit 9
export OUT=r05/ab_countagg
bash tools/gpu/run.sh tests tests/test_gpu_parity.py || exit 1
for rep in 1 2; do
  bash tools/gpu/run.sh bench new_$rep --cpu-baseline off --overlap-streams 0 || exit 2
  ASP_LIB=$GRAFT_REPO_ROOT/astro-sph-tools_amd/ab_base/libasp_hip.so bash tools/gpu/run.sh bench base_$rep --cpu-baseline off --overlap-streams 0 || exit 3
done
bash tools/gpu/run.sh bench new_cell --cpu-baseline off --overlap-streams 0 --order cell || exit 4
ASP_LIB=$GRAFT_REPO_ROOT/astro-sph-tools_amd/ab_base/libasp_hip.so bash tools/gpu/run.sh bench base_cell --cpu-baseline off --overlap-streams 0 --order cell || exit 5
