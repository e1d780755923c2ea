#!/bin/bash
# Same-box A/B of the scatter workgroup size (kBatch fixed at 1024 particles).
cd "$GRAFT_REPO_ROOT" || exit 9
export OUT=r05/${TAG:-ab_blk}
R=$GRAFT_REPO_ROOT/astro-sph-tools_amd
for rep in 1 2 3; do
  for lib in new blk256 blk1024; do
    l=""; [ $lib != new ] && l="ASP_LIB=$R/ab_$lib/libasp_hip.so"
    env $l bash tools/gpu/run.sh bench ${lib}_$rep --cpu-baseline off || exit 2
  done
done
