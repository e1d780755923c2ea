#!/bin/bash
# Same-box A/B of the headline map under library switches: one bench line per variant
# (gpurun_out/r03/ab/<name>.json), then the stage table.  Variants:
#   base     ASP_SCATTER_PAIRS=0 ASP_ITEM_ORDER=0 (round-2 scatter, Morton item order)
#   order    ASP_SCATTER_PAIRS=0 (largest items first)
#   pairs    the default build (64-B pair scatter + item order)
#   noconf   base with the conflict-free deposit ablation build (wrong maps: timing only)
cd "$GRAFT_REPO_ROOT" || exit 9
o=gpurun_out/r03/ab
mkdir -p $o
b() { local name=$1; shift; env "$@" timeout -k 10 200 python bench.py --cpu-baseline off > $o/$name.json 2> $o/$name.err; echo "$name rc=$?"; }
b base ASP_SCATTER_PAIRS=0 ASP_ITEM_ORDER=0
b order ASP_SCATTER_PAIRS=0
b pairs ASP_X=1
b noconf ASP_LIB=astro-sph-tools_amd/lib_abl/libasp_hip.so ASP_SCATTER_PAIRS=0 ASP_ITEM_ORDER=0
python tools/stages.py $o/base.json $o/order.json $o/pairs.json $o/noconf.json
