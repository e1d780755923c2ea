#!/bin/bash
# Same-box A/B of the headline map under library switches: one bench line per variant
# (gpurun_out/r03/ab/<name>.json), then the stage table.  $VARIANTS picks from:
#   base     ASP_ITEM_ORDER=0 (round-2 order: Morton items)
#   order    the default build (single-record scatter, largest items first)
#   pairs    ASP_SCATTER_PAIRS=1 (64-B pair scatter)
#   both     pairs + base
#   abl      the experiment build lib_abl/ (e.g. -DASP_ABLATE_DEP_CONFLICTS: timing only)
cd "$GRAFT_REPO_ROOT" || exit 9
o=gpurun_out/r03/ab
mkdir -p $o
b() { local name=$1; shift; env "$@" timeout -k 10 200 python bench.py --cpu-baseline off > $o/$name.json 2> $o/$name.err; echo "$name rc=$?"; }
files=(); i=0
for v in ${VARIANTS:-order pairs order}; do
  i=$((i+1)); n=${i}_$v
  case $v in
    base) b $n ASP_ITEM_ORDER=0 ;;
    order) b $n ASP_X=1 ;;
    pairs) b $n ASP_SCATTER_PAIRS=1 ;;
    both) b $n ASP_SCATTER_PAIRS=1 ASP_ITEM_ORDER=0 ;;
    abl) b $n ASP_LIB=astro-sph-tools_amd/lib_abl/libasp_hip.so ;;
  esac
  files+=($o/$n.json)
done
python tools/stages.py "${files[@]}"
