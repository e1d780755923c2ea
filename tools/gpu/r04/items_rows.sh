#!/bin/bash
# deposit items per map (ASP_ITEMS) on the row shares and the full map
cd "$GRAFT_REPO_ROOT" || exit 9
export TMPDIR=/tmp
o=gpurun_out/r04/items_rows; mkdir -p $o
for it in ${ITEMS:-1024 512 768 2048}; do
  echo "== $(date +%T) items=$it"
  ASP_ITEMS=$it timeout -k 10 400 python tools/decomp_probe.py --stages --out $o/items_$it.json > $o/items_$it.log 2>&1 || { tail -5 $o/items_$it.log; exit 1; }
  grep -E "full map|rows, two|rows max" $o/items_$it.log
done
