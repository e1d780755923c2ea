#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 9
export TMPDIR=/tmp
out=gpurun_out/prof_band; mkdir -p $out
export ASP_BAND_COLS=64
for pass in "pA SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD" "pB SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT"; do
  set -- $pass; name=$1; shift
  timeout -k 10 400 rocprofv3 --pmc "$@" --output-format csv -d $out/$name -o $name -- python3 tools/prof_driver.py --h-law physical --iters 1 > $out/$name.log 2>&1 || { echo "$name failed"; tail -5 $out/$name.log; exit 1; }
done
python3 tools/pmc_summary.py $out > $out/summary.txt 2>&1; grep -A12 "k_band\|k_deposit" $out/summary.txt | head -80
