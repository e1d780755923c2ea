#!/bin/bash
# Kernel trace + SQ + HBM traffic passes for one workload:
#   bash tools/gpu/prof_full.sh <tag> [prof_driver args]
# Each PMC pass is its own rocprofv3 run (FETCH_SIZE and WRITE_SIZE cannot share one).
cd "$GRAFT_REPO_ROOT" || exit 9
export TMPDIR=/tmp
tag=$1; shift
out=gpurun_out/prof_$tag
mkdir -p $out
run() {
  local name=$1; shift
  timeout -k 10 240 rocprofv3 "$@" --output-format csv -d $out/$name -o $name -- python3 tools/prof_driver.py "${DRV[@]}" > $out/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc"; return $rc
}
DRV=("$@")
run kt --kernel-trace --stats || exit $?
DRV=("$@" --iters 2)
run pA --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY || exit $?
run pB --pmc SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM || exit $?
run pF --pmc FETCH_SIZE || exit $?
run pW --pmc WRITE_SIZE || exit $?
python3 tools/pmc_summary.py $out > $out/summary.txt 2>&1
grep -E "^== |avg_us|hbm_bytes|FETCH|WRITE_SIZE|LDS_BANK|ACTIVE_INST_LDS" $out/summary.txt | head -120
