#!/bin/bash
# Occupancy / issue counters for one workload: bash tools/gpu/prof3.sh <tag> [prof_driver args]
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
run pA --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY || exit $?
run pC --pmc SQ_LEVEL_WAVES SQ_ACTIVE_INST_VALU2 SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU_TRANS_F32 SQ_IFETCH SQ_INSTS_BRANCH SQ_BUSY_CU_CYCLES SQ_INST_CYCLES_SALU GRBM_GUI_ACTIVE || exit $?
python3 tools/pmc_summary.py $out > $out/summary.txt 2>&1
grep -A30 "== k_gather\|== k_deposit" $out/summary.txt | head -80
