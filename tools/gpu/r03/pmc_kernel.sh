#!/bin/bash
# PMC passes of one workload (tools/prof_driver.py $DRIVER_ARGS), each pass its own rocprofv3
# run; summary of kernel $KERN.  Output: gpurun_out/r03/$TAG/
cd "$GRAFT_REPO_ROOT" || exit 9
export TMPDIR=/tmp
o=gpurun_out/r03/${TAG:-pmc}
mkdir -p $o
run() {
  local name=$1; shift
  timeout -k 10 150 rocprofv3 "$@" --output-format csv -d $o/$name -o $name -- python3 tools/prof_driver.py --iters 3 $DRIVER_ARGS > $o/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc"; return $rc
}
run kt --kernel-trace --stats || exit 1
run pA --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY || exit 1
run pB --pmc SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM || exit 1
run pC --pmc SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 || exit 1
python3 tools/pmc_summary.py $o > $o/summary.txt 2>&1
grep -A30 "== ${KERN:-k_gather}" $o/summary.txt | head -45
