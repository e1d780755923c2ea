#!/bin/bash
# Kernel trace + SQ passes over an arbitrary python command line:
#   bash tools/gpu/prof_cmd.sh <tag> <script.py> [args]
cd "$GRAFT_REPO_ROOT" || exit 9
export TMPDIR=/tmp
tag=$1; shift
out=gpurun_out/prof_$tag
mkdir -p $out
run() {
  local name=$1; shift
  timeout -k 10 300 rocprofv3 "$@" --output-format csv -d $out/$name -o $name -- python3 "${CMD[@]}" > $out/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc"; return $rc
}
CMD=("$@")
run kt --kernel-trace --stats || exit $?
run pA --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY || exit $?
run pB --pmc SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_TRANS_F32 SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU_FMA_F64 || exit $?
python3 tools/pmc_summary.py $out > $out/summary.txt 2>&1
grep -E "^== |avg_us|calls|SQ_" $out/summary.txt | head -80
