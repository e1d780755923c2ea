#!/bin/bash
# PMC A/B of the scatter: pairs (default) vs single records (ASP_SCATTER_PAIRS=0), the
# headline workload, a few counters per pass (each pass its own rocprofv3 run).
cd "$GRAFT_REPO_ROOT" || exit 9
export TMPDIR=/tmp
o=gpurun_out/r03/pmc_ab
mkdir -p $o
run() {
  local tag=$1 name=$2; shift 2
  timeout -k 10 120 rocprofv3 "$@" --output-format csv -d $o/$tag/$name -o $name -- python3 tools/prof_driver.py --iters 3 > $o/$tag/$name.log 2>&1
  local rc=$?; echo "$tag $name rc=$rc"; return $rc
}
for tag in pairs single; do
  mkdir -p $o/$tag
  if [ $tag = single ]; then export ASP_SCATTER_PAIRS=0; else unset ASP_SCATTER_PAIRS; fi
  run $tag kt --kernel-trace --stats || exit 1
  run $tag pA --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY || exit 1
  run $tag pB --pmc SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM || exit 1
  run $tag pW --pmc WRITE_SIZE || exit 1
  run $tag pF --pmc FETCH_SIZE || exit 1
  python3 tools/pmc_summary.py $o/$tag > $o/$tag/summary.txt 2>&1
  grep -A14 "== k_scatter" $o/$tag/summary.txt | head -40
done
