#!/bin/bash
# PMC A/B of one kernel under library switches, the headline workload (prof_driver), a few
# counters per pass (each pass its own rocprofv3 run).  $VARIANTS: "name:VAR=x,VAR2=y ..."
# (default: single-record vs pair scatter); $KERN: the summary section to print.
cd "$GRAFT_REPO_ROOT" || exit 9
export TMPDIR=/tmp
o=gpurun_out/r03/pmc_ab
mkdir -p $o
run() {
  local tag=$1 name=$2; shift 2
  timeout -k 10 120 rocprofv3 "$@" --output-format csv -d $o/$tag/$name -o $name -- python3 tools/prof_driver.py --iters 3 > $o/$tag/$name.log 2>&1
  local rc=$?; echo "$tag $name rc=$rc"; return $rc
}
for v in ${VARIANTS:-single:ASP_X=1 pairs:ASP_SCATTER_PAIRS=1}; do
  tag=${v%%:*}; envs=${v#*:}
  mkdir -p $o/$tag
  (
    for kv in ${envs//,/ }; do export "$kv"; done
    run $tag kt --kernel-trace --stats || exit 1
    run $tag pA --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY || exit 1
    run $tag pB --pmc SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM || exit 1
    run $tag pW --pmc WRITE_SIZE || exit 1
    run $tag pF --pmc FETCH_SIZE || exit 1
  ) || exit 1
  python3 tools/pmc_summary.py $o/$tag > $o/$tag/summary.txt 2>&1
  grep -A22 "== ${KERN:-k_scatter}" $o/$tag/summary.txt | head -50
done
