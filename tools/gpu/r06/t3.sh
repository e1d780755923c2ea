#!/bin/bash
# Round 6: PMC of the single-pass binning experiment's scatter (ASP_SP_EXPERIMENT=1; the
# two-pass scatter's PMC of the same code is profiles/r05/final/pmc_cfg3_summary_r05.txt).
cd "$GRAFT_REPO_ROOT" || exit 9
export TMPDIR=/tmp
ASP_SP_EXPERIMENT=1 bash tools/gpu/prof_full.sh r06_sp --iters 3 || exit 1
