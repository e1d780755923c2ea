#!/bin/bash
# Round 5: full GPU suite + smoke, the headline line (CPU baseline on), the k-NN line, the
# two-rank bench rehearsals, and (PMC=1) the headline's PMC passes.
cd "$GRAFT_REPO_ROOT" || exit 9
export OUT=r05/${TAG:-suite}
bash tools/gpu/run.sh suite || exit 1
bash tools/gpu/run.sh bench bench_n1 || exit 2
bash tools/gpu/run.sh bench bench_knn_1e7 --workload knn --n 10000000 || exit 3
if [ -n "$PMC" ]; then bash tools/gpu/r05/wc_pmc.sh || exit 5; fi
echo "== $(date +%T) done"
