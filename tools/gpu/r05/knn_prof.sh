#!/bin/bash
# k-NN kernel trace (10^7 Plummer, k = 32).
cd "$GRAFT_REPO_ROOT" || exit 9
export TMPDIR=/tmp
o=gpurun_out/r05/knn_prof; mkdir -p $o
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/kt -o kt -- python3 tools/prof_driver.py --workload knn --n 10000000 --iters 3 > $o/kt.log 2>&1 || { tail -20 $o/kt.log; exit 1; }
f=$(find $o/kt -name "*kernel_stats.csv" | head -1); cut -d, -f1-6 $f | head -30
