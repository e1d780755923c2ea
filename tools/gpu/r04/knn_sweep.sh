#!/bin/bash
# kNN 10^7: window half-width / verification-cell level sweep (ASP_KNN_WINDOW, ASP_KNN_FINE).
cd "$GRAFT_REPO_ROOT" || exit 9
export TMPDIR=/tmp
o=gpurun_out/r04/${TAG:-knn_sweep}
mkdir -p $o
for cfg in ${CFGS:-"128 1" "128 2" "64 1" "256 1" "64 2" "128 0"}; do
  set -- $cfg
  echo "== $(date +%T) W=$1 fine=$2"
  ASP_KNN_WINDOW=$1 ASP_KNN_FINE=$2 timeout -k 10 200 python bench.py --workload knn --n 10000000 --steps 3 --warmup 1 --cpu-baseline off > $o/knn_$1_$2.json 2> $o/knn_$1_$2.err || { tail -5 $o/knn_$1_$2.err; exit 1; }
  python -c "import json;d=json.load(open('$o/knn_$1_$2.json'));print('W $1 fine $2', d['ms_per_step'], d['output_ok'])"
done
