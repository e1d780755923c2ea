#!/bin/bash
# kNN time split: ASP_KNN_DIAG 0 (full), 1 (window only), 2 (+ cell walk and lookups), 3 (+ cell walk only)
cd "$GRAFT_REPO_ROOT" || exit 9
export TMPDIR=/tmp
o=gpurun_out/r04/knn_diag
mkdir -p $o
for v in 0 1 2 3; do
  echo "== $(date +%T) diag=$v"
  ASP_KNN_DIAG=$v timeout -k 10 200 python bench.py --workload knn --n 10000000 --steps 3 --warmup 1 --cpu-baseline off > $o/knn_$v.json 2> $o/knn_$v.err || [ $? -eq 3 ] || { tail -5 $o/knn_$v.err; exit 1; }
  python -c "import json;d=json.load(open('$o/knn_$v.json'));print('diag $v', d['ms_per_step'], d['output_ok'])"
done
