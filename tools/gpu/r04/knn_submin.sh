#!/bin/bash
# k-NN 10^7: sub-table threshold sweep (ASP_KNN_SUBMIN)
cd "$GRAFT_REPO_ROOT" || exit 9
export TMPDIR=/tmp
o=gpurun_out/r04/knn_submin; mkdir -p $o
for v in ${VALS:-64 16 32 128 256 64}; do
  ASP_KNN_SUBMIN=$v timeout -k 10 200 python bench.py --workload knn --n 10000000 --steps 3 --warmup 1 --cpu-baseline off > $o/knn_$v.json 2> $o/knn_$v.err || { tail -5 $o/knn_$v.err; exit 1; }
  python -c "import json;d=json.load(open('$o/knn_$v.json'));print('submin $v', d['ms_per_step'], d['output_ok'])"
done
