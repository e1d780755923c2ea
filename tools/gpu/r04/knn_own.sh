#!/bin/bash
# kNN: own cell first (ASP_KNN_OWN = level offset, -100 = off) -- parity tests, then a sweep.
cd "$GRAFT_REPO_ROOT" || exit 9
export TMPDIR=/tmp
o=gpurun_out/r04/knn_own
mkdir -p $o
echo "== $(date +%T) tests"
timeout -k 10 300 python -u -m pytest tests/test_gpu_knn.py -x -q --timeout 120 --timeout-method thread > $o/tests.log 2>&1 || { tail -20 $o/tests.log; exit 1; }
tail -2 $o/tests.log
for v in ${OWNS:--100 0 1 -1 -2 2}; do
  echo "== $(date +%T) own=$v"
  ASP_KNN_OWN=$v timeout -k 10 200 python bench.py --workload knn --n 10000000 --steps 3 --warmup 1 --cpu-baseline off > $o/knn_$v.json 2> $o/knn_$v.err || { tail -5 $o/knn_$v.err; exit 1; }
  python -c "import json;d=json.load(open('$o/knn_$v.json'));print('own $v', d['ms_per_step'], d['output_ok'])"
done
