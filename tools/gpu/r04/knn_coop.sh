#!/bin/bash
# kNN: the wave-union cell pass (ASP_KNN_COOP = max cells, 0 = per-lane cells) -- parity
# tests first, then a sweep of the 10^7 bench.
cd "$GRAFT_REPO_ROOT" || exit 9
export TMPDIR=/tmp
o=gpurun_out/r04/knn_coop
mkdir -p $o
echo "== $(date +%T) tests"
ASP_KNN_COOP=${TEST_COOP:-4096} timeout -k 10 300 python -u -m pytest tests/test_gpu_knn.py -x -q --timeout 120 --timeout-method thread > $o/tests.log 2>&1 || { tail -20 $o/tests.log; exit 1; }
tail -2 $o/tests.log
for cfg in ${CFGS:-"0 1" "64 1" "512 1" "4096 1" "512 2" "4096 2"}; do
  set -- $cfg
  echo "== $(date +%T) coop=$1 fine=$2"
  ASP_KNN_COOP=$1 ASP_KNN_COOP_FINE=$2 timeout -k 10 200 python bench.py --workload knn --n 10000000 --steps 3 --warmup 1 --cpu-baseline off > $o/knn_$1_$2.json 2> $o/knn_$1_$2.err || { tail -5 $o/knn_$1_$2.err; exit 1; }
  python -c "import json;d=json.load(open('$o/knn_$1_$2.json'));print('coop $1 fine $2', d['ms_per_step'], d['output_ok'])"
done
