#!/bin/bash
# kNN: parity tests, then the 10^7 bench (and the 10^8 one with BIG=1).
cd "$GRAFT_REPO_ROOT" || exit 9
export TMPDIR=/tmp
o=gpurun_out/r04/${TAG:-knn_run}
mkdir -p $o
echo "== $(date +%T) tests"
timeout -k 10 300 python -u -m pytest tests/test_gpu_knn.py -x -q --timeout 120 --timeout-method thread > $o/tests.log 2>&1 || { tail -20 $o/tests.log; exit 1; }
tail -2 $o/tests.log
for rep in 1 2; do
  echo "== $(date +%T) bench $rep"
  timeout -k 10 200 python bench.py --workload knn --n 10000000 --steps 3 --warmup 1 --cpu-baseline off > $o/knn_$rep.json 2> $o/knn_$rep.err || { tail -5 $o/knn_$rep.err; exit 1; }
  python -c "import json;d=json.load(open('$o/knn_$rep.json'));print('knn 1e7', d['ms_per_step'], d['output_ok'])"
done
if [ -n "$BIG" ]; then
  timeout -k 10 300 python bench.py --workload knn --n 100000000 --steps 2 --warmup 1 --cpu-baseline off > $o/knn_1e8.json 2> $o/knn_1e8.err || { tail -5 $o/knn_1e8.err; exit 1; }
  python -c "import json;d=json.load(open('$o/knn_1e8.json'));print('knn 1e8', d['ms_per_step'], d['output_ok'])"
fi
