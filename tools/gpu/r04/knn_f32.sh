#!/bin/bash
# k-NN: fp32 window prefilter (ASP_KNN_F32=1, default) vs fp64 window (0), same box; parity first
cd "$GRAFT_REPO_ROOT" || exit 9
export TMPDIR=/tmp
o=gpurun_out/r04/knn_f32; mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_gpu_knn.py -x -q --timeout 120 --timeout-method thread > $o/tests.log 2>&1 || { tail -20 $o/tests.log; exit 1; }
tail -1 $o/tests.log
for rep in 1 2; do for v in 1 0; do
  ASP_KNN_F32=$v timeout -k 10 200 python bench.py --workload knn --n 10000000 --steps 3 --warmup 1 --cpu-baseline off > $o/knn_${v}_$rep.json 2> $o/knn_${v}_$rep.err || { tail -5 $o/knn_${v}_$rep.err; exit 1; }
  python -c "import json;d=json.load(open('$o/knn_${v}_$rep.json'));print('f32 $v', d['ms_per_step'], d['output_ok'])"
done; done
ASP_KNN_DIAG=1 timeout -k 10 200 python bench.py --workload knn --n 10000000 --steps 3 --warmup 1 --cpu-baseline off > $o/knn_window_only.json 2> /dev/null; python -c "import json;d=json.load(open('$o/knn_window_only.json'));print('window only (f32)', d['ms_per_step'])"
