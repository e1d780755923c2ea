#!/bin/bash
# k-NN tuning sweep: window half-width x verification cell refinement, 1e7 Plummer.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out/knn
for w in ${WS:-128 256 512}; do for f in ${FS:-0 1}; do
  ASP_KNN_WINDOW=$w ASP_KNN_FINE=$f timeout -k 10 200 python bench.py --workload knn --n 10000000 --steps 2 --warmup 1 --cpu-baseline off > gpurun_out/knn/w${w}_f$f.json 2> gpurun_out/knn/w${w}_f$f.err || { echo "w=$w f=$f failed"; tail -3 gpurun_out/knn/w${w}_f$f.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/knn/w${w}_f$f.json')); print('W=$w fine=$f', d['ms_per_step'], 'ms')"
done; done
