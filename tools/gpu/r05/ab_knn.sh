#!/bin/bash
# k-NN A/B on one box: the HEAD build (ab_base) against the working build, 10^7 Plummer,
# alternating twice, then the k-NN GPU tests (bit-exact against scipy) on the working build.
cd "$GRAFT_REPO_ROOT" || exit 9
export OUT=r05/${TAG:-ab_knn}
o=gpurun_out/$OUT; mkdir -p $o
for rep in 1 2; do
  ASP_LIB=$GRAFT_REPO_ROOT/astro-sph-tools_amd/ab_base/libasp_hip.so bash tools/gpu/run.sh bench base_$rep --workload knn --n 10000000 --cpu-baseline off || exit 3
  bash tools/gpu/run.sh bench new_$rep --workload knn --n 10000000 --cpu-baseline off || exit 4
done
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_knn.py > $o/knn_tests.log 2>&1; r=$?; tail -3 $o/knn_tests.log; exit $r
