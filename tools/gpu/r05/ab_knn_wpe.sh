#!/bin/bash
# k-NN search compiled for 4 waves per SIMD (ab_w4: -DASP_KNN_WPE=4, 128 registers, spills)
# against the default build (157 VGPRs, 3 waves), 10^7 Plummer, alternating twice; the
# k-NN GPU tests (bit-exact against scipy) on the ab_w4 build.
cd "$GRAFT_REPO_ROOT" || exit 9
export OUT=r05/${TAG:-ab_knn_wpe}
o=gpurun_out/$OUT; mkdir -p $o
W=$GRAFT_REPO_ROOT/astro-sph-tools_amd/ab_w4/libasp_hip.so
for rep in 1 2; do
  bash tools/gpu/run.sh bench base_$rep --workload knn --n 10000000 --cpu-baseline off || exit 3
  ASP_LIB=$W bash tools/gpu/run.sh bench w4_$rep --workload knn --n 10000000 --cpu-baseline off || exit 4
done
ASP_LIB=$W timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_knn.py > $o/knn_tests_w4.log 2>&1; r=$?; tail -3 $o/knn_tests_w4.log; exit $r
