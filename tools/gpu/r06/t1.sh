#!/bin/bash
# Round 6, first GPU call: the new tests (BASELINE-size parity, SPH weights, the cube axis
# beyond 32768), the LDS microbenchmark with the two-word fixed point, a bench line with
# the placement trials printed per slot.
cd "$GRAFT_REPO_ROOT" || exit 9
export OUT=r06/t1
o=gpurun_out/$OUT; mkdir -p $o
bash tools/gpu/run.sh tests tests/test_gpu_props.py tests/test_gpu_baseline_sizes.py tests/test_gpu_cube.py || exit 1
timeout -k 10 120 ./tools/mb_lds > $o/mb_lds.txt 2>&1 || exit 2
ASP_PRINT_ALLOC=1 bash tools/gpu/run.sh bench bench_alloc || exit 3
