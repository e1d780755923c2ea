#!/bin/bash
# Round-4 PMC of the secondary kernels: the 512^3 cube (10^8 particles, physical h) and the
# k-NN search (10^7), each pass its own rocprofv3 run (tools/gpu/prof_full.sh).
cd "$GRAFT_REPO_ROOT" || exit 9
export TMPDIR=/tmp
bash tools/gpu/prof_full.sh r04cube --workload cube --iters 3 || exit 1
bash tools/gpu/prof_full.sh r04knn --workload knn --n 10000000 --iters 3 || exit 2
grep -E "^== |avg_us|SQ_INSTS_VALU|SQ_ACTIVE_INST_VALU|SQ_WAIT_INST_LDS|SQ_LDS_BANK|SQ_WAVE_CYCLES|hbm_bytes" gpurun_out/prof_r04cube/summary.txt gpurun_out/prof_r04knn/summary.txt | head -80
