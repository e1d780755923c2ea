#!/bin/bash
# Round 6: the N = 8 share (1.25e7 -> 4096^2): count-block sweep at 256 scatter workgroups
# (ASP_BIN_BLOCKS / ASP_SCATTER_GROUP), two streams gated / ungated, the Z-slab share beside
# the reduce stand-in, and the two-rank bench path (gloo) test.
cd "$GRAFT_REPO_ROOT" || exit 9
export OUT=r06/t8
S="--n 12500000 --steps 50 --cpu-baseline off --overlap-streams 0"
for r in 1 2; do
  bash tools/gpu/run.sh bench nb1024_$r $S || exit 1
  ASP_BIN_BLOCKS=512 ASP_SCATTER_GROUP=2 bash tools/gpu/run.sh bench nb512_$r $S || exit 2
  ASP_BIN_BLOCKS=256 ASP_SCATTER_GROUP=1 bash tools/gpu/run.sh bench nb256_$r $S || exit 3
done
ASP_SCATTER_GATE=1 bash tools/gpu/run.sh bench s2_gate $S --streams 2 || exit 4
ASP_SCATTER_GATE=0 bash tools/gpu/run.sh bench s2_nogate $S --streams 2 || exit 5
timeout -k 10 300 python3 tools/decomp_probe.py --skip-decomp --interference --out gpurun_out/$OUT/interference.json > gpurun_out/$OUT/interference.log 2>&1 || exit 6
tail -4 gpurun_out/$OUT/interference.log
bash tools/gpu/run.sh tests tests/test_gpu_bench_multirank.py || exit 7
