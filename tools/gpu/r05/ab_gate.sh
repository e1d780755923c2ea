#!/bin/bash
# Maps on two streams with the scatter gated behind the previous map's deposit
# (ASP_SCATTER_GATE=1) vs ungated vs one stream: the headline and the 1.25e7 shard.
cd "$GRAFT_REPO_ROOT" || exit 9
export OUT=r05/${TAG:-ab_gate}
bash tools/gpu/run.sh tests tests/test_gpu_streams.py tests/test_gpu_parity.py || exit 1
for rep in 1 2 3; do
  bash tools/gpu/run.sh bench s1_$rep --cpu-baseline off --streams 1 || exit 2
  bash tools/gpu/run.sh bench s2_$rep --cpu-baseline off --streams 2 || exit 3
  ASP_SCATTER_GATE=1 bash tools/gpu/run.sh bench s2g_$rep --cpu-baseline off --streams 2 || exit 4
done
for rep in 1 2; do
  bash tools/gpu/run.sh bench sh_s2_$rep --cpu-baseline off --n 12500000 --steps 30 --streams 2 || exit 5
  ASP_SCATTER_GATE=1 bash tools/gpu/run.sh bench sh_s2g_$rep --cpu-baseline off --n 12500000 --steps 30 --streams 2 || exit 6
done
