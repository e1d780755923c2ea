#!/bin/bash
# Round 6: the N = 8 rank's share (1.25e7 particles -> 4096^2, weighted Wendland, pixel h):
# bench lines on one and two (gated) streams, a kernel trace of the one-stream line (the
# gaps between launches), and the Z-slab share beside the reduce stand-in (decomp_probe).
cd "$GRAFT_REPO_ROOT" || exit 9
export OUT=r06/t4 TMPDIR=/tmp
o=gpurun_out/$OUT; mkdir -p $o
bash tools/gpu/run.sh bench shard_1s --n 12500000 --steps 30 --cpu-baseline off --overlap-streams 0 || exit 1
ASP_SCATTER_GATE=1 bash tools/gpu/run.sh bench shard_2s --n 12500000 --steps 30 --cpu-baseline off --streams 2 --overlap-streams 0 || exit 2
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $o/kt_shard -o kt -- python3 bench.py --n 12500000 --steps 30 --cpu-baseline off --overlap-streams 0 > $o/kt_shard.json 2> $o/kt_shard.err || exit 3
timeout -k 10 300 python3 tools/decomp_probe.py --skip-decomp --interference --out $o/interference.json > $o/interference.log 2>&1 || exit 4
tail -5 $o/interference.log
