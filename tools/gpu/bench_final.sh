#!/bin/bash
# The default bench line (CPU baseline on) and the rocprof kernel stats of the same command.
cd "$GRAFT_REPO_ROOT" || exit 9
export TMPDIR=/tmp
o=gpurun_out/final; mkdir -p $o
timeout -k 10 300 python bench.py > $o/bench_n1.json 2> $o/bench_n1.err || { tail -5 $o/bench_n1.err; exit 1; }
cut -c1-300 $o/bench_n1.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/rp_bench -o bench -- python3 bench.py --cpu-baseline off > $o/rp_bench.json 2> $o/rp_bench.err || exit 1
cut -c1-200 $o/rp_bench.json
