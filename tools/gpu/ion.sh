#!/bin/bash
# ion-mass workload: bench line + rocprof kernel stats
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out/ion
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --workload ion --steps 10 --warmup 3 > gpurun_out/ion/bench_ion.json 2> gpurun_out/ion/bench_ion.err || { tail -5 gpurun_out/ion/bench_ion.err; exit 1; }
cat gpurun_out/ion/bench_ion.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ion/prof -o ion -- python3 bench.py --workload ion --steps 10 --warmup 3 --cpu-baseline off > gpurun_out/ion/prof.log 2>&1 || { tail -5 gpurun_out/ion/prof.log; exit 1; }
find gpurun_out/ion/prof -name '*kernel_stats.csv' -exec cat {} \;
exit 0
