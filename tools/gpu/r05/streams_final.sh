#!/bin/bash
# The two-stream default: stream tests, two default bench lines, the rocprofv3 kernel trace
# of the bench command, and the two-rank bench path.
cd "$GRAFT_REPO_ROOT" || exit 9
export TMPDIR=/tmp
export OUT=r05/${TAG:-streams}
o=gpurun_out/$OUT; mkdir -p $o
bash tools/gpu/run.sh tests tests/test_gpu_streams.py tests/test_gpu_bench_multirank.py || exit 1
bash tools/gpu/run.sh bench bench_n1_a || exit 2
bash tools/gpu/run.sh bench bench_n1_b --cpu-baseline off || exit 3
echo "== $(date +%T) rocprof of the bench command"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/rp_bench -o bench -- python3 bench.py --cpu-baseline off > $o/rp_bench.json 2> $o/rp_bench.err || { tail -5 $o/rp_bench.err; exit 4; }
python3 -c "
import csv, json
for r in csv.DictReader(open('$o/rp_bench/bench_kernel_stats.csv')):
    if 'asp::' in r['Name']: print(r['Name'][:45], r['Calls'], round(float(r['AverageNs'])/1e3, 1), 'us')
d = json.loads(open('$o/rp_bench.json').read().strip().splitlines()[-1])
print('line', d['ms_per_step'], d['roofline']['kernel_ms_per_step'], d['roofline']['frac'], d['roofline']['pipeline_frac'])
"
bash tools/gpu/run.sh bench bench_shard --cpu-baseline off --n 12500000 --steps 30 || exit 5
