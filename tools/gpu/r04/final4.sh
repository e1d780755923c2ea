#!/bin/bash
# Round-4 closing evidence on the final build: GPU suite, smoke, the default bench line,
# rocprof kernel stats of the same command, and the other workloads' lines.
cd "$GRAFT_REPO_ROOT" || exit 9
export TMPDIR=/tmp
o=gpurun_out/r04/final4; mkdir -p $o
echo "== $(date +%T) gpu suite"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/gputest.log 2>&1 || { tail -30 $o/gputest.log; exit 1; }
tail -1 $o/gputest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || { tail -5 $o/smoke.log; exit 2; }
tail -1 $o/smoke.log
echo "== $(date +%T) bench line"
timeout -k 10 600 python bench.py > $o/bench_n1.json 2> $o/bench_n1.err || { tail -5 $o/bench_n1.err; exit 3; }
echo "== $(date +%T) rocprof of the bench command"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/rp_bench -o bench -- python3 bench.py --cpu-baseline off > $o/rp_bench.json 2> $o/rp_bench.err || exit 4
echo "== $(date +%T) other lines"
timeout -k 10 300 python bench.py --cpu-baseline off --n 10000000 --grid 2048 --kernel cubic --map surface --h-law physical > $o/bench_cfg2_physical.json 2> $o/bench_cfg2_physical.err || exit 5
timeout -k 10 300 python bench.py --cpu-baseline off --n 10000000 --grid 2048 --kernel cubic --map surface > $o/bench_cfg2_pixel.json 2> $o/bench_cfg2_pixel.err || exit 6
timeout -k 10 300 python bench.py --workload cube > $o/bench_cube.json 2> $o/bench_cube.err || exit 7
timeout -k 10 300 python bench.py --workload knn --n 10000000 > $o/bench_knn_1e7.json 2> $o/bench_knn_1e7.err || exit 8
timeout -k 10 300 python bench.py --workload knn --n 100000000 --steps 2 --warmup 1 --cpu-baseline off > $o/bench_knn_1e8.json 2> $o/bench_knn_1e8.err || exit 9
timeout -k 10 300 python bench.py --n 12500000 --steps 30 --cpu-baseline off > $o/bench_shard.json 2> $o/bench_shard.err || exit 10
for f in bench_n1 rp_bench bench_cfg2_physical bench_cfg2_pixel bench_cube bench_knn_1e7 bench_knn_1e8 bench_shard; do
python3 -c "import json;d=json.loads(open('$o/$f.json').read().strip().splitlines()[-1]);print('$f', d['ms_per_step'], d.get('output_ok'), d.get('roofline',{}).get('kernel'), d.get('roofline',{}).get('frac'), (d.get('cpu_baseline') or {}).get('value'))"
done
echo "== $(date +%T) done"
