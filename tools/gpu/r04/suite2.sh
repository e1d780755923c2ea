#!/bin/bash
# Round-4 late evidence: the whole GPU suite on the final build, then the cube and k-NN lines
# and the rocprof kernel stats of the cube bench.
cd "$GRAFT_REPO_ROOT" || exit 9
export TMPDIR=/tmp
o=gpurun_out/r04/${TAG:-final2}; mkdir -p $o
echo "== $(date +%T) gpu suite"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/gputest.log 2>&1 || { tail -30 $o/gputest.log; exit 1; }
tail -2 $o/gputest.log
echo "== $(date +%T) lines"
timeout -k 10 300 python bench.py --workload cube > $o/bench_cube.json 2> $o/bench_cube.err || exit 2
timeout -k 10 300 python bench.py --workload knn --n 10000000 > $o/bench_knn_1e7.json 2> $o/bench_knn_1e7.err || exit 3
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/rp_cube -o cube -- python3 bench.py --workload cube --cpu-baseline off > $o/rp_cube.json 2> $o/rp_cube.err || exit 4
for f in bench_cube bench_knn_1e7 rp_cube; do
python3 -c "import json;d=json.loads(open('$o/$f.json').read().strip().splitlines()[-1]);print('$f', d['ms_per_step'], d.get('output_ok'), d.get('cpu_baseline',{}).get('value'))"
done
echo "== $(date +%T) done"
