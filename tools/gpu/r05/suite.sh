#!/bin/bash
# Round 5: full GPU suite, smoke, k-NN line, headline line; then the write-combining PMC A/B.
cd "$GRAFT_REPO_ROOT" || exit 9
export TMPDIR=/tmp
o=gpurun_out/r05/${TAG:-suite}; mkdir -p $o
echo "== $(date +%T) gpu suite"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/gputest.log 2>&1 || { tail -40 $o/gputest.log; exit 1; }
tail -1 $o/gputest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || { tail -5 $o/smoke.log; exit 2; }
tail -1 $o/smoke.log
echo "== $(date +%T) knn"
timeout -k 10 300 python bench.py --workload knn --n 10000000 > $o/bench_knn_1e7.json 2> $o/bench_knn_1e7.err || { tail -5 $o/bench_knn_1e7.err; exit 3; }
echo "== $(date +%T) bench"
timeout -k 10 300 python bench.py --cpu-baseline off > $o/bench_n1.json 2> $o/bench_n1.err || { tail -5 $o/bench_n1.err; exit 4; }
for f in bench_knn_1e7 bench_n1; do
python3 -c "import json;d=json.loads(open('$o/$f.json').read().strip().splitlines()[-1]);print('$f', d['ms_per_step'], d.get('output_ok'), d.get('roofline'), {k:round(v.get('ms_per_step', v.get('ms_per_launch')),3) for k,v in d.get('stages',{}).items()})"
done
echo "== $(date +%T) pmc"
[ -n "$PMC" ] && { bash tools/gpu/r05/wc_pmc.sh || exit 5; }
echo "== $(date +%T) done"
