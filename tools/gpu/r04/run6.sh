#!/bin/bash
# Round-4: decomposition probe with two-stream row shares; the default bench line with the
# CPU baseline (stratified cost model); the deterministic line.
cd "$GRAFT_REPO_ROOT" || exit 9
export TMPDIR=/tmp
o=gpurun_out/r04/${TAG:-run6}
mkdir -p $o
echo "== $(date +%T) decomposition probe"
timeout -k 10 300 python tools/decomp_probe.py --out $o/decomp.json > $o/decomp.log 2>&1 || { tail -5 $o/decomp.log; exit 1; }
tail -5 $o/decomp.log
echo "== $(date +%T) bench with CPU baseline"
timeout -k 10 600 python bench.py > $o/bench_full.json 2> $o/bench_full.err || { tail -5 $o/bench_full.err; exit 1; }
python -c "import json;d=json.load(open('$o/bench_full.json'));print(d['ms_per_step'], d['value'], json.dumps(d['cpu_baseline']))"
TAG=${TAG:-run6} BENCHES="det1" bash tools/gpu/r04/iter.sh
echo "== $(date +%T) done"
