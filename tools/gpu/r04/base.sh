#!/bin/bash
# Round-4 checkpoint: GPU suite, the default bench line, the same with no stage events
# (event overhead), the N = 8 shard size, and a rocprofv3 kernel-trace of the bench command.
cd "$GRAFT_REPO_ROOT" || exit 9
export TMPDIR=/tmp
o=gpurun_out/r04/${TAG:-base}
mkdir -p $o
step() { echo "== $(date +%T) $*"; }
if [ -z "$NOTEST" ]; then
step pytest
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf > $o/gputest.log 2>&1; rc=$?; tail -15 $o/gputest.log
[ $rc -le 1 ] || exit $rc
fi
step bench
timeout -k 10 300 python bench.py --cpu-baseline off > $o/bench_n1.json 2> $o/bench_n1.err || { tail -5 $o/bench_n1.err; exit 1; }
cut -c1-900 $o/bench_n1.json
step bench one stream
timeout -k 10 300 python bench.py --cpu-baseline off --streams 1 > $o/bench_s1.json 2> $o/bench_s1.err || { tail -5 $o/bench_s1.err; exit 1; }
cut -c1-400 $o/bench_s1.json
step bench no events
timeout -k 10 300 python bench.py --cpu-baseline off --no-stage-events > $o/bench_noev.json 2> $o/bench_noev.err || { tail -5 $o/bench_noev.err; exit 1; }
cut -c1-300 $o/bench_noev.json
step bench deterministic
timeout -k 10 300 python bench.py --cpu-baseline off --deterministic > $o/bench_det.json 2> $o/bench_det.err; echo "rc=$?"; tail -2 $o/bench_det.err
python -c "import json;d=json.load(open('$o/bench_det.json'));print('det', d['ms_per_step'], d['output_ok'], {k:round(v['ms_per_step'],4) for k,v in d['stages'].items()})"
step shard
for i in 1 2; do
timeout -k 10 300 python bench.py --cpu-baseline off --n 12500000 --steps 30 --streams $i > $o/shard_$i.json 2> $o/shard_$i.err || { tail -5 $o/shard_$i.err; exit 1; }
python -c "import json;d=json.load(open('$o/shard_$i.json'));print('shard', d['ms_per_step'], {k:round(v['ms_per_step'],4) for k,v in d['stages'].items()})"
done
if [ -z "$NOPROF" ]; then
step rocprof
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$o/prof -o bench -- python3 $GRAFT_REPO_ROOT/bench.py --cpu-baseline off --steps 20 > $GRAFT_REPO_ROOT/$o/prof_bench.json 2> $GRAFT_REPO_ROOT/$o/prof_bench.err || { tail -5 $GRAFT_REPO_ROOT/$o/prof_bench.err; exit 1; }
cd $GRAFT_REPO_ROOT
find $o/prof -name "*stats*" | head
fi
if [ -z "$NOPROBE" ]; then
step decomposition probe
timeout -k 10 300 python tools/decomp_probe.py --interference --out $o/decomp.json > $o/decomp.log 2>&1 || { tail -5 $o/decomp.log; exit 1; }
tail -8 $o/decomp.log
fi
step rehearsal N=2 gloo on one GPU
for dc in zslab rows; do
ASP_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 2 --decomp $dc > $o/rehearsal_n2_$dc.json 2> $o/rehearsal_n2_$dc.err; echo "rc=$?"; tail -3 $o/rehearsal_n2_$dc.err | cut -c1-300
cut -c1-600 $o/rehearsal_n2_$dc.json
done
step overlap probe
timeout -k 10 300 python tools/overlap_probe.py --out $o/overlap.json > $o/overlap.log 2>&1; echo "rc=$?"; tail -6 $o/overlap.log
step done
