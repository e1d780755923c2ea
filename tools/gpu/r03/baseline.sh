#!/bin/bash
# Round-3 checkpoint: GPU tests (all, no -x), the default bench line, cfg2 at physical h
# (VALU roofline block), the LDS microbenchmark.
cd "$GRAFT_REPO_ROOT" || exit 9
export TMPDIR=/tmp
o=gpurun_out/r03/${TAG:-baseline}
mkdir -p $o
step() { echo "== $(date +%T) $*"; }
step pytest
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf > $o/gputest.log 2>&1; rc=$?; tail -15 $o/gputest.log
[ $rc -le 1 ] || exit $rc
step bench
timeout -k 10 300 python bench.py --cpu-baseline off > $o/bench_n1.json 2> $o/bench_n1.err || { tail -5 $o/bench_n1.err; exit 1; }
cut -c1-700 $o/bench_n1.json
step bench cfg2 physical
timeout -k 10 300 python bench.py --cpu-baseline off --n 10000000 --grid 2048 --kernel cubic --map surface --h-law physical > $o/bench_cfg2_physical.json 2> $o/bench_cfg2_physical.err || { tail -5 $o/bench_cfg2_physical.err; exit 1; }
python -c "import json;d=json.load(open('$o/bench_cfg2_physical.json'));print(d['ms_per_step'], json.dumps(d['roofline']))"
if [ -z "$TAG" ]; then
step microbench lds
hipcc -O3 --offload-arch=gfx950 -munsafe-fp-atomics -o /tmp/mb_lds tools/microbench/lds.hip && timeout -k 10 120 /tmp/mb_lds > $o/microbench_lds.txt 2>&1; cat $o/microbench_lds.txt
fi
step done
