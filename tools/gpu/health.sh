#!/bin/bash
# Health check on one MI355X: GPU test suite, smoke(), default bench line.
cd "$GRAFT_REPO_ROOT" || exit 9
export TMPDIR=/tmp
o=gpurun_out/h
mkdir -p $o
step() { echo "== $(date +%T) $*"; }
step pytest
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $o/gputest.log 2>&1
rc=$?; tail -3 $o/gputest.log; [ $rc -ne 0 ] && exit $rc
step smoke
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || { tail -5 $o/smoke.log; exit 1; }
cat $o/smoke.log
step bench
timeout -k 10 300 python bench.py --cpu-baseline off > $o/bench.json 2> $o/bench.err || { tail -5 $o/bench.err; exit 1; }
cut -c1-600 $o/bench.json
step done
