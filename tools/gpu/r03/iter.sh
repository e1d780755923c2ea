#!/bin/bash
# Round-3 iteration: selected GPU tests ($TESTS, default all), the default bench line
# (BENCH=0 skips), and extra commands ($EXTRA, run with bash -c, each under its own timeout).
cd "$GRAFT_REPO_ROOT" || exit 9
export TMPDIR=/tmp
o=gpurun_out/r03/${TAG:-iter}
mkdir -p $o
step() { echo "== $(date +%T) $*"; }
if [ "${TESTS:-all}" != "none" ]; then
  step pytest ${TESTS:-all}
  sel=${TESTS:-tests}; [ "$sel" = "all" ] && sel=tests
  timeout -k 10 900 python -u -m pytest $sel -m gpu -q --timeout 300 --timeout-method thread -rf > $o/gputest.log 2>&1; rc=$?; tail -6 $o/gputest.log
  [ $rc -le 1 ] || exit $rc
fi
if [ "${BENCH:-1}" = "1" ]; then
  step bench
  timeout -k 10 300 python bench.py --cpu-baseline off > $o/bench_n1.json 2> $o/bench_n1.err || { tail -5 $o/bench_n1.err; exit 1; }
  python -c "import json;d=json.load(open('$o/bench_n1.json'));print(d['ms_per_step'], {k: round(v['ms_per_launch'],4) for k,v in d['stages'].items()})"
fi
if [ -n "$EXTRA" ]; then
  step extra
  timeout -k 10 600 bash -c "$EXTRA" > $o/extra.log 2>&1; rc=$?; tail -40 $o/extra.log; exit $rc
fi
step done
