#!/bin/bash
# Round-4: new props tests + the full suite, headline and cfg2 physical lines.
cd "$GRAFT_REPO_ROOT" || exit 9
export TMPDIR=/tmp
o=gpurun_out/r04/${TAG:-run5}
mkdir -p $o
echo "== $(date +%T) pytest props"
timeout -k 10 300 python -u -m pytest tests/test_gpu_props.py -q --timeout 200 --timeout-method thread -rf -x > $o/gputest_props.log 2>&1; rc=$?; tail -25 $o/gputest_props.log
[ $rc -le 1 ] || exit $rc
echo "== $(date +%T) pytest all"
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf > $o/gputest.log 2>&1; rc=$?; tail -6 $o/gputest.log
[ $rc -le 1 ] || exit $rc
TAG=${TAG:-run5} BENCHES="${BENCHES:-head cfg2p shard}" bash tools/gpu/r04/iter.sh || exit 1
echo "== $(date +%T) done"
