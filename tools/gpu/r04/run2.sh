#!/bin/bash
# Round-4 second checkpoint: GPU suite, bench lines (iter.sh), the decomposition probe.
cd "$GRAFT_REPO_ROOT" || exit 9
export TMPDIR=/tmp
o=gpurun_out/r04/${TAG:-run2}
mkdir -p $o
echo "== $(date +%T) pytest"
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf > $o/gputest.log 2>&1; rc=$?; tail -15 $o/gputest.log
[ $rc -le 1 ] || exit $rc
TAG=${TAG:-run2} BENCHES="${BENCHES:-head det1 shard shard1 cfg2p}" bash tools/gpu/r04/iter.sh || exit 1
echo "== $(date +%T) decomposition probe"
timeout -k 10 300 python tools/decomp_probe.py --out $o/decomp.json > $o/decomp.log 2>&1 || { tail -5 $o/decomp.log; exit 1; }
tail -4 $o/decomp.log
echo "== $(date +%T) done"
