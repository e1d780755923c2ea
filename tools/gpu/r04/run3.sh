#!/bin/bash
# Round-4: row tests, shard / cfg2 physical A/B against the round-3 library, decomposition probe.
cd "$GRAFT_REPO_ROOT" || exit 9
export TMPDIR=/tmp
o=gpurun_out/r04/${TAG:-run3}
mkdir -p $o
echo "== $(date +%T) pytest rows"
timeout -k 10 300 python -u -m pytest tests/test_gpu_rows.py tests/test_gpu_streams.py -q --timeout 200 --timeout-method thread -rf > $o/gputest.log 2>&1; tail -4 $o/gputest.log
TAG=${TAG:-run3} BENCHES="${BENCHES:-shard shard1 shard_r03 cfg2p cfg2p_r03 cfg2p head1 head_r03}" bash tools/gpu/r04/iter.sh || exit 1
echo "== $(date +%T) decomposition probe"
timeout -k 10 300 python tools/decomp_probe.py --out $o/decomp.json > $o/decomp.log 2>&1 || { tail -5 $o/decomp.log; exit 1; }
tail -4 $o/decomp.log
echo "== $(date +%T) done"
