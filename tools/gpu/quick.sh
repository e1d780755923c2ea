#!/bin/bash
# Quick loop: GPU parity tests, then the shard-size sweep, then a 2-rank gloo rehearsal.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out/q
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/q/pytest.log 2>&1
rc=$?; tail -2 gpurun_out/q/pytest.log; [ $rc -ne 0 ] && exit $rc
bash tools/gpu/nsweep.sh || exit $?
if [ -n "$REHEARSE" ]; then
ASP_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 1 --op allreduce --quiet > gpurun_out/q/r2.json 2> gpurun_out/q/r2.err
rc=$?; echo "2-rank rehearsal rc=$rc"; cut -c1-200 gpurun_out/q/r2.json; [ $rc -ne 0 ] && tail -5 gpurun_out/q/r2.err
fi
exit 0
