#!/bin/bash
# One iteration: GPU parity suite, then the headline config and the 8-GPU shard size.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out/it
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/it/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/it/pytest.log; [ $rc -ne 0 ] && exit $rc
bash tools/gpu/libs.sh "${1:-base}"
