#!/bin/bash
# GPU parity suite (verbose, per-test timeout), then the default bench line.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out/t2
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/t2/pytest.log 2>&1
rc=$?; tail -15 gpurun_out/t2/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --cpu-baseline off > gpurun_out/t2/bench.json 2> gpurun_out/t2/bench.err || { tail -5 gpurun_out/t2/bench.err; exit 1; }
cut -c1-400 gpurun_out/t2/bench.json
python3 -c "import json; d=json.load(open('gpurun_out/t2/bench.json')); print({k: round(v['ms_per_launch'],4) for k,v in d['stages'].items()})"
