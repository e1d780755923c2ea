#!/bin/bash
# GPU iteration: parity tests, headline bench, optional extra command ($1).
cd "$GRAFT_REPO_ROOT" || exit 9
export TMPDIR=/tmp
mkdir -p gpurun_out/q
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/q/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/q/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --cpu-baseline off --quiet > gpurun_out/q/bench.json 2> gpurun_out/q/bench.err
rc=$?
python3 - <<'PY'
import json; d=json.load(open("gpurun_out/q/bench.json"))
print("headline", d["ms_per_step"], d["output_ok"], {k: round(v["ms_per_launch"],3) for k,v in d["stages"].items() if v["launches"]})
PY
[ $rc -ne 0 ] && exit $rc
if [ -n "$1" ]; then timeout -k 10 300 bash -c "$1" > gpurun_out/q/extra.log 2>&1; rc=$?; cat gpurun_out/q/extra.log | tail -40; exit $rc; fi
exit 0
