#!/bin/bash
# One headline-bench run with extra bench.py flags ($@); prints the stage breakdown.
cd "$GRAFT_REPO_ROOT" || exit 9
export TMPDIR=/tmp
mkdir -p gpurun_out/v
timeout -k 10 240 python bench.py --cpu-baseline off --quiet "$@" > gpurun_out/v/bench.json 2> gpurun_out/v/bench.err
rc=$?
[ $rc -ne 0 ] && tail -5 gpurun_out/v/bench.err
[ -s gpurun_out/v/bench.json ] || exit $rc
python3 - <<'PY'
import json; d=json.load(open("gpurun_out/v/bench.json"))
print("variant", d["ms_per_step"], d["output_ok"], {k: round(v["ms_per_launch"],3) for k,v in d["stages"].items() if v["launches"]})
PY
exit $rc
