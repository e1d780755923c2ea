#!/bin/bash
# parameter sweep of a library tuning knob on one config: tools_gpu_sweep.sh VAR "v1 v2 .." bench-args...
cd "$GRAFT_REPO_ROOT" || exit 9
var=$1; vals=$2; shift 2
mkdir -p gpurun_out/sweep
for v in $vals; do
  env $var=$v timeout -k 10 300 python bench.py --cpu-baseline off --quiet "$@" > gpurun_out/sweep/$var-$v.json 2> gpurun_out/sweep/$var-$v.err || exit $?
  python - "$var=$v" gpurun_out/sweep/$var-$v.json <<'PY'
import json,sys; d=json.load(open(sys.argv[2]))
print(sys.argv[1], d["ms_per_step"], {k: round(v["ms_per_launch"],3) for k,v in d["stages"].items() if v["launches"]})
PY
done
