#!/bin/bash
# Headline bench once per environment setting: bash tools/gpu_env_sweep.sh VAR v1 v2 ...
cd "$GRAFT_REPO_ROOT" || exit 9
export TMPDIR=/tmp
mkdir -p gpurun_out/v
var=$1; shift
for val in "$@"; do
  env "$var=$val" timeout -k 10 240 python bench.py --cpu-baseline off --quiet > gpurun_out/v/$var$val.json 2> gpurun_out/v/$var$val.err
  rc=$?
  [ -s gpurun_out/v/$var$val.json ] || { echo "$var=$val failed rc=$rc"; tail -5 gpurun_out/v/$var$val.err; exit 1; }
  python3 - gpurun_out/v/$var$val.json "$var=$val" <<'PY'
import json,sys; d=json.load(open(sys.argv[1]))
print(f"{sys.argv[2]:>22}", d["ms_per_step"], d["output_ok"], {k: round(v["ms_per_launch"],3) for k,v in d["stages"].items() if v["launches"]})
PY
done
