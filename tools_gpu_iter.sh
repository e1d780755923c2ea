#!/bin/bash
# one iteration: GPU tests, headline bench, physical-h configs
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out/iter
timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/iter/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/iter/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --cpu-baseline off --quiet > gpurun_out/iter/bench.json 2> gpurun_out/iter/bench.err || exit $?
python - <<'PY'
import json; d=json.load(open("gpurun_out/iter/bench.json"))
print("headline", d["ms_per_step"], {k: round(v["ms_per_launch"],3) for k,v in d["stages"].items() if v["launches"]})
PY
./tools_gpu_cfgs.sh || exit $?
for f in gpurun_out/cfgs/*.json; do python - "$f" <<'PY'
import json,sys; d=json.load(open(sys.argv[1]))
print(sys.argv[1].split("/")[-1], d["ms_per_step"], "rec/p", d["records_per_particle"], "wide", d["wide_particles"], {k: round(v["ms_per_launch"],3) for k,v in d["stages"].items() if v["launches"]})
PY
done
