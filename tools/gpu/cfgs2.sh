#!/bin/bash
# Stage breakdowns of the BASELINE configs (no CPU baseline), plus gather-threshold sweep.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out/cfgs2
run() {  # name, env..., -- bench args
  local name=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 300 python bench.py --cpu-baseline off --quiet "$@" > gpurun_out/cfgs2/$name.json 2> gpurun_out/cfgs2/$name.err || { echo "$name failed"; tail -3 gpurun_out/cfgs2/$name.err; return 1; }
  python3 - gpurun_out/cfgs2/$name.json $name <<'PY'
import json,sys; d=json.load(open(sys.argv[1]))
print(sys.argv[2], d["ms_per_step"], d["output_ok"], "large", d.get("large_records"), {k: round(v["ms_per_launch"],3) for k,v in d["stages"].items()})
PY
}
run cfg3_pixel A=1 -- --steps 10 || exit 1
run cfg2_pixel A=1 -- --n 10000000 --grid 2048 --kernel cubic --map surface --steps 20 || exit 1
for gm in 8 12 16 24 65; do
  run cfg2_phys_g$gm ASP_GATHER_MIN=$gm -- --n 10000000 --grid 2048 --kernel cubic --map surface --h-law physical --steps 5 --warmup 2 || exit 1
done
run cfg3_phys A=1 -- --h-law physical --steps 3 --warmup 1 || exit 1
