#!/bin/bash
# A/B: headline bench with the product library and each diagnostic variant lib/libasp_hip_<V>.so
# (variants build wrong maps on purpose: a failed output check is reported, not fatal).
for v in "" "$@"; do
  lib=astro-sph-tools_amd/lib/libasp_hip${v:+_$v}.so
  ASP_LIB=$GRAFT_REPO_ROOT/$lib timeout -k 10 200 python bench.py --cpu-baseline off --quiet > gpurun_out/q/ab_${v:-prod}.json 2> gpurun_out/q/ab_${v:-prod}.err
  rc=$?
  [ -s gpurun_out/q/ab_${v:-prod}.json ] || { echo "$v failed rc=$rc"; tail -3 gpurun_out/q/ab_${v:-prod}.err; exit 1; }
  python3 - ${v:-prod} <<'PY'
import json,sys; d=json.load(open(f"gpurun_out/q/ab_{sys.argv[1]}.json"))
print(f"{sys.argv[1]:>22}", d["ms_per_step"], d["output_ok"], {k: round(v["ms_per_launch"],3) for k,v in d["stages"].items() if v["launches"]})
PY
done
