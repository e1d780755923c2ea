#!/bin/bash
# Per-rank compute at the strong-scaling shard sizes (10^8 / N particles, full 4096^2 map).
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out/ns
for n in 12500000 25000000 50000000 100000000; do
  timeout -k 10 200 python bench.py --cpu-baseline off --quiet --n $n --steps 20 > gpurun_out/ns/n$n.json 2> gpurun_out/ns/n$n.err || { echo "n=$n failed"; tail -5 gpurun_out/ns/n$n.err; exit 1; }
  python3 - $n <<'PY'
import json,sys; d=json.load(open(f"gpurun_out/ns/n{sys.argv[1]}.json"))
print(sys.argv[1], d["ms_per_step"], d["output_ok"], {k: round(v["ms_per_launch"],3) for k,v in d["stages"].items()})
PY
done
