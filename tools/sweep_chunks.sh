#!/bin/bash
# bench.py at several chunk counts (scatter/deposit overlap depth)
for c in ${CHUNKS:-1 2 3 4}; do
  timeout -k 10 200 python bench.py --cpu-baseline off --quiet --chunks $c "$@" > gpurun_out/q/chunks_$c.json 2> gpurun_out/q/chunks_$c.err || { echo "chunks $c failed"; tail -5 gpurun_out/q/chunks_$c.err; exit 1; }
  python3 - $c <<'PY'
import json,sys; d=json.load(open(f"gpurun_out/q/chunks_{sys.argv[1]}.json"))
print("chunks", sys.argv[1], d["ms_per_step"], d["output_ok"], {k: round(v["ms_per_launch"]*v["launches"]/d["steps"],3) for k,v in d["stages"].items() if v["launches"]})
PY
done
