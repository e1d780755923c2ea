#!/bin/bash
# PMC pass over the cube bench (one counter set, kernel trace only)
cd "$GRAFT_REPO_ROOT" || exit 9
export TMPDIR=/tmp
mkdir -p gpurun_out/cube_pmc
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT --output-format csv -d gpurun_out/cube_pmc/p1 -o p1 -- python3 bench.py --workload cube --steps 1 --warmup 0 --cpu-baseline off > gpurun_out/cube_pmc/p1.log 2>&1 || { tail -5 gpurun_out/cube_pmc/p1.log; exit 1; }
f=$(find gpurun_out/cube_pmc/p1 -name '*counter_collection.csv' | head -1)
python3 - "$f" <<'PY'
import csv, sys, collections
acc = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(sys.argv[1])):
    k = r["Kernel_Name"][:60]
    if "k3_" not in k: continue
    acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, d in acc.items():
    print(k); [print("   ", c, f"{v:,.0f}") for c, v in sorted(d.items())]
PY
