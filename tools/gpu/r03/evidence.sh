#!/bin/bash
# Round-3 evidence for the bench line: PMC traffic of the headline map and of cfg 2 physical
# (tools/gpu/prof_full.sh, each pass its own rocprofv3 run) into gpurun_out/pmc_latest.json
# (copied to profiles/pmc_latest.json afterwards), then the default bench line (CPU baseline
# on) and the rocprof kernel stats of the same bench command (tools/gpu/bench_final.sh).
cd "$GRAFT_REPO_ROOT" || exit 9
export TMPDIR=/tmp
mkdir -p gpurun_out/final && cp profiles/pmc_latest.json gpurun_out/pmc_latest.json
bash tools/gpu/prof_full.sh r03cfg3 || exit 1
python3 tools/pmc_summary.py gpurun_out/prof_r03cfg3 --json gpurun_out/pmc_latest.json \
  --key n100000000_g4096_wendland_c2_pixel_weighted \
  --source "rocprofv3 PMC passes (FETCH_SIZE x2 + WRITE_SIZE), tools/gpu/r03/evidence.sh (prof_full.sh r03cfg3), round 3" > /dev/null || exit 2
bash tools/gpu/prof_full.sh r03cfg2p --n 10000000 --grid 2048 --kernel cubic --map surface --h-law physical || exit 3
python3 tools/pmc_summary.py gpurun_out/prof_r03cfg2p --json gpurun_out/pmc_latest.json \
  --key n10000000_g2048_cubic_physical_surface \
  --source "rocprofv3 PMC passes, tools/gpu/r03/evidence.sh (prof_full.sh r03cfg2p), round 3" > /dev/null || exit 4
cp gpurun_out/pmc_latest.json profiles/pmc_latest.json
bash tools/gpu/bench_final.sh || exit 5
mkdir -p gpurun_out/final
timeout -k 10 300 python bench.py --cpu-baseline off --n 10000000 --grid 2048 --kernel cubic --map surface --h-law physical > gpurun_out/final/bench_cfg2_physical.json 2> gpurun_out/final/bench_cfg2_physical.err || exit 6
timeout -k 10 300 python bench.py --cpu-baseline off --n 10000000 --grid 2048 --kernel cubic --map surface > gpurun_out/final/bench_cfg2_pixel.json 2> gpurun_out/final/bench_cfg2_pixel.err || exit 7
timeout -k 10 300 python bench.py --workload cube > gpurun_out/final/bench_cube.json 2> gpurun_out/final/bench_cube.err || exit 8
timeout -k 10 300 python bench.py --workload knn --n 10000000 > gpurun_out/final/bench_knn_1e7.json 2> gpurun_out/final/bench_knn_1e7.err || exit 9
python3 tools/stages.py gpurun_out/final/bench_n1.json gpurun_out/final/bench_cfg2_physical.json gpurun_out/final/bench_cfg2_pixel.json
python3 -c "
import json
for f in ['bench_cube','bench_knn_1e7']:
    d=json.load(open('gpurun_out/final/'+f+'.json')); print(f, d['ms_per_step'], d.get('stages'))"
