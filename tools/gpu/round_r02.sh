#!/bin/bash
# Round-2 evidence run on one MI355X: GPU tests, the default bench line (with the CPU
# baseline), the rocprof kernel stats of that same bench command, PMC traffic passes,
# the other configs' bench lines, and placement probes.  Output: gpurun_out/r02/.
cd "$GRAFT_REPO_ROOT" || exit 9
export TMPDIR=/tmp
o=gpurun_out/r02
mkdir -p $o
step() { echo "== $(date +%T) $*"; }
step pytest
timeout -k 10 300 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > $o/gputest.log 2>&1; tail -2 $o/gputest.log
step bench default
timeout -k 10 300 python bench.py > $o/bench_n1.json 2> $o/bench_n1.err || { tail -5 $o/bench_n1.err; exit 1; }
cat $o/bench_n1.json | head -c 400; echo
step rocprof bench
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/rp_bench -o bench -- python3 bench.py --cpu-baseline off > $o/rp_bench.json 2> $o/rp_bench.err || exit 1
step pmc
bash tools/gpu/prof_full.sh r02cfg3 --iters 3 > $o/pmc.log 2>&1 || { tail -5 $o/pmc.log; exit 1; }
python3 tools/pmc_summary.py gpurun_out/prof_r02cfg3 --json $o/pmc_latest.json --key n100000000_g4096_wendland_c2_pixel_weighted --source "rocprofv3 PMC passes (FETCH_SIZE x2 + WRITE_SIZE), tools/gpu/prof_full.sh r02cfg3, same build as bench_n1.json" > /dev/null
step configs
timeout -k 10 200 python bench.py --cpu-baseline off --n 10000000 --grid 2048 --kernel cubic --map surface --h-law pixel > $o/bench_cfg2_pixel.json 2>/dev/null || exit 1
timeout -k 10 200 python bench.py --cpu-baseline off --n 10000000 --grid 2048 --kernel cubic --map surface --h-law physical > $o/bench_cfg2_physical.json 2>/dev/null || exit 1
timeout -k 10 300 python bench.py --cpu-baseline off --h-law physical --steps 3 --warmup 1 > $o/bench_cfg3_physical.json 2>/dev/null || exit 1
timeout -k 10 300 python bench.py --workload cube --cpu-baseline off > $o/bench_cube.json 2>/dev/null || exit 1
timeout -k 10 300 python bench.py --workload knn --n 10000000 --cpu-baseline off > $o/bench_knn_1e7.json 2>/dev/null || exit 1
timeout -k 10 200 python bench.py --workload stage --cpu-baseline off > $o/bench_stage.json 2>/dev/null || exit 1
timeout -k 10 200 python bench.py --workload ion --cpu-baseline off > $o/bench_ion.json 2>/dev/null || exit 1
step rocprof cfg2 physical
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/rp_cfg2phys -o cfg2phys -- python3 bench.py --cpu-baseline off --n 10000000 --grid 2048 --kernel cubic --map surface --h-law physical > /dev/null 2>&1 || exit 1
step alloc probe
TRIALS=8 timeout -k 10 300 python -u tools/alloc_probe.py > $o/alloc_probe.log 2>&1 || exit 1
step done
