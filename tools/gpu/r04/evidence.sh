#!/bin/bash
# Round-4 evidence: PMC passes of the headline and of cfg 2 physical (tools/gpu/prof_full.sh,
# each pass its own rocprofv3 run) into gpurun_out/pmc_latest.json, the default bench line
# (CPU baseline on), the rocprof kernel stats of the same bench command, and the other
# workloads' lines.
cd "$GRAFT_REPO_ROOT" || exit 9
export TMPDIR=/tmp
o=gpurun_out/r04/final; mkdir -p $o
cp profiles/pmc_latest.json gpurun_out/pmc_latest.json
bash tools/gpu/prof_full.sh r04cfg3 || exit 1
python3 tools/pmc_summary.py gpurun_out/prof_r04cfg3 --json gpurun_out/pmc_latest.json \
  --key n100000000_g4096_wendland_c2_pixel_weighted \
  --source "rocprofv3 PMC passes (FETCH_SIZE x2 + WRITE_SIZE), tools/gpu/r04/evidence.sh (prof_full.sh r04cfg3), round 4" > /dev/null || exit 2
bash tools/gpu/prof_full.sh r04cfg2p --n 10000000 --grid 2048 --kernel cubic --map surface --h-law physical || exit 3
python3 tools/pmc_summary.py gpurun_out/prof_r04cfg2p --json gpurun_out/pmc_latest.json \
  --key n10000000_g2048_cubic_physical_surface \
  --source "rocprofv3 PMC passes, tools/gpu/r04/evidence.sh (prof_full.sh r04cfg2p), round 4" > /dev/null || exit 4
cp gpurun_out/pmc_latest.json $o/pmc_latest.json
cp gpurun_out/pmc_latest.json profiles/pmc_latest.json
echo "== $(date +%T) bench line"
timeout -k 10 600 python bench.py > $o/bench_n1.json 2> $o/bench_n1.err || { tail -5 $o/bench_n1.err; exit 5; }
cut -c1-400 $o/bench_n1.json
echo "== $(date +%T) rocprof of the bench command"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/rp_bench -o bench -- python3 bench.py --cpu-baseline off > $o/rp_bench.json 2> $o/rp_bench.err || exit 6
cut -c1-200 $o/rp_bench.json
echo "== $(date +%T) other lines"
timeout -k 10 300 python bench.py --cpu-baseline off --n 10000000 --grid 2048 --kernel cubic --map surface --h-law physical > $o/bench_cfg2_physical.json 2> $o/bench_cfg2_physical.err || exit 7
timeout -k 10 300 python bench.py --cpu-baseline off --n 10000000 --grid 2048 --kernel cubic --map surface > $o/bench_cfg2_pixel.json 2> $o/bench_cfg2_pixel.err || exit 8
timeout -k 10 300 python bench.py --workload cube > $o/bench_cube.json 2> $o/bench_cube.err || exit 9
timeout -k 10 300 python bench.py --workload knn --n 10000000 > $o/bench_knn_1e7.json 2> $o/bench_knn_1e7.err || exit 10
for f in bench_n1 bench_cfg2_physical bench_cfg2_pixel bench_cube bench_knn_1e7; do
python3 -c "import json;d=json.load(open('$o/$f.json'));print('$f', d['ms_per_step'], d.get('output_ok'), d.get('roofline',{}).get('kernel'), d.get('roofline',{}).get('frac'))"
done
echo "== $(date +%T) done"
