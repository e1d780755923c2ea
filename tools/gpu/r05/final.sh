#!/bin/bash
# Round-5 evidence on one build: GPU suite + smoke, the default bench line (CPU baseline on),
# the rocprofv3 kernel trace of the same command, the other workloads' lines, and the N = 2
# bench path rehearsed over gloo on this one GPU (both decompositions).
cd "$GRAFT_REPO_ROOT" || exit 9
export TMPDIR=/tmp
export OUT=r05/${TAG:-final}
o=gpurun_out/$OUT; mkdir -p $o
[ -z "$NOSUITE" ] && { bash tools/gpu/run.sh suite || exit 1; }
bash tools/gpu/run.sh bench bench_n1 || exit 2
echo "== $(date +%T) rocprof of the bench command"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/rp_bench -o bench -- python3 bench.py --cpu-baseline off > $o/rp_bench.json 2> $o/rp_bench.err || { tail -5 $o/rp_bench.err; exit 3; }
# the scatter launches of the sequential timed region: after the placement trials' own
# kernel (PROBE), warmup 3 - 1 (the first warmup map's scatter is a trial) + 10 timed
tr=$(find $o/rp_bench -name "*kernel_trace.csv" | head -1)
python3 tools/rocprof_timed.py $tr 'k_scatter<1, 2, 0, false, 0, 0, 0>' --skip 2 --count 10 > $o/rp_bench_timed.txt && tail -1 $o/rp_bench_timed.txt
bash tools/gpu/run.sh bench bench_cfg2_physical --cpu-baseline off --n 10000000 --grid 2048 --kernel cubic --map surface --h-law physical || exit 4
bash tools/gpu/run.sh bench bench_cfg2_pixel --cpu-baseline off --n 10000000 --grid 2048 --kernel cubic --map surface || exit 5
bash tools/gpu/run.sh bench bench_cube --workload cube || exit 6
bash tools/gpu/run.sh bench bench_knn_1e7 --workload knn --n 10000000 || exit 7
bash tools/gpu/run.sh bench bench_knn_1e8 --workload knn --n 100000000 --steps 2 --warmup 1 --cpu-baseline off || exit 8
bash tools/gpu/run.sh bench bench_shard --n 12500000 --steps 30 --cpu-baseline off || exit 9
bash tools/gpu/run.sh bench bench_stage --workload stage || exit 10
bash tools/gpu/run.sh bench bench_ion --workload ion || exit 11
for d in zslab rows; do
  echo "== $(date +%T) rehearsal N=2 $d (gloo, one GPU)"
  ASP_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 2 --cpu-baseline off --decomp $d > $o/reh_n2_$d.json 2> $o/reh_n2_$d.err || { tail -5 $o/reh_n2_$d.err; exit 12; }
  python3 -c "import json;d=json.loads(open('$o/reh_n2_$d.json').read().strip().splitlines()[-1]);print('$d', d['ms_per_step'], d['output_ok'], d['config']['workload'], d.get('partition_ms'), d['roofline']['frac'])"
done
[ -n "$CUBEPMC" ] && { bash tools/gpu/prof_full.sh r05cube_final --workload cube --iters 3 > $o/cube_pmc.log 2>&1 || exit 13; }
echo "== $(date +%T) done"
