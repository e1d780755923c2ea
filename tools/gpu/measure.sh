#!/bin/bash
# Full measurement session: tests, PMC traffic, bench (with CPU baseline), rocprof stats,
# and a 2-rank rehearsal of the distributed path (gloo, both ranks on the one GPU).
cd "$GRAFT_REPO_ROOT" || exit 9
export TMPDIR=/tmp
mkdir -p gpurun_out/meas
timeout -k 10 500 python -m pytest tests -m gpu -q -p no:cacheprovider --timeout 200 > gpurun_out/meas/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/meas/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash tools/profile_session.sh meas || exit $?
python3 tools/pmc_summary.py gpurun_out/prof_meas --json gpurun_out/meas/pmc_latest.json \
  --key n100000000_g4096_wendland_c2_pixel_weighted --source "rocprofv3 PMC passes, tools/prof_driver.py (same config as bench.py defaults)" > /dev/null
timeout -k 10 600 python bench.py --pmc gpurun_out/meas/pmc_latest.json > gpurun_out/meas/bench.json 2> gpurun_out/meas/bench.err
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/meas/bench.json | cut -c1-300
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/meas/rocprof_bench -o bench -- python3 bench.py --cpu-baseline off --steps 10 --warmup 3 > gpurun_out/meas/rocprof_bench.log 2>&1
rc=$?; echo "rocprof bench rc=$rc"
[ $rc -ne 0 ] && exit $rc
ASP_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 1 --op allreduce > gpurun_out/meas/bench_2rank_gloo.json 2> gpurun_out/meas/bench_2rank_gloo.err
rc=$?; echo "2-rank rehearsal rc=$rc"; tail -1 gpurun_out/meas/bench_2rank_gloo.json | cut -c1-300
timeout -k 10 300 python bench.py --workload stage --steps 10 --warmup 2 > gpurun_out/meas/bench_stage.json 2> gpurun_out/meas/bench_stage.err
rc=$?; echo "stage bench rc=$rc"; tail -1 gpurun_out/meas/bench_stage.json | cut -c1-300
timeout -k 10 300 python bench.py --workload cube --steps 3 --warmup 1 > gpurun_out/meas/bench_cube.json 2> gpurun_out/meas/bench_cube.err
rc=$?; echo "cube bench rc=$rc"; tail -1 gpurun_out/meas/bench_cube.json | cut -c1-300
exit 0
