# Cube deposit PMC for the current library and ab/colwalk (kernel trace + two SQ passes each).
cd "$GRAFT_REPO_ROOT" || exit 9
bash tools/gpu/prof_cmd.sh cube_sweep bench.py --workload cube --cpu-baseline off --steps 3 --warmup 1 > gpurun_out/cube_sweep.log 2>&1 || { tail gpurun_out/cube_sweep.log; exit 1; }
ASP_LIB=$PWD/ab/colwalk/libasp_hip.so bash tools/gpu/prof_cmd.sh cube_colwalk bench.py --workload cube --cpu-baseline off --steps 3 --warmup 1 > gpurun_out/cube_colwalk.log 2>&1 || { tail gpurun_out/cube_colwalk.log; exit 1; }
for t in sweep colwalk; do echo "## $t"; grep -A24 "== k3_deposit" gpurun_out/prof_cube_$t/summary.txt | grep -E "avg_us|SQ_"; done
