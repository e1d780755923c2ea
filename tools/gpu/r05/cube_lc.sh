#!/bin/bash
# Column classes baked in: lane_cols sweep (same process), then the cube tests.
cd "$GRAFT_REPO_ROOT" || exit 9
o=gpurun_out/r05/cube_lc; mkdir -p $o
timeout -k 10 400 python tools/cube_ab.py 'ASP_CUBE_LANE_COLS=48' 'ASP_CUBE_LANE_COLS=36' 'ASP_CUBE_LANE_COLS=64' 'ASP_CUBE_LANE_COLS=96' > $o/ab.log 2>&1 || { tail -20 $o/ab.log; exit 1; }
cat $o/ab.log
OUT=r05/cube_lc bash tools/gpu/run.sh tests tests/test_gpu_cube.py || exit 2
