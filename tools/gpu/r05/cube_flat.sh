#!/bin/bash
# Flattened column queue in the cube deposit: same-process A/B, then the cube tests.
cd "$GRAFT_REPO_ROOT" || exit 9
o=gpurun_out/r05/cube_flat; mkdir -p $o
timeout -k 10 300 python tools/cube_ab.py 'ASP_CUBE_FLAT=0' 'ASP_CUBE_FLAT=1' > $o/ab.log 2>&1 || { tail -20 $o/ab.log; exit 1; }
cat $o/ab.log
OUT=r05/cube_flat bash tools/gpu/run.sh tests tests/test_gpu_cube.py || exit 2
