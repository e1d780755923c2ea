#!/bin/bash
# 32x16x32 bricks (working library) vs 16x16x32 (ab_bx16, same sources) vs HEAD (ab_base):
# cube tests on the working library first.
cd "$GRAFT_REPO_ROOT" || exit 9
o=gpurun_out/r05/cube_bx; mkdir -p $o
OUT=r05/cube_bx bash tools/gpu/run.sh tests tests/test_gpu_cube.py || exit 1
for rep in 1 2; do
  for v in base bx16 ""; do
    if [ -n "$v" ]; then export ASP_LIB=astro-sph-tools_amd/ab_$v/libasp_hip.so; else unset ASP_LIB; fi
    timeout -k 10 300 python tools/cube_ab.py 'ASP_CUBE_DIAG=0' > $o/${v:-work}_$rep.log 2>&1 || { tail -20 $o/${v:-work}_$rep.log; exit 2; }
    grep "rep 1" $o/${v:-work}_$rep.log | sed "s/^/${v:-work} /"
  done
done
