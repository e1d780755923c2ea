#!/bin/bash
# Box and offsets carried in the cube records: tests, then base (HEAD) vs working library.
cd "$GRAFT_REPO_ROOT" || exit 9
o=gpurun_out/r05/cube_rec; mkdir -p $o
OUT=r05/cube_rec bash tools/gpu/run.sh tests tests/test_gpu_cube.py tests/test_gpu_streams.py || exit 1
for rep in 1 2; do
  ASP_LIB=astro-sph-tools_amd/ab_base/libasp_hip.so timeout -k 10 300 python tools/cube_ab.py 'ASP_CUBE_DIAG=0' > $o/base_$rep.log 2>&1 || { tail -20 $o/base_$rep.log; exit 2; }
  grep "rep 1" $o/base_$rep.log | sed "s/^/base /"
  timeout -k 10 300 python tools/cube_ab.py 'ASP_CUBE_DIAG=0' > $o/new_$rep.log 2>&1 || { tail -20 $o/new_$rep.log; exit 3; }
  grep "rep 1" $o/new_$rep.log | sed "s/^/new /"
done
