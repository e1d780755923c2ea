#!/bin/bash
# Working library vs ab_base (HEAD), alternating processes; the working one also split by class.
cd "$GRAFT_REPO_ROOT" || exit 9
o=gpurun_out/r05/${TAG:-cube_ab_base}; mkdir -p $o
for rep in 1 2; do
  ASP_LIB=astro-sph-tools_amd/ab_base/libasp_hip.so timeout -k 10 300 python tools/cube_ab.py 'ASP_CUBE_DIAG=0' > $o/base_$rep.log 2>&1 || { tail -20 $o/base_$rep.log; exit 2; }
  grep "rep 1" $o/base_$rep.log | sed "s/^/base /"
  timeout -k 10 300 python tools/cube_ab.py 'ASP_CUBE_DIAG=0' ${SPLIT:+'ASP_CUBE_DIAG=1' 'ASP_CUBE_DIAG=2'} > $o/new_$rep.log 2>&1 || { tail -20 $o/new_$rep.log; exit 3; }
  grep "rep 1" $o/new_$rep.log | sed "s/^/new /"
done
