#!/bin/bash
# Compile-time variants of the cube deposit (ab_* builds) against the working library.
cd "$GRAFT_REPO_ROOT" || exit 9
o=gpurun_out/r05/cube_variants; mkdir -p $o
for v in "" $VARIANTS; do
  if [ -n "$v" ]; then export ASP_LIB=astro-sph-tools_amd/ab_$v/libasp_hip.so; else unset ASP_LIB; fi
  timeout -k 10 300 python tools/cube_ab.py 'ASP_CUBE_DIAG=0' > $o/${v:-work}.log 2>&1 || { tail -20 $o/${v:-work}.log; exit 2; }
  grep "rep 1" $o/${v:-work}.log | sed "s/^/${v:-work} /"
done
