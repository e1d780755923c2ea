#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 9
o=gpurun_out/r05/cube_diag3; mkdir -p $o
timeout -k 10 300 python tools/cube_ab.py 'ASP_CUBE_DIAG=0' 'ASP_CUBE_DIAG=3' 'ASP_CUBE_DIAG=1' 'ASP_CUBE_DIAG=2' > $o/ab.log 2>&1 || { tail -20 $o/ab.log; exit 1; }
cat $o/ab.log
