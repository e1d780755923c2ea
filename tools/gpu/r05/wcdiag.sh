#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 9
o=gpurun_out/r05/wcdiag; mkdir -p $o
ASP_WC_DIAG=1 timeout -k 10 200 python -u tools/prof_driver.py --iters 2 > $o/diag.log 2>&1 || { tail -20 $o/diag.log; exit 1; }
grep "asp wc" $o/diag.log | head -20
