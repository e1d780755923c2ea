#!/bin/bash
# Cube A/B in one process: compacted scatter, scatter block count.
cd "$GRAFT_REPO_ROOT" || exit 9
o=gpurun_out/r05/cube_ab; mkdir -p $o
timeout -k 10 300 python tools/cube_ab.py 'ASP_CUBE_COMPACT=0,ASP_CUBE_NBLK=512' 'ASP_CUBE_COMPACT=1,ASP_CUBE_NBLK=512' \
  'ASP_CUBE_COMPACT=0,ASP_CUBE_NBLK=256' 'ASP_CUBE_COMPACT=1,ASP_CUBE_NBLK=256' 'ASP_CUBE_COMPACT=1,ASP_CUBE_NBLK=1024' > $o/ab.log 2>&1 || { tail -20 $o/ab.log; exit 1; }
cat $o/ab.log
