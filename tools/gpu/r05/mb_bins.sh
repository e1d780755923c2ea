#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 9
o=gpurun_out/r05/mb; mkdir -p $o /tmp/mb
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -Wno-unused-result -o /tmp/mb/bins tools/microbench/bins.hip || exit 1
timeout -k 10 200 /tmp/mb/bins | tee $o/bins.log
