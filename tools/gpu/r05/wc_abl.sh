#!/bin/bash
# Where the scatter's time goes: stores ablated (wrong maps), write-combining on / off.
cd "$GRAFT_REPO_ROOT" || exit 9
o=gpurun_out/r05/wcabl; mkdir -p $o
AB_NOCHECK=1 timeout -k 10 300 python -u tools/scatter_ab.py ASP_WC_SLOTS=0 ASP_WC_SLOTS=0,ASP_WC_DIAG=2 ASP_WC_SLOTS=352 ASP_WC_SLOTS=352,ASP_WC_DIAG=2 ASP_WC_SLOTS=352,ASP_WC_DIAG=6 > $o/abl.log 2>&1 || { tail -20 $o/abl.log; exit 1; }
grep -v amdgpu.ids $o/abl.log
echo "== segmented-reduction microbenchmark"
mkdir -p /tmp/mb && /opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -munsafe-fp-atomics -o /tmp/mb/seg tools/microbench/segred.hip && timeout -k 10 60 /tmp/mb/seg > $o/segred.log 2>&1; cat $o/segred.log
