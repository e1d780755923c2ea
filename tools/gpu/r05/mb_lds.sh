#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 9
o=gpurun_out/r05/mb; mkdir -p $o
mkdir -p /tmp/mb
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -munsafe-fp-atomics -o /tmp/mb/lds tools/microbench/lds.hip || exit 1
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -munsafe-fp-atomics -fgpu-flush-denormals-to-zero -o /tmp/mb/lds_ftz tools/microbench/lds.hip || exit 1
echo "== default denormal mode"; timeout -k 10 60 /tmp/mb/lds | grep "span  8192" | tee $o/lds.log
echo "== flush denormals"; timeout -k 10 60 /tmp/mb/lds_ftz | grep "span  8192" | tee $o/lds_ftz.log
