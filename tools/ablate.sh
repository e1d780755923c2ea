#!/bin/bash
# Build diagnostic variants of libasp_hip.so (never the product library):
#   lib/libasp_hip_<MACRO><k>.so with -D<MACRO>=k   (MACRO: ASP_ABLATE, ASP_ABLATE_SCATTER)
#   usage: tools/ablate.sh MACRO k1 k2 ...
cd "$(dirname "$0")/../astro-sph-tools_amd" || exit 1
m=$1; shift
for k in "$@"; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -ffp-contract=off -munsafe-fp-atomics \
    -D$m=$k -shared -o lib/libasp_hip_$m$k.so csrc/asp_project2d.hip csrc/asp_project3d.hip csrc/asp_stage.hip csrc/asp_knn.hip csrc/asp_table.hip || exit 1
done
