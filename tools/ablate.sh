#!/bin/bash
# Build diagnostic variants of libasp_hip.so (never the product library):
#   lib/libasp_hip_ablate<k>.so with -DASP_ABLATE=k
cd "$(dirname "$0")/../astro-sph-tools_amd" || exit 1
for k in "$@"; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -ffp-contract=off -munsafe-fp-atomics \
    -DASP_ABLATE=$k -shared -o lib/libasp_hip_ablate$k.so csrc/asp_project2d.hip || exit 1
done
