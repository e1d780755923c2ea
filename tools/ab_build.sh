#!/bin/bash
# Same-box A/B builds: compile the library of a git revision (default HEAD) into
# astro-sph-tools_amd/ab_<name>/libasp_hip.so (git-ignored; it travels with gpurun -- delete it
# after the A/B: every lease ships it), to run
# beside the working build with ASP_LIB=astro-sph-tools_amd/ab_<name>/libasp_hip.so.
#   bash tools/ab_build.sh <name> [rev] [extra hipcc flags]
set -e
name=$1; rev=${2:-HEAD}; extra=$3
root=$(cd "$(dirname "$0")/.." && pwd)
tmp=$(mktemp -d /tmp/ab_XXXX)
git -C "$root" archive "$rev" astro-sph-tools_amd/csrc astro-sph-tools_amd/Makefile include | tar -x -C "$tmp"
make -C "$tmp/astro-sph-tools_amd" -j8 HIPFLAGS="-O3 -std=c++17 --offload-arch=gfx950 -fPIC -ffp-contract=off -Wall -Wno-unused-result -munsafe-fp-atomics $extra" > "$tmp/build.log" 2>&1 || { tail -20 "$tmp/build.log"; exit 1; }
mkdir -p "$root/astro-sph-tools_amd/ab_$name"
cp "$tmp/astro-sph-tools_amd/lib/libasp_hip.so" "$root/astro-sph-tools_amd/ab_$name/"
rm -rf "$tmp"
echo "built ab_$name from $rev"
