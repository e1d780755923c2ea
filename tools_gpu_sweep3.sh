#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 9
export ASP_LIB=$PWD/astro-sph-tools_amd/lib/libasp_hip_ASP_COUNT_BLOCK1024.so
./tools_gpu_sweep.sh ASP_BIN_BLOCKS "128 256 512" --steps 5 --warmup 2
