#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 9
./tools_gpu_sweep.sh ASP_WIDE_TILES "16 64 256 1024" --n 100000000 --grid 4096 --h-law physical --steps 2 --warmup 1 || exit $?
./tools_gpu_sweep.sh ASP_WIDE_TILES "16 64 256 1024" --n 10000000 --grid 2048 --h-law physical --kernel cubic --map surface --steps 3 --warmup 1 || exit $?
