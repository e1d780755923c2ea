#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out/cfgs
run() { local name=$1; shift; timeout -k 10 300 python bench.py --cpu-baseline off --quiet "$@" > gpurun_out/cfgs/$name.json 2> gpurun_out/cfgs/$name.err; local rc=$?; echo "$name rc=$rc"; return $rc; }
run cfg2_phys_cubic_surface --n 10000000 --grid 2048 --h-law physical --kernel cubic --map surface --steps 5 --warmup 2 || exit $?
run cfg3_phys_wendland_weighted --n 100000000 --grid 4096 --h-law physical --steps 3 --warmup 1 || exit $?
run cfg3_pixel_cubic_surface --n 100000000 --grid 4096 --kernel cubic --map surface --steps 5 --warmup 2 || exit $?
exit 0
