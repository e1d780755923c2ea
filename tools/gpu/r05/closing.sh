#!/bin/bash
# Closing check on the final build: GPU suite + smoke, the default bench line (CPU baseline
# on), the cube line.
cd "$GRAFT_REPO_ROOT" || exit 9
export OUT=r05/closing
bash tools/gpu/run.sh suite || exit 1
bash tools/gpu/run.sh bench bench_n1 || exit 2
bash tools/gpu/run.sh bench bench_cube --workload cube || exit 3
