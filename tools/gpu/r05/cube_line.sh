#!/bin/bash
# Cube bench lines (two streams default, and one stream).
cd "$GRAFT_REPO_ROOT" || exit 9
export OUT=r05/${TAG:-cube_line}
bash tools/gpu/run.sh reps 2 cube --workload cube --cpu-baseline off || exit 1
bash tools/gpu/run.sh bench cube_s1 --workload cube --streams 1 --cpu-baseline off || exit 2
