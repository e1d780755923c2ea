#!/bin/bash
# PMC of the headline map (kernel trace + SQ + HBM passes) on the current build.
cd "$GRAFT_REPO_ROOT" || exit 9
bash tools/gpu/prof_full.sh r05cfg3 --iters 3 || exit 1
