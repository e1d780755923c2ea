#!/bin/bash
# PMC of the headline scatter with and without write-combining (ASP_WC_SLOTS=0).
cd "$GRAFT_REPO_ROOT" || exit 9
ASP_WC_SLOTS=0 bash tools/gpu/prof_full.sh r05_wc0 --iters 3 || exit 1
bash tools/gpu/prof_full.sh r05_wc352 --iters 3 || exit 2
