#!/bin/bash
# Round 6: the GPU suite + smoke on the build with k_binscan (column + tile scans in one
# launch, no counter memset) and the deposit-fused merge; then the bench lines (events
# around the dominant kernel only in the timed region) for the full map and the share.
cd "$GRAFT_REPO_ROOT" || exit 9
export OUT=r06/t6
bash tools/gpu/run.sh suite || exit 1
bash tools/gpu/run.sh bench full --steps 20 --cpu-baseline off --overlap-streams 2 || exit 2
bash tools/gpu/run.sh bench shard_1s --n 12500000 --steps 50 --cpu-baseline off --overlap-streams 0 || exit 3
ASP_SCATTER_GATE=1 bash tools/gpu/run.sh bench shard_2s --n 12500000 --steps 50 --cpu-baseline off --streams 2 --overlap-streams 0 || exit 4
