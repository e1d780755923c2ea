#!/bin/bash
# Round 6: the stage events' share of the step (timed region with and without them), on
# the N = 8 share and the full map, alternating to cancel drift.
cd "$GRAFT_REPO_ROOT" || exit 9
export OUT=r06/t5
for r in 1 2; do
  bash tools/gpu/run.sh bench shard_ev_$r --n 12500000 --steps 50 --cpu-baseline off --overlap-streams 0 || exit 1
  bash tools/gpu/run.sh bench shard_noev_$r --n 12500000 --steps 50 --cpu-baseline off --overlap-streams 0 --no-stage-events || exit 2
done
bash tools/gpu/run.sh bench full_ev --steps 20 --cpu-baseline off --overlap-streams 0 || exit 3
bash tools/gpu/run.sh bench full_noev --steps 20 --cpu-baseline off --overlap-streams 0 --no-stage-events || exit 4
