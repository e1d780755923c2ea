#!/bin/bash
# Placement certainty: the default bench line in 8 fresh processes (each process runs its own
# placement trials in the warmup), then the 8-GPU shard size (1.25e7) and 2.5e7 on one GPU.
cd "$GRAFT_REPO_ROOT" || exit 9
o=gpurun_out/r03/placement8
mkdir -p $o
for i in 1 2 3 4 5 6 7 8; do
  timeout -k 10 200 python bench.py --cpu-baseline off --steps 10 > $o/p$i.json 2> $o/p$i.err || { tail -5 $o/p$i.err; exit 1; }
done
python tools/stages.py $o/p*.json
for n in 12500000 25000000; do
  timeout -k 10 200 python bench.py --cpu-baseline off --n $n > $o/n$n.json 2> $o/n$n.err || { tail -5 $o/n$n.err; exit 1; }
done
python tools/stages.py $o/n*.json
