#!/bin/bash
# N = 4 bench path rehearsed over gloo on this one GPU (four ranks share the card).
cd "$GRAFT_REPO_ROOT" || exit 9
o=gpurun_out/r05/reh_n4; mkdir -p $o
for d in zslab rows; do
  echo "== $(date +%T) rehearsal N=4 $d"
  ASP_DIST_BACKEND=gloo timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node=4 --master-addr 127.0.0.1 --master-port 29519 bench.py --gpus 4 --steps 4 --warmup 2 --cpu-baseline off --decomp $d > $o/reh_n4_$d.json 2> $o/reh_n4_$d.err || { tail -5 $o/reh_n4_$d.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$o/reh_n4_$d.json').read().strip().splitlines()[-1]);print('$d', d['ms_per_step'], d['output_ok'], d['config']['workload'], d['config'].get('streams'), d['config'].get('scatter_gate'), d.get('partition_ms'))"
done
