#!/bin/bash
# Round-4: full GPU suite, N = 2 / 4 rehearsals over gloo on one GPU (both decompositions).
cd "$GRAFT_REPO_ROOT" || exit 9
export TMPDIR=/tmp
o=gpurun_out/r04/${TAG:-run4}
mkdir -p $o
echo "== $(date +%T) pytest"
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf > $o/gputest.log 2>&1; rc=$?; tail -6 $o/gputest.log
[ $rc -le 1 ] || exit $rc
for cfg in "2 rows dst" "2 rows all" "2 zslab dst" "4 rows all" "4 zslab dst"; do
  set -- $cfg
  echo "== $(date +%T) rehearsal N=$1 $2 $3"
  ASP_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $1 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus $1 --steps 5 --warmup 2 --decomp $2 --rows-gather $3 > $o/reh_n$1_$2_$3.json 2> $o/reh_n$1_$2_$3.err; echo "rc=$?"
  grep -v "Gloo\|socket.cpp\|amdgpu.ids\|data ready" $o/reh_n$1_$2_$3.err | tail -3 | cut -c1-300
  python -c "import json;d=json.load(open('$o/reh_n$1_$2_$3.json'));print(d['ms_per_step'], d['output_ok'], d['config']['workload'], d['roofline']['kernel'], d['roofline']['frac'])" 2>/dev/null
done
echo "== $(date +%T) done"
