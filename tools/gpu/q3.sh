cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out/q3
for cfg in "1024 4" "2048 8" "2048 4" "4096 16" "512 2"; do
  set -- $cfg
  ASP_BIN_BLOCKS=$1 ASP_SCATTER_GROUP=$2 timeout -k 10 200 python bench.py --cpu-baseline off --quiet --steps 10 > gpurun_out/q3/b_$1_$2.json 2>/dev/null || { echo fail; exit 1; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/q3/b_$1_$2.json')); print('$1 $2', d['ms_per_step'], {k: round(v['ms_per_launch'],3) for k,v in d['stages'].items()})"
done
