cd "$GRAFT_REPO_ROOT" || exit 9
for n in 100000000 50000000 25000000 12500000 6250000; do
  timeout -k 10 200 python bench.py --cpu-baseline off --quiet --steps 10 --n $n 2>/dev/null | python3 -c "import json,sys; d=json.load(sys.stdin); s=d['stages']; print($n, d['ms_per_step'], {k: round(v['ms_per_launch'],3) for k,v in s.items() if v['launches']}, 'scatter ns/particle', round(s['scatter']['ms_per_launch']*1e6/$n,4))" || exit 1
done
