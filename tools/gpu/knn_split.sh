cd "$GRAFT_REPO_ROOT" || exit 9
for d in 0 1; do
  ASP_KNN_DIAG=$d timeout -k 10 200 python bench.py --workload knn --n 10000000 --cpu-baseline off --steps 3 --warmup 1 2>/dev/null | python3 -c "import json,sys; d=json.load(sys.stdin); print('diag $d', d['ms_per_step'], {k: round(v['ms_per_launch'],3) for k,v in d.get('stages',{}).items()})"
done
