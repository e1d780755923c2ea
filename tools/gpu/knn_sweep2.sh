cd "$GRAFT_REPO_ROOT" || exit 9
for w in ${KNN_W:-64 128 192}; do for f in ${KNN_F:-0 1 2}; do
  ASP_KNN_WINDOW=$w ASP_KNN_FINE=$f timeout -k 10 200 python bench.py --workload knn --n 10000000 --cpu-baseline off --steps 3 --warmup 1 2>/dev/null | python3 -c "import json,sys; d=json.load(sys.stdin); print('W $w fine $f', d['ms_per_step'])"
done; done
