# k-NN bench (10^7) for each library directory given: bash tools/gpu/knn_ab.sh <libdir>...
cd "$GRAFT_REPO_ROOT" || exit 9
for L in "$@"; do
  ASP_LIB=$PWD/$L/libasp_hip.so timeout -k 10 200 python bench.py --workload knn --n 10000000 --cpu-baseline off --steps 3 --warmup 1 2>/dev/null | python3 -c "import json,sys; d=json.load(sys.stdin); print('$L', d['ms_per_step'])" || exit 1
done
