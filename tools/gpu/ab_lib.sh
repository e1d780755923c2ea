# A/B of library builds on one box: bash tools/gpu/ab_lib.sh <libdir>... (cfg3 bench each, twice)
cd "$GRAFT_REPO_ROOT" || exit 9
for rep in 1 2; do
  for L in "$@"; do
    ASP_LIB=$PWD/$L/libasp_hip.so timeout -k 10 200 python bench.py --cpu-baseline off --quiet --steps 10 2>/dev/null | python3 -c "import json,sys; d=json.load(sys.stdin); print('$L', d['ms_per_step'], {k: round(v['ms_per_launch'],3) for k,v in d['stages'].items()})" || exit 1
  done
done
