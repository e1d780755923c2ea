#!/bin/bash
# A/B of library builds on one box, then a GPU test pass with the product build:
#   bash tools/gpu/ab_run.sh <bench args> -- <libdir>...
cd "$GRAFT_REPO_ROOT" || exit 9
args=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do args+=("$1"); shift; done; shift
for rep in ${REPS:-1 2}; do
  for L in "$@"; do
    ASP_LIB=$PWD/$L/libasp_hip.so timeout -k 10 200 python bench.py --cpu-baseline off --quiet --steps 10 "${args[@]}" 2>/dev/null | python3 -c "import json,sys; d=json.load(sys.stdin); print('$L', d['ms_per_step'], d.get('output_ok'), {k: round(v['ms_per_launch'],3) for k,v in d.get('stages', {}).items() if v['launches']})" || exit 1
  done
done
