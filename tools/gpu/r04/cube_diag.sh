#!/bin/bash
# cube deposit split: ASP_CUBE_DIAG 0 (full), 1 (lane classes only), 2 (wave class only)
cd "$GRAFT_REPO_ROOT" || exit 9
export TMPDIR=/tmp
o=gpurun_out/r04/${TAG:-cube_diag}
mkdir -p $o
for v in ${DIAGS:-0 1 2}; do
  echo "== $(date +%T) diag=$v"
  ASP_CUBE_DIAG=$v timeout -k 10 300 python bench.py --workload cube --steps 5 --cpu-baseline off > $o/cube_$v.json 2> $o/cube_$v.err || [ $? -eq 3 ] || { tail -5 $o/cube_$v.err; exit 1; }
  python -c "import json;d=json.load(open('$o/cube_$v.json'));print('diag $v', d['ms_per_step'], d.get('output_ok'), {k:round(v['ms_per_step'],3) for k,v in d.get('stages',{}).items()})"
done
