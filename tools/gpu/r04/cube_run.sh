#!/bin/bash
# cube: GPU tests, then the 512^3 bench (twice)
cd "$GRAFT_REPO_ROOT" || exit 9
export TMPDIR=/tmp
o=gpurun_out/r04/${TAG:-cube_run}
mkdir -p $o
echo "== $(date +%T) tests"
timeout -k 10 400 python -u -m pytest tests/test_gpu_cube.py tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread > $o/tests.log 2>&1 || { tail -20 $o/tests.log; exit 1; }
tail -2 $o/tests.log
for rep in 1 2; do
  echo "== $(date +%T) bench $rep"
  timeout -k 10 300 python bench.py --workload cube --steps 5 --cpu-baseline off > $o/cube_$rep.json 2> $o/cube_$rep.err || { tail -5 $o/cube_$rep.err; exit 1; }
  python -c "import json;d=json.load(open('$o/cube_$rep.json'));print('cube', d['ms_per_step'], d.get('output_ok'), {k:round(v['ms_per_launch'],3) for k,v in d.get('stages',{}).items()})"
done
