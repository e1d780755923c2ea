#!/bin/bash
# cube: batch-interleaved count / scatter (ASP_CUBE_INTERLEAVE 1) vs contiguous (0), same box
cd "$GRAFT_REPO_ROOT" || exit 9
export TMPDIR=/tmp
o=gpurun_out/r04/cube_inter; mkdir -p $o
timeout -k 10 400 python -u -m pytest tests/test_gpu_cube.py tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread > $o/tests.log 2>&1 || { tail -20 $o/tests.log; exit 1; }
tail -1 $o/tests.log
for rep in 1 2; do for v in 1 0; do
  ASP_CUBE_INTERLEAVE=$v timeout -k 10 300 python bench.py --workload cube --steps 5 --cpu-baseline off > $o/cube_${v}_$rep.json 2> $o/cube_${v}_$rep.err || { tail -5 $o/cube_${v}_$rep.err; exit 1; }
  python -c "import json;d=json.load(open('$o/cube_${v}_$rep.json'));print('inter $v', d['ms_per_step'], d.get('output_ok'), {k:round(v['ms_per_launch'],3) for k,v in d.get('stages',{}).items()})"
done; done
