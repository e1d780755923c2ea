#!/bin/bash
# same-box A/B of the cube: working build vs lib_base (tools/ab_build.sh), GPU tests first
cd "$GRAFT_REPO_ROOT" || exit 9
export TMPDIR=/tmp
o=gpurun_out/r04/${TAG:-ab_cube}
mkdir -p $o
if [ -z "$NOTEST" ]; then
  echo "== $(date +%T) tests"
  timeout -k 10 400 python -u -m pytest tests/test_gpu_cube.py tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread > $o/tests.log 2>&1 || { tail -20 $o/tests.log; exit 1; }
  tail -2 $o/tests.log
fi
for rep in 1 2; do
  for lib in new base; do
    l=""; [ $lib = base ] && l="ASP_LIB=$GRAFT_REPO_ROOT/astro-sph-tools_amd/lib_base/libasp_hip.so"
    env $l timeout -k 10 300 python bench.py --workload cube --steps 5 --cpu-baseline off ${ARGS} > $o/cube_${lib}_$rep.json 2> $o/cube_${lib}_$rep.err || { tail -5 $o/cube_${lib}_$rep.err; exit 1; }
    python -c "import json;d=json.load(open('$o/cube_${lib}_$rep.json'));print('$lib', d['ms_per_step'], d.get('output_ok'), {k:round(v['ms_per_launch'],3) for k,v in d.get('stages',{}).items()})"
  done
done
