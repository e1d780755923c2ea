#!/bin/bash
# same-box A/B of one bench line: working build vs lib_base (tools/ab_build.sh).
#   ARGS="--n 10000000 ..." TESTS="tests/test_gpu_x.py ..." bash tools/gpu/r04/ab_bench.sh
cd "$GRAFT_REPO_ROOT" || exit 9
export TMPDIR=/tmp
o=gpurun_out/r04/${TAG:-ab_bench}
mkdir -p $o
if [ -n "$TESTS" ]; then
  echo "== $(date +%T) tests"
  timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -q --timeout 300 --timeout-method thread > $o/tests.log 2>&1 || { tail -30 $o/tests.log; exit 1; }
  tail -2 $o/tests.log
fi
for rep in 1 2; do
  for lib in new base; do
    l=""; [ $lib = base ] && l="ASP_LIB=$GRAFT_REPO_ROOT/astro-sph-tools_amd/lib_base/libasp_hip.so"
    env $l timeout -k 10 300 python bench.py --cpu-baseline off $ARGS > $o/${lib}_$rep.json 2> $o/${lib}_$rep.err || { tail -5 $o/${lib}_$rep.err; exit 1; }
    python -c "import json;d=json.load(open('$o/${lib}_$rep.json'));print('$lib', d['ms_per_step'], d.get('output_ok'), {k:round(v['ms_per_step'],3) for k,v in d.get('stages',{}).items()})"
  done
done
