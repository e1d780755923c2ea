#!/bin/bash
# One parameterised GPU step per call (chain calls with && inside one gpurun command).
# Output under gpurun_out/$OUT/ (default r05).  Every GPU step runs under its own timeout.
#   bash tools/gpu/run.sh suite                       pytest -m gpu (all) + smoke()
#   bash tools/gpu/run.sh tests FILE...               pytest -m gpu on some files
#   bash tools/gpu/run.sh bench NAME [bench args]     one bench.py line -> NAME.json
#   bash tools/gpu/run.sh sweep VAR "V1 V2" NAME [bench args]
#                                                     one line per VAR=Vi -> NAME_Vi.json
#   bash tools/gpu/run.sh reps N NAME [bench args]    N fresh processes -> NAME_i.json
#   bash tools/gpu/run.sh prof TAG [prof_driver args] kernel trace + PMC passes (prof_full.sh)
#   bash tools/gpu/run.sh ab NAME "LIBS" REPS [bench args]
#                                                     same-box A/B: REPS rounds, each running one
#                                                     line per build in LIBS ("work" = the working
#                                                     library, X = astro-sph-tools_amd/ab_X/, from
#                                                     tools/ab_build.sh) -> NAME_<lib>_<rep>.json
#   bash tools/gpu/run.sh trace NAME [bench args]     rocprofv3 kernel trace of one bench line ->
#                                                     NAME/, per-stream and timeline summaries
#   bash tools/gpu/run.sh cube_ab NAME 'ENV=A' ...    tools/cube_ab.py: same-process cube A/B of
#                                                     environment settings -> NAME.log
# Every per-round script of rounds 3-6 was an instance of these modes; tools/gpu/README.md
# lists the command line of each measurement kept under profiles/.
cd "$GRAFT_REPO_ROOT" || exit 9
export TMPDIR=/tmp
o=gpurun_out/${OUT:-r06}; mkdir -p $o
mode=$1; shift
summ() {  # name: ms, output check, dominant kernel, frac, per-stage ms
  python3 -c "import json,sys;d=json.loads(open('$o/$1.json').read().strip().splitlines()[-1]);r=d.get('roofline',{});print('$1', d['ms_per_step'], d.get('output_ok'), r.get('kernel'), r.get('frac'), 'ovl', (d.get('overlapped') or {}).get('ms_per_step'), (d.get('overlapped') or {}).get('output_ok'), {k:round(v.get('ms_per_step', v.get('ms_per_launch', 0)),3) for k,v in d.get('stages',{}).items()})"
}
line() {  # name args...
  local name=$1; shift
  echo "== $(date +%T) $name: $*"
  timeout -k 10 ${LIMIT:-300} python bench.py "$@" > $o/$name.json 2> $o/$name.err || { tail -5 $o/$name.err; return 1; }
  summ $name
}
case $mode in
  suite)
    echo "== $(date +%T) gpu suite"
    timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/gputest.log 2>&1 || { tail -40 $o/gputest.log; exit 1; }
    tail -1 $o/gputest.log
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || { tail -5 $o/smoke.log; exit 2; }
    tail -1 $o/smoke.log ;;
  tests)
    echo "== $(date +%T) tests $*"
    timeout -k 10 ${LIMIT:-900} python -u -m pytest "$@" -m gpu -x -q --timeout 300 --timeout-method thread > $o/tests.log 2>&1 || { tail -40 $o/tests.log; exit 1; }
    tail -1 $o/tests.log ;;
  bench)
    line "$@" || exit 3 ;;
  sweep)
    var=$1; vals=$2; name=$3; shift 3
    for v in $vals; do export "$var=$v"; line ${name}_$v "$@" || exit 3; done ;;
  reps)
    n=$1; name=$2; shift 2
    for i in $(seq 1 $n); do line ${name}_$i "$@" || exit 3; done ;;
  prof)
    bash tools/gpu/prof_full.sh "$@" || exit 4 ;;
  ab)
    name=$1; libs=$2; reps=$3; shift 3
    for r in $(seq 1 $reps); do
      for l in $libs; do
        if [ "$l" = work ]; then lib=astro-sph-tools_amd/lib/libasp_hip.so; else lib=astro-sph-tools_amd/ab_$l/libasp_hip.so; fi
        ASP_LIB=$lib line ${name}_${l}_$r "$@" || exit 5
      done
    done ;;
  trace)
    name=$1; shift
    echo "== $(date +%T) trace $name: $*"
    timeout -k 10 ${LIMIT:-300} rocprofv3 --kernel-trace --stats --output-format csv -d $o/$name -o kt -- python3 bench.py "$@" > $o/$name.json 2> $o/$name.err || { tail -5 $o/$name.err; exit 6; }
    python3 tools/stream_phase.py $o/$name/kt_kernel_trace.csv > $o/${name}_streams.txt
    python3 tools/timeline.py $o/$name/kt_kernel_trace.csv > $o/${name}_timeline.txt
    tail -1 $o/${name}_timeline.txt ;;
  cube_ab)
    name=$1; shift
    echo "== $(date +%T) cube_ab $name: $*"
    timeout -k 10 ${LIMIT:-400} python tools/cube_ab.py "$@" > $o/$name.log 2>&1 || { tail -20 $o/$name.log; exit 7; }
    grep "rep 1" $o/$name.log ;;
  *) echo "unknown mode $mode"; exit 8 ;;
esac
