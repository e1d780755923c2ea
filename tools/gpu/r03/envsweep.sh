#!/bin/bash
# Same-box sweep of the headline map under run-time switches: one bench line per variant
# (gpurun_out/r03/$TAG/<i>_<name>.json), then the stage table.  $VARIANTS: "name:VAR=x,VAR2=y ...";
# $BENCH_ARGS: extra bench.py arguments (default: the headline workload).
cd "$GRAFT_REPO_ROOT" || exit 9
o=gpurun_out/r03/${TAG:-sweep}
mkdir -p $o
files=(); i=0
for v in $VARIANTS; do
  i=$((i+1)); name=${v%%:*}; envs=${v#*:}; [ "$envs" = "$v" ] && envs=""
  f=$o/${i}_$name
  env ${envs//,/ } timeout -k 10 240 python bench.py --cpu-baseline off $BENCH_ARGS > $f.json 2> $f.err
  rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || { tail -5 $f.err; exit $rc; }
  files+=($f.json)
done
python tools/stages.py "${files[@]}"
