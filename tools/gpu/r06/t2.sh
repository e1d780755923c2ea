#!/bin/bash
# Round 6: the single-pass binning experiment (ASP_SP_EXPERIMENT=1: SP scatter + chunk-list
# finalize, stage events) and kernel traces of the default bench with and without the
# scatter gate (the overlapped region's alternating scatter durations).
cd "$GRAFT_REPO_ROOT" || exit 9
export OUT=r06/t2 TMPDIR=/tmp
o=gpurun_out/$OUT; mkdir -p $o
ASP_SP_EXPERIMENT=1 bash tools/gpu/run.sh bench bench_sp --overlap-streams 0 || exit 1
grep "SP experiment" $o/bench_sp.err | head -5
bash tools/gpu/run.sh bench bench_base --overlap-streams 0 || exit 2
for gate in 0 1; do
  ASP_SCATTER_GATE=$gate timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $o/kt_gate$gate -o kt -- python3 bench.py > $o/kt_gate$gate.json 2> $o/kt_gate$gate.err || exit 3
  echo "gate $gate: $(tail -c 300 $o/kt_gate$gate.json)"
done
