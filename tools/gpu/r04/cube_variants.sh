#!/bin/bash
# cube deposit: compile-time class variants (lib_vA/vB/vC, tools/ab_build.sh) against the working build
cd "$GRAFT_REPO_ROOT" || exit 9
export TMPDIR=/tmp
o=gpurun_out/r04/cube_variants; mkdir -p $o
for rep in 1 2; do for lib in new vA vB vC; do
  l=""; [ $lib != new ] && l="ASP_LIB=$GRAFT_REPO_ROOT/astro-sph-tools_amd/lib_$lib/libasp_hip.so"
  env $l timeout -k 10 300 python bench.py --workload cube --steps 5 --cpu-baseline off > $o/${lib}_$rep.json 2> $o/${lib}_$rep.err || { tail -5 $o/${lib}_$rep.err; exit 1; }
  python -c "import json;d=json.load(open('$o/${lib}_$rep.json'));print('$lib', d['ms_per_step'], d.get('output_ok'), round(d['stages']['cube_deposit']['ms_per_launch'],3))"
done; done
