#!/bin/bash
# Round 6: where the scatter's time goes on the current build -- production vs
# ASP_SCATTER_ABLATE=1 (no record stores) vs 2 (no stores, no cursor atomics); the ablated
# builds' deposit kernels return at once, so their lines fail the output check (exit 3,
# ignored here: only the stage times are read).
cd "$GRAFT_REPO_ROOT" || exit 9
o=gpurun_out/r06/t9; mkdir -p $o
S="--steps 20 --cpu-baseline off --overlap-streams 0"
for r in 1 2; do
  for v in prod abl1 abl2; do
    lib=astro-sph-tools_amd/lib/libasp_hip.so; [ $v != prod ] && lib=astro-sph-tools_amd/ab_$v/libasp_hip.so
    ASP_LIB=$lib timeout -k 10 300 python bench.py $S > $o/${v}_$r.json 2> $o/${v}_$r.err
    rc=$?; [ $rc -ne 0 ] && [ $rc -ne 3 ] && { echo "$v rc=$rc"; tail -3 $o/${v}_$r.err; exit 1; }
    python3 -c "import json;d=json.loads(open('$o/${v}_$r.json').read().strip().splitlines()[-1]);print('$v', $r, d['ms_per_step'], {k:round(x['ms_per_launch'],4) for k,x in d['stages'].items()})"
  done
done
