#!/bin/bash
# Round-4 quick iteration: selected bench lines (BENCHES env: space-separated names).
cd "$GRAFT_REPO_ROOT" || exit 9
export TMPDIR=/tmp
o=gpurun_out/r04/${TAG:-iter}
mkdir -p $o
step() { echo "== $(date +%T) $*"; }
run() {  # name args...   (LIB=dir: ASP_LIB=astro-sph-tools_amd/dir/libasp_hip.so)
  local name=$1; shift
  step "$name: $*"
  local lib=""; [ -n "$LIB" ] && lib="ASP_LIB=$GRAFT_REPO_ROOT/astro-sph-tools_amd/$LIB/libasp_hip.so"
  env $lib timeout -k 10 300 python bench.py --cpu-baseline off "$@" > $o/$name.json 2> $o/$name.err
  local rc=$?
  [ $rc -eq 0 ] || [ $rc -eq 3 ] || { tail -5 $o/$name.err; return 1; }  # 3: output check failed
  python -c "import json;d=json.load(open('$o/$name.json'));print('$name', d['ms_per_step'], d.get('latency_ms_per_map'), d['output_ok'], d['roofline']['kernel'], d['roofline']['frac'], {k:round(v['ms_per_step'],4) for k,v in d['stages'].items()})"
}
for b in ${BENCHES:-head}; do
  case $b in
    head) run head ;;
    head1) run head1 --streams 1 ;;
    det) run det --deterministic ;;
    det1) run det1 --deterministic --streams 1 ;;
    shard) run shard --n 12500000 --steps 30 ;;
    shard1) run shard1 --n 12500000 --steps 30 --streams 1 ;;
    cfg2p) run cfg2p --n 10000000 --grid 2048 --kernel cubic --map surface --h-law physical ;;
    cfg2p1) run cfg2p1 --n 10000000 --grid 2048 --kernel cubic --map surface --h-law physical --streams 1 ;;
    cfg2) run cfg2 --n 10000000 --grid 2048 --kernel cubic --map surface ;;
    cfg2p_r03) LIB=lib_r03 run cfg2p_r03 --n 10000000 --grid 2048 --kernel cubic --map surface --h-law physical ;;
    head_r03) LIB=lib_r03 run head_r03 ;;
    shard_r03) LIB=lib_r03 run shard_r03 --n 12500000 --steps 30 --streams 1 ;;
    rows8) run rows8 --n 12500000 --steps 30 ;;
    cube) run cube --workload cube --steps 5 ;;
    knn) run knn --workload knn --n 10000000 --steps 3 --warmup 1 ;;
    *) echo "unknown $b" ;;
  esac || exit 1
done
step done
