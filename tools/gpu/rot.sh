#!/bin/bash
# GPU parity suite, then alloc_probe (6 placements of the record buffer) for two builds.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out/rot
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/rot/pytest.log 2>&1
rc=$?; tail -2 gpurun_out/rot/pytest.log; [ $rc -ne 0 ] && exit $rc
for v in base ${1:-ASP_ROTATE0}; do
  lib=astro-sph-tools_amd/lib/libasp_hip.so
  [ "$v" != base ] && lib=astro-sph-tools_amd/lib/libasp_hip_$v.so
  ASP_LIB=$PWD/$lib NOSHIFT=1 TRIALS=6 timeout -k 10 200 python tools/alloc_probe.py ${2:-100000000} > gpurun_out/rot/$v.log 2>&1 || exit $?
  echo "== $v"; grep trial gpurun_out/rot/$v.log | cut -c1-140
done
