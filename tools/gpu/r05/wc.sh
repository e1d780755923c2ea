#!/bin/bash
# Round 5: scatter write-combining -- parity tests, same-process A/B (ASP_WC_SLOTS), bench.
cd "$GRAFT_REPO_ROOT" || exit 9
export TMPDIR=/tmp
o=gpurun_out/r05/${TAG:-wc}; mkdir -p $o
echo "== $(date +%T) tests"
timeout -k 10 900 python -u -m pytest ${TESTS:-tests/test_gpu_parity.py tests/test_gpu_fp64.py tests/test_gpu_configs.py} -m gpu -x -q --timeout 300 --timeout-method thread > $o/tests.log 2>&1 || { tail -30 $o/tests.log; exit 1; }
tail -1 $o/tests.log
echo "== $(date +%T) A/B"
timeout -k 10 300 python -u tools/scatter_ab.py ASP_WC_SLOTS=0 ASP_WC_SLOTS=352 ASP_WC_SLOTS=128 > $o/ab.log 2>&1 || { tail -20 $o/ab.log; exit 2; }
cat $o/ab.log
echo "== $(date +%T) bench"
timeout -k 10 300 python bench.py --cpu-baseline off > $o/bench.json 2> $o/bench.err || { tail -5 $o/bench.err; exit 3; }
python3 -c "import json;d=json.load(open('$o/bench.json'));print(d['ms_per_step'], d['output_ok'], d['roofline']['kernel'], d['roofline']['frac'], {k:round(v['ms_per_step'],3) for k,v in d['stages'].items()})"
