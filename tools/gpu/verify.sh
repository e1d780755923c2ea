cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out/v
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/v/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/v/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/v/smoke.log 2>&1 || exit $?
cat gpurun_out/v/smoke.log
timeout -k 10 300 python bench.py > gpurun_out/v/bench.json 2> gpurun_out/v/bench.err || exit $?
cut -c1-400 gpurun_out/v/bench.json
