cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/q
for n in 12500000 100000000; do
for f in "" "--no-stage-events"; do
timeout -k 10 200 python bench.py --cpu-baseline off --quiet --n $n --steps 20 $f > gpurun_out/q/ev.json 2>gpurun_out/q/ev.err || { tail -3 gpurun_out/q/ev.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/q/ev.json')); print($n, '$f', d['ms_per_step'])"
done; done
