# Scatter placement mode vs the record buffer's address, over fresh processes.
cd "$GRAFT_REPO_ROOT" || exit 9
for i in 1 2 3 4 5 6 7 8; do
  ASP_PRINT_ALLOC=1 timeout -k 10 120 python -u tools/scatter_ab.py ASP_SCATTER_GROUP=4 > gpurun_out/mp_$i.out 2> gpurun_out/mp_$i.err || exit 1
  echo "$i $(grep -o "'scatter': [0-9.]*" gpurun_out/mp_$i.out | head -1) $(sort -k3 -n gpurun_out/mp_$i.err | grep 'asp alloc' | sort -t' ' -k3 -n | tail -1)"
done
