# the ranking entries from k_list_build's dense copies of the claimed slots (MSA_DENSE_ENTRIES=0: through the lists)
export TMPDIR=/tmp; D=gpurun_out/r04_t44; mkdir -p $D
timeout -k 10 900 python -u -m pytest -x -q tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_gpu_dist.py tests/test_gpu_comp_sort.py --timeout 800 --timeout-method thread > $D/tests.log 2>&1 || { tail -30 $D/tests.log; exit 1; }
for v in dense:X=1 lists:MSA_DENSE_ENTRIES=0 dense_b:X=1 lists_b:MSA_DENSE_ENTRIES=0; do
  n=${v%%:*}; env ${v#*:} timeout -k 10 300 python -u tools/highcard_bench.py 4100000 --steps 3 > $D/hc_$n.txt 2>&1 || exit 1
  echo "$n $(tail -n 3 $D/hc_$n.txt | head -2 | tr '\n' ' ' | cut -c1-420)" >> $D/summary.txt
done
bash tools/ab_env.sh r04_t44/ab "dense:X=1" "lists:MSA_DENSE_ENTRIES=0" || exit 1
echo __done__
