# words' composite radix key (MSA_COMP_SORT=0: the K2/K1 sort), pipelined ghist, staged key blob, whole-table clears:
# parity (new width cases + radix-forced designs + configs[4] run), configs[4] A/B, kernel trace
export TMPDIR=/tmp; D=gpurun_out/r04_t32; mkdir -p $D
timeout -k 10 900 python -u -m pytest -x -v tests/test_gpu_comp_sort.py tests/test_gpu_scale.py tests/test_gpu_parity.py -k "comp_sort or sort_designs or configs4_run or torture or golden" --timeout 800 --timeout-method thread > $D/tests.log 2>&1 || { tail -30 $D/tests.log; exit 1; }
for v in comp:X=1 k2k1:MSA_COMP_SORT=0 comp_b:X=1; do
  n=${v%%:*}; env ${v#*:} timeout -k 10 300 python -u tools/highcard_bench.py 4100000 --steps 3 > $D/hc_$n.txt 2>&1 || exit 1
  echo "$n $(tail -n 3 $D/hc_$n.txt | head -2 | tr '\n' ' ' | cut -c1-500)" >> $D/summary.txt
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $D/prof_hc -o run -- python3 tools/highcard_bench.py 4100000 --steps 2 > $D/prof_hc.log 2>&1 && python3 tools/timeline.py $D/prof_hc > $D/timeline_hc.txt
echo __done__
