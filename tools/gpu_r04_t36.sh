# bucketed miss aggregation (MSA_MISS_BUCKETS: auto/forced/off) + composite final loads + growth policy
export TMPDIR=/tmp; D=gpurun_out/r04_t36; mkdir -p $D
timeout -k 10 900 python -u -m pytest -x -q tests/test_gpu_miss_buckets.py tests/test_gpu_comp_sort.py tests/test_gpu_scale.py -k "miss_buckets or comp_sort or sort_designs or configs4_run" --timeout 800 --timeout-method thread > $D/tests.log 2>&1 || { tail -30 $D/tests.log; exit 1; }
for v in auto:X=1 off:MSA_MISS_BUCKETS=0 auto_s1m2:MSA_GROW_MUL=2,MSA_GROW_STEP=1 auto_b:X=1 off_b:MSA_MISS_BUCKETS=0; do
  n=${v%%:*}; env $(echo ${v#*:} | tr ',' ' ') timeout -k 10 300 python -u tools/highcard_bench.py 4100000 --steps 3 > $D/hc_$n.txt 2>&1 || exit 1
  echo "$n $(tail -n 3 $D/hc_$n.txt | head -2 | tr '\n' ' ' | cut -c1-500)" >> $D/summary.txt
done
bash tools/ab_env.sh r04_t36/ab "base:X=1" "mb1:MSA_MISS_BUCKETS=1" "base_b:X=1" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $D/prof_hc -o run -- python3 tools/highcard_bench.py 4100000 --steps 2 > $D/prof_hc.log 2>&1 && python3 tools/timeline.py $D/prof_hc > $D/timeline_hc.txt
echo __done__
