# text.csv's gather forked behind the miss aggregation (MSA_TEXT_AT_AGG=1) vs at the split's read-back; configs[4] check
export TMPDIR=/tmp; D=gpurun_out/r04_t37; mkdir -p $D
timeout -k 10 600 python -u -m pytest -x -q tests/test_gpu_parity.py tests/test_gpu_split.py --timeout 300 --timeout-method thread > $D/tests.log 2>&1 || { tail -30 $D/tests.log; exit 1; }
MSA_TEXT_AT_AGG=1 timeout -k 10 600 python -u -m pytest -x -q tests/test_gpu_parity.py tests/test_gpu_split.py --timeout 300 --timeout-method thread > $D/tests_agg.log 2>&1 || { tail -30 $D/tests_agg.log; exit 1; }
bash tools/ab_env.sh r04_t37/ab "split:X=1" "agg:MSA_TEXT_AT_AGG=1" "split_b:X=1" "agg_b:MSA_TEXT_AT_AGG=1" "split_c:X=1" "agg_c:MSA_TEXT_AT_AGG=1" || exit 1
timeout -k 10 300 python -u tools/highcard_bench.py 4100000 --steps 3 > $D/hc.txt 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $D/prof -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > $D/prof.log 2>&1 && python3 tools/timeline.py $D/prof > $D/timeline.txt
echo __done__
