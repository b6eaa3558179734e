# text.csv early (LDS-free gather beside the token pass): parity, A/B vs deferred, configs[4] trace
export TMPDIR=/tmp; D=gpurun_out/r04_t13; mkdir -p $D
timeout -k 10 300 python -u -m pytest -x -q tests/test_gpu_parity.py tests/test_gpu_split.py --timeout 200 --timeout-method thread > $D/tests.log 2>&1 || { tail -30 $D/tests.log; exit 1; }
bash tools/ab_env.sh r04_t13/ab 'early:X=1' 'deferred:MSA_EARLY_TEXT=0' 'early_b:X=1' 'deferred_b:MSA_EARLY_TEXT=0' || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $D/prof1 -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > $D/prof1.log 2>&1 || exit 1
python3 tools/timeline.py $D/prof1 > $D/timeline.txt
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $D/prof -o run -- python3 tools/highcard_bench.py 4100000 --steps 2 > $D/hc.txt 2>&1 || exit 1
