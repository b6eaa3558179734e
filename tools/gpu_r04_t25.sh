# text gather forked at the split's read-back (MSA_TEXT_AT_SPLIT=1) vs forked by msa_count: parity with it on, A/B, trace
export TMPDIR=/tmp; D=gpurun_out/r04_t25; mkdir -p $D
MSA_TEXT_AT_SPLIT=1 timeout -k 10 400 python -u -m pytest -x -q tests/test_gpu_parity.py tests/test_gpu_split.py tests/test_gpu_dist.py --timeout 200 --timeout-method thread > $D/tests.log 2>&1 || { tail -30 $D/tests.log; exit 1; }
bash tools/ab_env.sh r04_t25/ab "at_split:MSA_TEXT_AT_SPLIT=1" "base:X=1" "at_split_b:MSA_TEXT_AT_SPLIT=1" "base_b:X=1" "at_split_c:MSA_TEXT_AT_SPLIT=1" "base_c:X=1" || exit 1
MSA_TEXT_AT_SPLIT=1 timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $D/prof -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > $D/prof.log 2>&1 && python3 tools/timeline.py $D/prof > $D/timeline.txt
