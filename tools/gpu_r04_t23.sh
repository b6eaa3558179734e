# artist count at the end of the split (before its read-back) + text gather forked before the long words: parity (all API flows), A/B vs HEAD, trace
export TMPDIR=/tmp; D=gpurun_out/r04_t23; V=$PWD/music-analyst-ai_amd/variants; mkdir -p $D
timeout -k 10 600 python -u -m pytest -x -q tests/test_gpu_parity.py tests/test_gpu_split.py tests/test_gpu_dist.py tests/test_gpu_cli.py --timeout 300 --timeout-method thread > $D/tests.log 2>&1 || { tail -30 $D/tests.log; exit 1; }
bash tools/ab_env.sh r04_t23/ab "new:X=1" "prev:MSA_LIB=$V/libmsa_hip_prev.so" "new_b:X=1" "prev_b:MSA_LIB=$V/libmsa_hip_prev.so" "new_c:X=1" "prev_c:MSA_LIB=$V/libmsa_hip_prev.so" || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $D/prof -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > $D/prof.log 2>&1 && python3 tools/timeline.py $D/prof > $D/timeline.txt
