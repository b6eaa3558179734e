# text gather: two-line slots composed by one mask select (vs the line loop in HEAD = prev): parity, configs[2] A/B + trace
export TMPDIR=/tmp; D=gpurun_out/r04_t21; V=$PWD/music-analyst-ai_amd/variants; mkdir -p $D
timeout -k 10 400 python -u -m pytest -x -q tests/test_gpu_parity.py tests/test_gpu_split.py tests/test_gpu_dist.py --timeout 200 --timeout-method thread > $D/tests.log 2>&1 || { tail -30 $D/tests.log; exit 1; }
bash tools/ab_env.sh r04_t21/ab "new:X=1" "prev:MSA_LIB=$V/libmsa_hip_prev.so" "new_b:X=1" "prev_b:MSA_LIB=$V/libmsa_hip_prev.so" "new_c:X=1" "prev_c:MSA_LIB=$V/libmsa_hip_prev.so" || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $D/prof -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > $D/prof.log 2>&1 && python3 tools/timeline.py $D/prof > $D/timeline.txt
