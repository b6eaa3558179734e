# scan top with batched loads (size-dependent block); text gather with 3 slots per thread per batch (variant)
export TMPDIR=/tmp; D=gpurun_out/r04_t43; V=$PWD/music-analyst-ai_amd/variants; mkdir -p $D
timeout -k 10 600 python -u -m pytest -x -q tests/test_gpu_parity.py tests/test_gpu_comp_sort.py --timeout 300 --timeout-method thread > $D/tests.log 2>&1 || { tail -30 $D/tests.log; exit 1; }
MSA_LIB=$V/libmsa_hip_cgb3.so timeout -k 10 600 python -u -m pytest -x -q tests/test_gpu_parity.py --timeout 300 --timeout-method thread > $D/tests_cgb3.log 2>&1 || { tail -30 $D/tests_cgb3.log; exit 1; }
bash tools/ab_env.sh r04_t43/ab "base:X=1" "cgb3:MSA_LIB=$V/libmsa_hip_cgb3.so" "base_b:X=1" "cgb3_b:MSA_LIB=$V/libmsa_hip_cgb3.so" "base_c:X=1" "cgb3_c:MSA_LIB=$V/libmsa_hip_cgb3.so" || exit 1
timeout -k 10 300 python -u tools/highcard_bench.py 4100000 --steps 3 > $D/hc.txt 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $D/prof -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > $D/prof.log 2>&1 && python3 tools/timeline.py $D/prof > $D/timeline.txt
echo __done__
