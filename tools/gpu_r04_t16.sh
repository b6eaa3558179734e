# k_miss_agg flush-and-reset of a full LDS table (default) vs an HBM insert per entry (maold): parity, configs[2] A/B, configs[4]
export TMPDIR=/tmp; D=gpurun_out/r04_t16; V=$PWD/music-analyst-ai_amd/variants; mkdir -p $D
timeout -k 10 400 python -u -m pytest -x -q tests/test_gpu_parity.py --timeout 200 --timeout-method thread > $D/tests.log 2>&1 || { tail -30 $D/tests.log; exit 1; }
timeout -k 10 600 python -u -m pytest -x -q tests/test_gpu_scale.py -k "highcard_overflows or configs4_run" --timeout 500 --timeout-method thread > $D/tests_scale.log 2>&1 || { tail -30 $D/tests_scale.log; exit 1; }
bash tools/ab_env.sh r04_t16/ab "flush:X=1" "maold:MSA_LIB=$V/libmsa_hip_maold.so" "flush_b:X=1" "maold_b:MSA_LIB=$V/libmsa_hip_maold.so" || exit 1
timeout -k 10 300 python -u tools/highcard_bench.py 4100000 --steps 2 > $D/hc_flush.txt 2>&1 || exit 1
MSA_LIB=$V/libmsa_hip_maold.so timeout -k 10 300 python -u tools/highcard_bench.py 4100000 --steps 2 > $D/hc_maold.txt 2>&1 || exit 1
