# direct miss stores (one buffer store per probe batch, fixed VMEM sequence) vs the LDS miss buffer (tokbuf):
# parity incl. log overflow + retry, configs[2] A/B, configs[4] stages
export TMPDIR=/tmp; D=gpurun_out/r04_t15; V=$PWD/music-analyst-ai_amd/variants; mkdir -p $D
timeout -k 10 400 python -u -m pytest -x -q tests/test_gpu_parity.py tests/test_gpu_dist.py tests/test_gpu_split.py --timeout 200 --timeout-method thread > $D/tests.log 2>&1 || { tail -30 $D/tests.log; exit 1; }
bash tools/ab_env.sh r04_t15/ab "direct:X=1" "tokbuf:MSA_LIB=$V/libmsa_hip_tokbuf.so" "nok1:MSA_ABLATE=16384" "direct_b:X=1" "tokbuf_b:MSA_LIB=$V/libmsa_hip_tokbuf.so" "nok1_b:MSA_ABLATE=16384" || exit 1
timeout -k 10 300 python -u tools/highcard_bench.py 4100000 --steps 2 > $D/hc_direct.txt 2>&1 || exit 1
MSA_LIB=$V/libmsa_hip_tokbuf.so timeout -k 10 300 python -u tools/highcard_bench.py 4100000 --steps 2 > $D/hc_tokbuf.txt 2>&1 || exit 1
