# wave-aggregated list appends + CAS-first probes: parity subset, configs[4] stages, A/B on configs[2]
export TMPDIR=/tmp; D=gpurun_out/r04_t9; V=$PWD/music-analyst-ai_amd/variants; mkdir -p $D
timeout -k 10 400 python -u -m pytest -x -q tests/test_gpu_parity.py tests/test_gpu_dist.py --timeout 200 --timeout-method thread > $D/tests.log 2>&1 || { tail -30 $D/tests.log; exit 1; }
timeout -k 10 300 python -u tools/highcard_bench.py 4100000 --steps 2 > $D/hc_base.txt 2>&1 || exit 1
MSA_LIB=$V/libmsa_hip_loadfirst.so timeout -k 10 300 python -u tools/highcard_bench.py 4100000 --steps 2 > $D/hc_loadfirst.txt 2>&1 || exit 1
bash tools/ab_env.sh r04_t9/ab 'base:X=1' "loadfirst:MSA_LIB=$V/libmsa_hip_loadfirst.so" "bf:MSA_LIB=$V/libmsa_hip_bf.so" 'base_b:X=1' "loadfirst_b:MSA_LIB=$V/libmsa_hip_loadfirst.so" "bf_b:MSA_LIB=$V/libmsa_hip_bf.so"
