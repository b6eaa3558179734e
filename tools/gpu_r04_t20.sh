# words' radix sort without K0 passes (ties refined from byte 8) + tie comparisons after k_rank_total's tile loop:
# parity (parity, scale incl. configs[4] vs oracle, sort designs), configs[2] A/B vs HEAD (prev), configs[4] with/without K0 passes
export TMPDIR=/tmp; D=gpurun_out/r04_t20; V=$PWD/music-analyst-ai_amd/variants; mkdir -p $D
timeout -k 10 300 python -u -m pytest -x -q tests/test_gpu_parity.py --timeout 200 --timeout-method thread > $D/tests.log 2>&1 || { tail -30 $D/tests.log; exit 1; }
timeout -k 10 700 python -u -m pytest -x -q tests/test_gpu_scale.py -k "highcard or configs4 or sort_designs" --timeout 600 --timeout-method thread > $D/tests_scale.log 2>&1 || { tail -30 $D/tests_scale.log; exit 1; }
bash tools/ab_env.sh r04_t20/ab "new:X=1" "prev:MSA_LIB=$V/libmsa_hip_prev.so" "new_b:X=1" "prev_b:MSA_LIB=$V/libmsa_hip_prev.so" || exit 1
timeout -k 10 300 python -u tools/highcard_bench.py 4100000 --steps 2 > $D/hc_new.txt 2>&1 || exit 1
MSA_SORT_K0=1 timeout -k 10 300 python -u tools/highcard_bench.py 4100000 --steps 2 > $D/hc_k0.txt 2>&1 || exit 1
