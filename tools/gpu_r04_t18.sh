# token pass with a full-rate partition hash (no 64-bit multiplies) + K1 change, vs HEAD's kernels (prev): parity subset, configs[2] A/B
export TMPDIR=/tmp; D=gpurun_out/r04_t18; V=$PWD/music-analyst-ai_amd/variants; mkdir -p $D
timeout -k 10 400 python -u -m pytest -x -q tests/test_gpu_parity.py tests/test_gpu_dist.py --timeout 200 --timeout-method thread > $D/tests.log 2>&1 || { tail -30 $D/tests.log; exit 1; }
bash tools/ab_env.sh r04_t18/ab "new:X=1" "prev:MSA_LIB=$V/libmsa_hip_prev.so" "new_b:X=1" "prev_b:MSA_LIB=$V/libmsa_hip_prev.so" "new_c:X=1" "prev_c:MSA_LIB=$V/libmsa_hip_prev.so" || exit 1
