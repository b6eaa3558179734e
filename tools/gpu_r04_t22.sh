# text gather with a byte slot map (9 KiB LDS per workgroup) [new], + 8 workgroups per CU (<= 64 VGPRs) [w8], vs HEAD [prev]
export TMPDIR=/tmp; D=gpurun_out/r04_t22; V=$PWD/music-analyst-ai_amd/variants; mkdir -p $D
timeout -k 10 400 python -u -m pytest -x -q tests/test_gpu_parity.py tests/test_gpu_split.py --timeout 200 --timeout-method thread > $D/tests.log 2>&1 || { tail -30 $D/tests.log; exit 1; }
MSA_LIB=$V/libmsa_hip_w8.so timeout -k 10 300 python -u -m pytest -x -q tests/test_gpu_parity.py -k "torture or medium or golden or edge" --timeout 200 --timeout-method thread > $D/tests_w8.log 2>&1 || { tail -30 $D/tests_w8.log; exit 1; }
bash tools/ab_env.sh r04_t22/ab "new:X=1" "w8:MSA_LIB=$V/libmsa_hip_w8.so" "prev:MSA_LIB=$V/libmsa_hip_prev.so" "new_b:X=1" "w8_b:MSA_LIB=$V/libmsa_hip_w8.so" "prev_b:MSA_LIB=$V/libmsa_hip_prev.so" || exit 1
