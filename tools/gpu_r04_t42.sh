# half-size artist count tables (AC_SLOTS 3072: room for gather workgroups on the CU) with the gather forked
# behind the miss aggregation (MSA_TEXT_AT_AGG=1), against the default
export TMPDIR=/tmp; D=gpurun_out/r04_t42; V=$PWD/music-analyst-ai_amd/variants; mkdir -p $D
MSA_LIB=$V/libmsa_hip_ac3k.so timeout -k 10 600 python -u -m pytest -x -q tests/test_gpu_parity.py --timeout 300 --timeout-method thread > $D/tests_ac3k.log 2>&1 || { tail -30 $D/tests_ac3k.log; exit 1; }
bash tools/ab_env.sh r04_t42/ab "base:X=1" "ac3k:MSA_LIB=$V/libmsa_hip_ac3k.so" "ac3k_agg:MSA_LIB=$V/libmsa_hip_ac3k.so MSA_TEXT_AT_AGG=1" "base_b:X=1" "ac3k_b:MSA_LIB=$V/libmsa_hip_ac3k.so" "ac3k_agg_b:MSA_LIB=$V/libmsa_hip_ac3k.so MSA_TEXT_AT_AGG=1" || exit 1
echo __done__
