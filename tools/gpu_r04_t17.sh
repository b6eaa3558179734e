# K1 with per-lane terminator counts (one wave reduction per chunk) vs the old per-block ballots (k1old): parity, configs[2] A/B
export TMPDIR=/tmp; D=gpurun_out/r04_t17; V=$PWD/music-analyst-ai_amd/variants; mkdir -p $D
timeout -k 10 400 python -u -m pytest -x -q tests/test_gpu_parity.py tests/test_gpu_dist.py tests/test_gpu_split.py tests/test_gpu_cli.py --timeout 200 --timeout-method thread > $D/tests.log 2>&1 || { tail -30 $D/tests.log; exit 1; }
bash tools/ab_env.sh r04_t17/ab "k1new:X=1" "k1old:MSA_LIB=$V/libmsa_hip_k1old.so" "k1new_b:X=1" "k1old_b:MSA_LIB=$V/libmsa_hip_k1old.so" || exit 1
