# A/B: deferred text.csv with the LDS gather vs the LDS-free gather; copy-rate calibration; parity of the LDS-free gather
export TMPDIR=/tmp; D=gpurun_out/r04_t14; mkdir -p $D
MSA_GATHER_W=1 timeout -k 10 300 python -u -m pytest -x -q tests/test_gpu_parity.py tests/test_gpu_split.py --timeout 200 --timeout-method thread > $D/tests.log 2>&1 || { tail -30 $D/tests.log; exit 1; }
bash tools/ab_env.sh r04_t14/ab 'lds:X=1' 'ldsfree:MSA_GATHER_W=1' 'lds_b:X=1' 'ldsfree_b:MSA_GATHER_W=1' || exit 1
timeout -k 10 120 python3 tools/copy_calib.py > $D/copy_calib.txt 2>&1 || exit 1
