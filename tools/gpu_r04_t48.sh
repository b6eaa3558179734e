# text.csv's side stream at the highest priority (MSA_SIDE_PRIO=1) vs default
export TMPDIR=/tmp; D=gpurun_out/r04_t48; mkdir -p $D
MSA_SIDE_PRIO=1 timeout -k 10 600 python -u -m pytest -x -q tests/test_gpu_parity.py --timeout 300 --timeout-method thread > $D/tests.log 2>&1 || { tail -30 $D/tests.log; exit 1; }
bash tools/ab_env.sh r04_t48/ab "base:X=1" "hi:MSA_SIDE_PRIO=1" "base_b:X=1" "hi_b:MSA_SIDE_PRIO=1" "base_c:X=1" "hi_c:MSA_SIDE_PRIO=1" || exit 1
echo __done__
