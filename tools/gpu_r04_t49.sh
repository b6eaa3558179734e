# rank2 (spans beside the token pass, artists' ranking) and aux (artist.csv) at the lowest priority
export TMPDIR=/tmp; D=gpurun_out/r04_t49; mkdir -p $D
MSA_RANK2_PRIO=-1 MSA_AUX_PRIO=-1 timeout -k 10 600 python -u -m pytest -x -q tests/test_gpu_parity.py --timeout 300 --timeout-method thread > $D/tests.log 2>&1 || { tail -30 $D/tests.log; exit 1; }
bash tools/ab_env.sh r04_t49/ab "base:X=1" "r2lo:MSA_RANK2_PRIO=-1" "auxlo:MSA_AUX_PRIO=-1" "both:MSA_RANK2_PRIO=-1 MSA_AUX_PRIO=-1" "base_b:X=1" "r2lo_b:MSA_RANK2_PRIO=-1" "auxlo_b:MSA_AUX_PRIO=-1" "both_b:MSA_RANK2_PRIO=-1 MSA_AUX_PRIO=-1" || exit 1
echo __done__
