# the next split's head (prologue, K1, K2) on rank2 beside the previous run's text.csv gather:
# configs[2] and configs[4] A/B, then the whole GPU suite with it on
export TMPDIR=/tmp; D=gpurun_out/r04_t51; mkdir -p $D
bash tools/ab_env.sh r04_t51/ab "on:X=1" "off:MSA_HEAD_BESIDE=0" "on_b:X=1" "off_b:MSA_HEAD_BESIDE=0" "on_c:X=1" "off_c:MSA_HEAD_BESIDE=0" || exit 1
for v in on:X=1 off:MSA_HEAD_BESIDE=0 on_b:X=1 off_b:MSA_HEAD_BESIDE=0; do
  n=${v%%:*}; env ${v#*:} timeout -k 10 300 python -u tools/highcard_bench.py 4100000 --steps 3 > $D/hc_$n.txt 2>&1 || exit 1
  echo "$n $(tail -n 3 $D/hc_$n.txt | head -2 | tr '\n' ' ' | cut -c1-330)" >> $D/summary.txt
done
s=$(date +%s)
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $D/gpu_tests.log 2>&1
echo "rc=$? seconds=$(( $(date +%s) - s ))" >> $D/gpu_tests.log
echo __done__
