# k_miss_agg: first probe slots of a full LDS table's entries loaded ahead (MSA_MA_PREF=0: one after another)
export TMPDIR=/tmp; D=gpurun_out/r04_t46; mkdir -p $D
timeout -k 10 600 python -u -m pytest -x -q tests/test_gpu_parity.py tests/test_gpu_scale.py -k "not configs4_cli" --timeout 800 --timeout-method thread > $D/tests.log 2>&1 || { tail -30 $D/tests.log; exit 1; }
for v in pref:X=1 nopref:MSA_MA_PREF=0 pref_b:X=1 nopref_b:MSA_MA_PREF=0; do
  n=${v%%:*}; env ${v#*:} timeout -k 10 300 python -u tools/highcard_bench.py 4100000 --steps 3 > $D/hc_$n.txt 2>&1 || exit 1
  echo "$n $(tail -n 3 $D/hc_$n.txt | head -2 | tr '\n' ' ' | cut -c1-420)" >> $D/summary.txt
done
bash tools/ab_env.sh r04_t46/ab "pref:X=1" "nopref:MSA_MA_PREF=0" "pref_b:X=1" "nopref_b:MSA_MA_PREF=0" || exit 1
echo __done__
