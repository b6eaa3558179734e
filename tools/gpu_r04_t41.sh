# word slot lists on rank2 beside the artist pass (MSA_LISTS_BESIDE=0: on the library stream)
export TMPDIR=/tmp; D=gpurun_out/r04_t41; mkdir -p $D
timeout -k 10 900 python -u -m pytest -x -q tests/test_gpu_parity.py tests/test_gpu_split.py tests/test_gpu_scale.py tests/test_gpu_cli.py --timeout 800 --timeout-method thread > $D/tests.log 2>&1 || { tail -30 $D/tests.log; exit 1; }
bash tools/ab_env.sh r04_t41/ab "beside:X=1" "main:MSA_LISTS_BESIDE=0" "beside_b:X=1" "main_b:MSA_LISTS_BESIDE=0" || exit 1
for v in beside:X=1 main:MSA_LISTS_BESIDE=0 beside_b:X=1 main_b:MSA_LISTS_BESIDE=0; do
  n=${v%%:*}; env ${v#*:} timeout -k 10 300 python -u tools/highcard_bench.py 4100000 --steps 3 > $D/hc_$n.txt 2>&1 || exit 1
  echo "$n $(tail -n 3 $D/hc_$n.txt | head -2 | tr '\n' ' ' | cut -c1-300)" >> $D/summary.txt
done
echo __done__
