# full GPU suite on the composite-key / tie-compaction build; configs[2] bench; configs[4] table growth multiplier A/B
export TMPDIR=/tmp; D=gpurun_out/r04_t33; mkdir -p $D
timeout -k 10 900 python -u -m pytest -x -q -m gpu tests --timeout 600 --timeout-method thread > $D/tests.log 2>&1 || { tail -30 $D/tests.log; exit 1; }
bash tools/ab_env.sh r04_t33/ab "base:X=1" "base_b:X=1" || exit 1
for v in g4:MSA_GROW_MUL=4 g3:MSA_GROW_MUL=3 g2:MSA_GROW_MUL=2; do
  n=${v%%:*}; env ${v#*:} timeout -k 10 300 python -u tools/highcard_bench.py 4100000 --steps 3 > $D/hc_$n.txt 2>&1 || exit 1
  echo "$n $(tail -n 3 $D/hc_$n.txt | head -2 | tr '\n' ' ' | cut -c1-500)" >> $D/summary.txt
done
echo __done__
