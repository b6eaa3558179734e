# configs[4]: rank2 (the artists' radix ranking beside the words') at the lowest priority
export TMPDIR=/tmp; D=gpurun_out/r04_t50; mkdir -p $D
for v in base:X=1 r2lo:MSA_RANK2_PRIO=-1 base_b:X=1 r2lo_b:MSA_RANK2_PRIO=-1 base_c:X=1 r2lo_c:MSA_RANK2_PRIO=-1; do
  n=${v%%:*}; env ${v#*:} timeout -k 10 300 python -u tools/highcard_bench.py 4100000 --steps 3 > $D/hc_$n.txt 2>&1 || exit 1
  echo "$n $(tail -n 3 $D/hc_$n.txt | head -2 | tr '\n' ' ' | cut -c1-330)" >> $D/summary.txt
done
echo __done__
