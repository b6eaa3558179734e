# round-4 measurement set 9: word tables zeroed beside the ranking (MSA_CLEAR_EARLY=0: in the next prologue);
# whole GPU suite, smoke, PMC (stamped), bench, configs[4] A/B, configs[2] A/B
export TMPDIR=/tmp; D=gpurun_out/r04_final9; mkdir -p $D
s=$(date +%s)
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 900 --timeout-method thread > $D/gpu_tests.log 2>&1
echo "rc=$? seconds=$(( $(date +%s) - s ))" >> $D/gpu_tests.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || exit 1
for v in early:X=1 late:MSA_CLEAR_EARLY=0 early_b:X=1 late_b:MSA_CLEAR_EARLY=0; do
  n=${v%%:*}; env ${v#*:} timeout -k 10 300 python -u tools/highcard_bench.py 4100000 --steps 3 > $D/hc_$n.txt 2>&1 || exit 1
  echo "$n $(tail -n 3 $D/hc_$n.txt | head -2 | tr '\n' ' ' | cut -c1-300)" >> $D/summary.txt
done
bash tools/pmc.sh $D/pmc > $D/pmc.log 2>&1 && cp $D/pmc/pmc.json $D/pmc_scan_main.json
timeout -k 10 300 python -u bench.py --pmc-file $D/pmc/pmc.json > $D/bench.json 2> $D/bench.err || exit 1
bash tools/ab_env.sh r04_final9/ab "early:X=1" "late:MSA_CLEAR_EARLY=0" "early_b:X=1" "late_b:MSA_CLEAR_EARLY=0" || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --memory-copy-trace --output-format csv -d $D/prof -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > $D/prof.log 2>&1 && python3 tools/timeline.py $D/prof > $D/timeline.txt
echo __done__
