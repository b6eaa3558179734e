# text gather forked at the spans (default) vs at the read-back (MSA_TEXT_AT_SPANS=0); LDS-staged key blob;
# whole-table clears for mostly-claimed tables (MSA_ABLATE=1048576: per-slot clears) on configs[4]
export TMPDIR=/tmp; D=gpurun_out/r04_t28; mkdir -p $D
timeout -k 10 600 python -u -m pytest -x -q tests/test_gpu_parity.py tests/test_gpu_split.py tests/test_gpu_dist.py tests/test_gpu_cli.py --timeout 300 --timeout-method thread > $D/tests.log 2>&1 || { tail -30 $D/tests.log; exit 1; }
bash tools/ab_env.sh r04_t28/ab "spans:X=1" "split:MSA_TEXT_AT_SPANS=0" "spans_b:X=1" "split_b:MSA_TEXT_AT_SPANS=0" "spans_c:X=1" "split_c:MSA_TEXT_AT_SPANS=0" || exit 1
for v in base:X=1 slotclr:MSA_ABLATE=1048576; do
  n=${v%%:*}; env ${v#*:} timeout -k 10 300 python -u tools/highcard_bench.py 4100000 --steps 3 > $D/hc_$n.txt 2>&1 || exit 1
  echo "$n $(tail -n 3 $D/hc_$n.txt | head -2 | tr '\n' ' ' | cut -c1-500)" >> $D/summary.txt
done
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $D/prof -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > $D/prof.log 2>&1 && python3 tools/timeline.py $D/prof > $D/timeline.txt
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $D/prof_hc -o run -- python3 tools/highcard_bench.py 4100000 --steps 2 > $D/prof_hc.log 2>&1 && python3 tools/timeline.py $D/prof_hc > $D/timeline_hc.txt
echo __done__
