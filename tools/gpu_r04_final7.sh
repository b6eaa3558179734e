# round-4 measurement set 7 (after the ranking work): whole GPU suite (timed), smoke, PMC passes (stamped), bench with the CPU leg, kernel trace + timeline
export TMPDIR=/tmp; D=gpurun_out/r04_final7; mkdir -p $D
s=$(date +%s)
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 900 --timeout-method thread > $D/gpu_tests.log 2>&1
echo "rc=$? seconds=$(( $(date +%s) - s ))" >> $D/gpu_tests.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || exit 1
bash tools/pmc.sh $D/pmc > $D/pmc.log 2>&1 && cp $D/pmc/pmc.json $D/pmc_scan_main.json
timeout -k 10 300 python -u bench.py --pmc-file $D/pmc/pmc.json > $D/bench.json 2> $D/bench.err || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --memory-copy-trace --output-format csv -d $D/prof -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > $D/prof.log 2>&1 && python3 tools/timeline.py $D/prof > $D/timeline.txt
echo __done__
