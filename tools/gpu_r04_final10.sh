# round-4 measurement set 10 (side stream at the highest priority): whole GPU suite, smoke, PMC (stamped),
# bench with the CPU leg, kernel trace + timeline, configs[4], configs[3] through the C host, A/B repeats
export TMPDIR=/tmp; D=gpurun_out/r04_final10; mkdir -p $D
s=$(date +%s)
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 900 --timeout-method thread > $D/gpu_tests.log 2>&1
echo "rc=$? seconds=$(( $(date +%s) - s ))" >> $D/gpu_tests.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || exit 1
bash tools/pmc.sh $D/pmc > $D/pmc.log 2>&1 && cp $D/pmc/pmc.json $D/pmc_scan_main.json
timeout -k 10 300 python -u bench.py --pmc-file $D/pmc/pmc.json > $D/bench.json 2> $D/bench.err || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --memory-copy-trace --output-format csv -d $D/prof -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > $D/prof.log 2>&1 && python3 tools/timeline.py $D/prof > $D/timeline.txt
timeout -k 10 300 python -u tools/highcard_bench.py 4100000 --steps 3 > $D/highcard.txt 2>&1 || exit 1
timeout -k 10 600 python -u bench.py --driver chost --gpus 1 --songs 100000000 --steps 3 --warmup 1 > $D/bench_chost_100m.json 2> $D/bench_chost_100m.err || exit 1
bash tools/ab_env.sh r04_final10/ab "hi:X=1" "base:MSA_SIDE_PRIO=0" "hi_b:X=1" "base_b:MSA_SIDE_PRIO=0" || exit 1
echo __done__
