# round-4 measurement set 8 (after the ranking work): configs[4] (seed 4, 4.1M songs) stages + kernel trace; configs[3] size through the C host (100M songs, 1 GPU)
export TMPDIR=/tmp; D=gpurun_out/r04_final8; mkdir -p $D
timeout -k 10 300 python -u tools/highcard_bench.py 4100000 --steps 3 > $D/highcard.txt 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof_hc -o run -- python3 tools/highcard_bench.py 4100000 --steps 2 > $D/prof_hc.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py --driver chost --gpus 1 --songs 100000000 --steps 3 --warmup 1 > $D/bench_chost_100m.json 2> $D/bench_chost_100m.err || exit 1

timeout -k 10 300 python -u bench.py --pmc-file profiles/pmc_scan_main.json > $D/bench2.json 2> $D/bench2.err || exit 1
bash tools/ab_env.sh r04_final8/ab "a:X=1" "b:X=1" "c:X=1" || exit 1
echo __done__
