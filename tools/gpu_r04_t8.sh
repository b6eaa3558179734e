# configs[4]-scale profile: the test's corpus (seed 4, 4.1M songs): stages + kernel trace of one step
export TMPDIR=/tmp; D=gpurun_out/r04_t8; mkdir -p $D
timeout -k 10 300 python -u tools/highcard_bench.py 4100000 --steps 2 > $D/highcard.txt 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof -o run -- python3 tools/highcard_bench.py 4100000 --steps 1 > $D/prof.log 2>&1
