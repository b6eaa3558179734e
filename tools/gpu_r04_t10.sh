# configs[4] corpus: whole-step kernel trace + PMC passes (steady-state dispatches) of the sort / scan / aggregation kernels
export TMPDIR=/tmp; D=gpurun_out/r04_t10; mkdir -p $D
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $D/prof -o run -- python3 tools/highcard_bench.py 4100000 --steps 2 > $D/prof.log 2>&1 || exit 1
timeout -k 10 600 bash tools/pmc_any.sh $D/pmc k_ -- python3 tools/highcard_bench.py 4100000 --steps 1 || exit 1
LAST=1 python3 tools/pmc_kernels.py $D/pmc k_ > $D/pmc/summary_last.txt
