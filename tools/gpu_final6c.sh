# Round measurement set, the main bench's part without the test suite (run ON
# the GPU box from the repo root):  bash tools/gpu_final6c.sh TAG
# PMC passes (stamped with this build id), the bench, kernel-trace statistics
# + one step's timeline -- for a bench.py change that leaves the kernels alone.
set -eo pipefail
export TMPDIR=/tmp
D=gpurun_out/${1:-final6}
mkdir -p $D
bash tools/pmc.sh $D/pmc
cp $D/pmc/pmc.json $D/pmc_scan_main.json
timeout -k 10 300 python -u bench.py > $D/bench.json 2> $D/bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-pcie > $D/prof.log 2>&1
python3 tools/timeline.py $D/prof > $D/step_timeline.txt 2>&1 || true
echo done
