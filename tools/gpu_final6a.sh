# Round measurement set, part 1 of 2 (run ON the GPU box from the repo root):
#   bash tools/gpu_final6a.sh TAG
# GPU tests, smoke, the main bench's PMC passes (stamped with this build id),
# the bench (with the CPU baseline), kernel-trace statistics + one step's
# timeline.  Every GPU step has its own time limit; a crash ends the script.
set -eo pipefail
export TMPDIR=/tmp
D=gpurun_out/${1:-final6}
mkdir -p $D
rc=0
timeout -k 10 700 python -u -m pytest tests -m gpu -v --durations=15 --timeout 600 --timeout-method thread \
    > $D/gpu_tests.log 2>&1 || rc=$?
echo "pytest rc $rc" | tee $D/pytest_rc.txt
[ $rc -le 1 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1
bash tools/pmc.sh $D/pmc
cp $D/pmc/pmc.json profiles/pmc_scan_main.json
cp $D/pmc/pmc.json $D/pmc_scan_main.json
timeout -k 10 300 python -u bench.py > $D/bench.json 2> $D/bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-pcie > $D/prof.log 2>&1
python3 tools/timeline.py $D/prof > $D/step_timeline.txt 2>&1 || true
echo done; exit $rc
