# Round measurement set (run ON the GPU box from the repo root):
#   bash tools/gpu_final6.sh TAG
# GPU tests, smoke, PMC passes of the main bench (stamped with this build id),
# the bench (with the CPU baseline), kernel-trace statistics and one step's
# timeline, the per-song counter's and the column splitter's PMC passes and
# benches, configs[4] stages, one-shot (cold) CLI runs.  The PMC passes run
# BEFORE the benches so that their `traffic` comes from the build they time.
# Every GPU step has its own time limit; a crash or a time limit ends the script.
set -eo pipefail
export TMPDIR=/tmp
D=gpurun_out/${1:-final6}
mkdir -p $D
rc=0
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --durations=15 --timeout 900 --timeout-method thread \
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
bash tools/pmc_wcs.sh $D/pmc_wcs
cp $D/pmc_wcs/pmc.json profiles/pmc_wcs_main.json
timeout -k 10 300 python -u tools/bench_wcs.py > $D/bench_wcs.json 2> $D/bench_wcs.err
bash tools/pmc_split.sh $D/pmc_split
cp $D/pmc_split/pmc.json profiles/pmc_split_main.json
cp $D/pmc_split/pmc.json $D/pmc_split_main.json
timeout -k 10 300 python -u tools/bench_wcs.py --path split > $D/bench_split.json 2> $D/bench_split.err
timeout -k 10 300 python -u tools/highcard_bench.py 4100000 --steps 5 > $D/highcard.txt 2>&1
bash tools/cold_run.sh ${1:-final6}/cold
echo done; exit $rc
