# Round measurement set (run ON the GPU box from the repo root):
#   bash tools/gpu_final.sh TAG
# GPU tests, smoke, PMC passes (stamped with this build's msa_build_id and
# installed as the PMC file the bench attaches), bench (with the CPU baseline),
# kernel-trace profile, PMC passes of the per-song counter (stamped the same
# way), per-song counter bench.  The PMC passes run BEFORE the
# bench so that its `traffic` comes from the build it times.  Every GPU step has
# its own time limit; a failing step ends the script.
set -eo pipefail
export TMPDIR=/tmp
D=gpurun_out/${1:-final}
mkdir -p $D
# test failures (rc 1) are reported and the measurements still run; anything
# else (a crash, a time limit) ends the script here
rc=0
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --durations=15 --timeout 600 --timeout-method thread \
    > $D/gpu_tests.log 2>&1 || rc=$?
echo "pytest rc $rc"
[ $rc -le 1 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1
bash tools/pmc.sh $D/pmc
cp $D/pmc/pmc.json profiles/pmc_scan_main.json
timeout -k 10 300 python -u bench.py > $D/bench.json 2> $D/bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-pcie > $D/prof.log 2>&1
bash tools/pmc_wcs.sh $D/pmc_wcs
cp $D/pmc_wcs/pmc.json profiles/pmc_wcs_main.json
timeout -k 10 300 python -u tools/bench_wcs.py > $D/bench_wcs.json 2> $D/bench_wcs.err
echo done; exit $rc
