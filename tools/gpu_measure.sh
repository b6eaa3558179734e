# Measurement set without the test suite (run ON the GPU box from the repo root):
#   bash tools/gpu_measure.sh TAG
# smoke, PMC passes (stamped with this build id, installed as the PMC files the
# benches attach), bench (CPU baseline included), kernel-trace profile with the
# per-dispatch trace kept, and the same for the per-song counter (row f).
# Each GPU step has its own time limit; any failure ends the script.
set -eo pipefail
export TMPDIR=/tmp
D=gpurun_out/${1:-measure}
mkdir -p $D
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1
bash tools/pmc.sh $D/pmc
cp $D/pmc/pmc.json profiles/pmc_scan_main.json
cp $D/pmc/pmc.json $D/pmc_scan_main.json
timeout -k 10 300 python -u bench.py > $D/bench.json 2> $D/bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-pcie > $D/prof.log 2>&1
bash tools/pmc_wcs.sh $D/pmc_wcs
cp $D/pmc_wcs/pmc.json profiles/pmc_wcs_main.json
cp $D/pmc_wcs/pmc.json $D/pmc_wcs_main.json
timeout -k 10 300 python -u tools/bench_wcs.py > $D/bench_wcs.json 2> $D/bench_wcs.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof_wcs -o run -- python3 tools/bench_wcs.py --steps 3 --warmup 1 --no-cpu-baseline > $D/prof_wcs.log 2>&1
echo done
