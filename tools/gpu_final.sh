# Round measurement set (run ON the GPU box from the repo root):
#   bash tools/gpu_final.sh TAG
# GPU tests, smoke, bench (with the CPU baseline), kernel-trace profile, PMC
# passes stamped with this build, per-song counter bench.  Every GPU step has
# its own time limit; a failing step ends the script.
set -eo pipefail
export TMPDIR=/tmp
D=gpurun_out/${1:-final}
mkdir -p $D
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > $D/gpu_tests.log 2>&1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1
timeout -k 10 300 python -u bench.py > $D/bench.json 2> $D/bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > $D/prof.log 2>&1
bash tools/pmc.sh $D/pmc
timeout -k 10 300 python -u tools/bench_wcs.py > $D/bench_wcs.json 2> $D/bench_wcs.err
echo done
