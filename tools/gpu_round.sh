set -e
export TMPDIR=/tmp
D=gpurun_out/${GR_TAG:-r7}
mkdir -p $D
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $D/gpu_tests.log 2>&1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1
timeout -k 10 300 python -u bench.py > $D/bench.json 2> $D/bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof -o run -- python3 bench.py --steps 6 --warmup 2 --no-cpu-baseline > $D/prof.log 2>&1
timeout -k 10 300 python -u tools/bench_wcs.py > $D/bench_wcs.json 2> $D/bench_wcs.err
echo done
