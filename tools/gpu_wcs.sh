set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/w9
timeout -k 10 400 python -u -m pytest tests/test_gpu_wcs.py -q --timeout 120 --timeout-method thread > gpurun_out/w9/wcs_tests.log 2>&1
timeout -k 10 300 python -u tools/bench_wcs.py > gpurun_out/w9/bench_wcs.json 2> gpurun_out/w9/bench_wcs.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/w9/prof -o run -- python3 tools/bench_wcs.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/w9/prof.log 2>&1
echo done
