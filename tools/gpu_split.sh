set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/s5
timeout -k 10 300 python -u -m pytest tests/test_gpu_split.py -q --timeout 120 --timeout-method thread > gpurun_out/s5/split_tests.log 2>&1
timeout -k 10 300 python -u tools/bench_wcs.py --path split > gpurun_out/s5/bench_split.json 2> gpurun_out/s5/bench_split.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/s5/prof -o run -- python3 tools/bench_wcs.py --path split --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/s5/prof.log 2>&1
echo done
