set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/r6
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r6/gpu_tests.log 2>&1
timeout -k 10 300 python -u bench.py > gpurun_out/r6/bench.json 2> gpurun_out/r6/bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r6/prof -o run -- python3 bench.py --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/r6/prof.log 2>&1
echo done
