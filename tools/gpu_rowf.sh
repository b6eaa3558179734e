set -e
export TMPDIR=/tmp
D=gpurun_out/${GR_TAG:-f1}
mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_gpu_wcs.py tests/test_gpu_split.py -q --timeout 120 --timeout-method thread > $D/tests.log 2>&1
timeout -k 10 300 python -u tools/bench_wcs.py > $D/bench_wcs.json 2> $D/bench_wcs.err
timeout -k 10 300 python -u tools/bench_wcs.py --path split > $D/bench_split.json 2> $D/bench_split.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof -o run -- python3 tools/bench_wcs.py --steps 3 --warmup 1 --no-cpu-baseline > $D/prof.log 2>&1
echo done
