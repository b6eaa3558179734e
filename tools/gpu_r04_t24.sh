# artists' radix ranking on its own host thread + stream beside the words': configs[4] parity (scale tests) and stages
export TMPDIR=/tmp; D=gpurun_out/r04_t24; mkdir -p $D
timeout -k 10 700 python -u -m pytest -x -q tests/test_gpu_scale.py -k "highcard or configs4 or sort_designs" --timeout 600 --timeout-method thread > $D/tests_scale.log 2>&1 || { tail -30 $D/tests_scale.log; exit 1; }
timeout -k 10 300 python -u -m pytest -x -q tests/test_gpu_parity.py tests/test_gpu_dist.py --timeout 200 --timeout-method thread > $D/tests.log 2>&1 || { tail -30 $D/tests.log; exit 1; }
timeout -k 10 300 python -u tools/highcard_bench.py 4100000 --steps 3 > $D/hc.txt 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $D/prof_hc -o run -- python3 tools/highcard_bench.py 4100000 --steps 2 > $D/prof_hc.log 2>&1 || exit 1
