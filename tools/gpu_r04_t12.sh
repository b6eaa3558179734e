# word entries as a grid-stride kernel (per-workgroup key-plane reduction): configs[4] stages + parity, configs[2] bench
export TMPDIR=/tmp; D=gpurun_out/r04_t12; mkdir -p $D
timeout -k 10 300 python -u tools/highcard_bench.py 4100000 --steps 3 > $D/hc.txt 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest -x -q tests/test_gpu_scale.py -k "highcard or configs4 or sort_designs" --timeout 500 --timeout-method thread > $D/tests_scale.log 2>&1 || { tail -30 $D/tests_scale.log; exit 1; }
timeout -k 10 300 python -u -m pytest -x -q tests/test_gpu_parity.py --timeout 200 --timeout-method thread > $D/tests.log 2>&1 || { tail -30 $D/tests.log; exit 1; }
bash tools/ab_env.sh r04_t12/ab 'base:X=1' 'base_b:X=1'
