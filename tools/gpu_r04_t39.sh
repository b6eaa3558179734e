# long-word insert back to one occurrence per thread; artist-merge list appends staged per workgroup
export TMPDIR=/tmp; D=gpurun_out/r04_t39; mkdir -p $D
timeout -k 10 900 python -u -m pytest -x -q tests/test_gpu_parity.py tests/test_gpu_split.py tests/test_gpu_scale.py --timeout 800 --timeout-method thread > $D/tests.log 2>&1 || { tail -30 $D/tests.log; exit 1; }
timeout -k 10 300 python -u tools/highcard_bench.py 4100000 --steps 3 > $D/hc.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/highcard_bench.py 4100000 --steps 3 > $D/hc_b.txt 2>&1 || exit 1
bash tools/ab_env.sh r04_t39/ab "base:X=1" "base_b:X=1" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $D/prof_hc -o run -- python3 tools/highcard_bench.py 4100000 --steps 2 > $D/prof_hc.log 2>&1 && python3 tools/timeline.py $D/prof_hc > $D/timeline_hc.txt
echo __done__
