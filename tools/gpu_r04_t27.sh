# artist.csv on an aux stream beside the ranking (default) vs the library stream (MSA_AUX_COL=0), text fork at the split on:
# parity, configs[2] A/B; then the radix tile shapes on configs[4] (t26)
export TMPDIR=/tmp; D=gpurun_out/r04_t27; mkdir -p $D
timeout -k 10 500 python -u -m pytest -x -q tests/test_gpu_parity.py tests/test_gpu_split.py tests/test_gpu_dist.py tests/test_gpu_cli.py --timeout 300 --timeout-method thread > $D/tests.log 2>&1 || { tail -30 $D/tests.log; exit 1; }
bash tools/ab_env.sh r04_t27/ab "aux:X=1" "noaux:MSA_AUX_COL=0" "aux_b:X=1" "noaux_b:MSA_AUX_COL=0" "aux_c:X=1" "noaux_c:MSA_AUX_COL=0" || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $D/prof -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > $D/prof.log 2>&1 && python3 tools/timeline.py $D/prof > $D/timeline.txt
bash tools/gpu_r04_t26.sh
