# round 4: split scan parity + A/B (fused vs split, occupancy, spans overlap) + timeline + dist/split tests
export TMPDIR=/tmp; D=gpurun_out/r04_t1; V=/root/repo/music-analyst-ai_amd/variants; mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $D/parity.log 2>&1 && \
bash tools/ab_env.sh r04_t1/ab 'fused:MSA_K3SPLIT=0' 'split5:MSA_K3SPLIT=1' 'split5_noov:MSA_ABLATE=8192' "split6:MSA_LIB=$V/libmsa_hip_w6.so" "split4:MSA_LIB=$V/libmsa_hip_w4.so" 'fused_b:MSA_K3SPLIT=0' 'split5_b:MSA_K3SPLIT=1' && \
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $D/prof -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > $D/prof.log 2>&1 && \
python3 tools/timeline.py $D/prof > $D/timeline.txt && \
timeout -k 10 700 python -u -m pytest tests/test_gpu_dist.py tests/test_gpu_split.py -x -q --timeout 300 --timeout-method thread > $D/dist_split.log 2>&1
