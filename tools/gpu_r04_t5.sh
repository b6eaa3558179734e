# round 4: race fixes (write-through scan totals, sync before free) + pipelined token pass + 2-deep struct prefetch
export TMPDIR=/tmp; D=gpurun_out/r04_t5; V=/root/repo/music-analyst-ai_amd/variants; mkdir -p $D
for v in s1 s2; do timeout -k 10 200 python -u tools/dbg_shards.py $D/$v 5 highcard 6000 5 > $D/$v.log 2>&1 || exit 1; done
rm -f $D/*/in.csv
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $D/parity.log 2>&1 || exit 1
bash tools/ab_env.sh r04_t5/ab 'base:MSA_K3SPLIT=1' "nopipe:MSA_LIB=$V/libmsa_hip_nopipe.so" "pf1:MSA_LIB=$V/libmsa_hip_pf1.so" 'base_b:MSA_K3SPLIT=1' "nopipe_b:MSA_LIB=$V/libmsa_hip_nopipe.so" "pf1_b:MSA_LIB=$V/libmsa_hip_pf1.so" || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $D/prof -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > $D/prof.log 2>&1 && python3 tools/timeline.py $D/prof > $D/timeline.txt
timeout -k 10 900 python -u -m pytest tests/test_gpu_dist.py tests/test_gpu_split.py -x -q --timeout 600 --timeout-method thread -k "not full_size" > $D/dist_split.log 2>&1
