# batched radix look-back (OS_LB=8 vs 1), short-key final without gathers, no count plane for radix-ranked words
export TMPDIR=/tmp; D=gpurun_out/r04_t34; V=$PWD/music-analyst-ai_amd/variants; mkdir -p $D
timeout -k 10 900 python -u -m pytest -x -q tests/test_gpu_comp_sort.py tests/test_gpu_scale.py tests/test_gpu_parity.py -k "comp_sort or sort_designs or configs4_run or torture or golden" --timeout 800 --timeout-method thread > $D/tests.log 2>&1 || { tail -30 $D/tests.log; exit 1; }
for v in lb8 lb1 lb8_b lb1_b; do
  case $v in lb1*) L=$V/libmsa_hip_lb1.so;; *) L=$PWD/music-analyst-ai_amd/libmsa_hip.so;; esac
  MSA_LIB=$L timeout -k 10 300 python -u tools/highcard_bench.py 4100000 --steps 3 > $D/hc_$v.txt 2>&1 || exit 1
  echo "$v $(tail -n 3 $D/hc_$v.txt | head -2 | tr '\n' ' ' | cut -c1-500)" >> $D/summary.txt
done
bash tools/ab_env.sh r04_t34/ab "base:X=1" "lb1:MSA_LIB=$V/libmsa_hip_lb1.so" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $D/prof_hc -o run -- python3 tools/highcard_bench.py 4100000 --steps 2 > $D/prof_hc.log 2>&1 && python3 tools/timeline.py $D/prof_hc > $D/timeline_hc.txt
echo __done__
