# radix pass tile shapes on configs[4] (rank_words): default 512x16, 512x12, 512x24, 256x32
export TMPDIR=/tmp; D=gpurun_out/r04_t26; V=$PWD/music-analyst-ai_amd/variants; mkdir -p $D
for v in base per12 per24 t256 base; do
  if [ $v = base ]; then L=$PWD/music-analyst-ai_amd/libmsa_hip.so; else L=$V/libmsa_hip_$v.so; fi
  MSA_LIB=$L timeout -k 10 300 python -u tools/highcard_bench.py 4100000 --steps 2 > $D/hc_$v.txt 2>&1 || exit 1
  echo "$v $(tail -n 3 $D/hc_$v.txt | head -2 | tr '\n' ' ' | cut -c1-400)" >> $D/summary.txt
done
MSA_LIB=$V/libmsa_hip_per12.so timeout -k 10 600 python -u -m pytest -x -q tests/test_gpu_scale.py -k "sort_designs or configs4_run" --timeout 500 --timeout-method thread > $D/tests_per12.log 2>&1
