set -e
mkdir -p gpurun_out
: > gpurun_out/var2.log
for v in base g1 g2 g3 g4; do
  if [ $v = base ]; then L=$PWD/music-analyst-ai_amd/libmsa_hip.so; else L=$PWD/music-analyst-ai_amd/variants/libmsa_hip_$v.so; fi
  echo "== $v" >> gpurun_out/var2.log
  MSA_LIB=$L timeout -k 10 120 python tools/ablate.py 2000000 0 >> gpurun_out/var2.log 2>&1
  MSA_LIB=$L timeout -k 10 200 python -m pytest -q -x tests/test_gpu_parity.py -k "torture or medium or golden" --timeout 120 --timeout-method thread 2>&1 | tail -1 >> gpurun_out/var2.log
done
