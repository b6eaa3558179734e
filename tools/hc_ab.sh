set -eo pipefail
export TMPDIR=/tmp
D=gpurun_out/r06_asd; mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_gpu_dense.py -x -q --timeout 300 --timeout-method thread > $D/tests.log 2>&1
for r in 1 2; do for v in base asd; do
  if [ $v = base ]; then L=$PWD/music-analyst-ai_amd/libmsa_hip.so; else L=$PWD/music-analyst-ai_amd/variants/libmsa_hip_$v.so; fi
  MSA_LIB=$L timeout -k 10 300 python -u tools/highcard_bench.py 4100000 --steps 5 > $D/$v.$r.txt 2>&1
  echo "$v $(grep ms/step $D/$v.$r.txt)" >> $D/summary.txt
done; done
