# A/B stage timings: the in-tree build's GPU parity tests, then tools/ablate.py
# per library variant (MSA_LIB).  Usage: bash tools/ab.sh OUT variant...
set -e
out=$1; shift
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/$out.tests.log 2>&1
tail -2 gpurun_out/$out.tests.log
for v in "$@"; do
  if [ "$v" = base ]; then L=$PWD/music-analyst-ai_amd/libmsa_hip.so; else L=$PWD/music-analyst-ai_amd/variants/libmsa_hip_$v.so; fi
  echo "== $v"
  MSA_LIB=$L timeout -k 10 150 python tools/ablate.py 5000000 0
done
