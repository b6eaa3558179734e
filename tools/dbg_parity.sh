# Quick parity subset per library variant with failure details (run ON the GPU box):
#   bash tools/dbg_parity.sh OUT variant...   ("base" = the in-tree build)
set -e
out=gpurun_out/$1; shift
mkdir -p $out
for v in "$@"; do
  if [ "$v" = base ]; then L=$PWD/music-analyst-ai_amd/libmsa_hip.so; else L=$PWD/music-analyst-ai_amd/variants/libmsa_hip_$v.so; fi
  MSA_LIB=$L timeout -k 10 200 python -m pytest -x -q tests/test_gpu_parity.py -k "torture or golden or small or medium" \
      --timeout 120 --timeout-method thread --tb=short > $out/$v.log 2>&1 || true
  tail -1 $out/$v.log
done
