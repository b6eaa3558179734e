# A/B of library variants (music-analyst-ai_amd/variants/libmsa_hip_<v>.so, `make variant`):
# per variant a quick parity subset, then the stage times of tools/ablate.py.
# Usage (on the GPU box): bash tools/abv.sh OUT variant...   ("base" = the in-tree build)
set -e
out=gpurun_out/$1; shift
mkdir -p gpurun_out
: > $out.log
for v in "$@"; do
  if [ "$v" = base ]; then L=$PWD/music-analyst-ai_amd/libmsa_hip.so; else L=$PWD/music-analyst-ai_amd/variants/libmsa_hip_$v.so; fi
  echo "== $v" >> $out.log
  MSA_LIB=$L timeout -k 10 200 python -m pytest -q -x tests/test_gpu_parity.py -k "torture or golden or small or medium" --timeout 120 --timeout-method thread 2>&1 | tail -1 >> $out.log
  MSA_LIB=$L timeout -k 10 150 python tools/ablate.py ${SONGS:-5000000} 0 >> $out.log 2>&1
done
echo done >> $out.log
