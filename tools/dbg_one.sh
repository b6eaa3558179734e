# One pytest selection per library variant, with failure details (run ON the GPU box):
#   bash tools/dbg_one.sh OUT "pytest args" variant...
set -e
out=gpurun_out/$1; sel=$2; shift 2
mkdir -p $out
for v in "$@"; do
  if [ "$v" = base ]; then L=$PWD/music-analyst-ai_amd/libmsa_hip.so; else L=$PWD/music-analyst-ai_amd/variants/libmsa_hip_$v.so; fi
  MSA_LIB=$L timeout -k 10 300 python -m pytest -x -q $sel --timeout 200 --timeout-method thread --tb=short > $out/$v.log 2>&1 || true
  echo "$v: $(tail -1 $out/$v.log)"
done
