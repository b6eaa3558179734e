# A/B of per-song counter builds (run ON the GPU box from the repo root):
#   bash tools/wcs_ab.sh TAG variant[:ablate]...   ("base" = music-analyst-ai_amd/libmsa_hip.so;
#   ablate = MSA_WCS_ABLATE bits, timing only)
# wcs GPU tests on the base build, then bench_wcs per variant.
set -eo pipefail
export TMPDIR=/tmp
D=gpurun_out/$1; shift
mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_gpu_wcs.py -x -q --timeout 120 --timeout-method thread > $D/tests.log 2>&1
for spec in "$@"; do
  v=${spec%%:*}; ab=0; [ "$spec" != "$v" ] && ab=${spec#*:}
  if [ "$v" = base ]; then L=music-analyst-ai_amd/libmsa_hip.so; else L=music-analyst-ai_amd/variants/libmsa_hip_$v.so; fi
  MSA_WCS_ABLATE=$ab MSA_LIB=$L timeout -k 10 200 python -u tools/bench_wcs.py --no-cpu-baseline > $D/$v$ab.json 2> $D/$v$ab.err
  python3 -c "import json,sys; d=json.load(open('$D/$v$ab.json')); print('$spec', d['value'], d['ms_per_step'])"
done
