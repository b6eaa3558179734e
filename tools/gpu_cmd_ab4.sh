# round-3 experiment: small-table ranking's tile loop split over 4 workgroup groups vs one (run ON the GPU box)
set -o pipefail
mkdir -p gpurun_out/ab4
L=$PWD/music-analyst-ai_amd/variants
b() {  # tag env...
  env "${@:2}" timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/ab4/$1.json 2>> gpurun_out/ab4/err.log || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/ab4/$1.json')); print('$1', d['ms_per_step'], json.dumps(d['stage_ms']))" | tee -a gpurun_out/ab4/ab.log
}
for r in 1 2 3; do
  b base$r X=1
  b prev_$r MSA_LIB=$L/libmsa_hip_prev.so
done
