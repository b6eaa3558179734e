# round-3 experiment: artist.csv on the rank2 stream (off the artist pass's read-back) vs the previous build (run ON the GPU box)
set -o pipefail
mkdir -p gpurun_out/ab2
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ab2/tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/ab2/tests.log; exit 1; }
tail -1 gpurun_out/ab2/tests.log
b() {  # tag env...
  env "${@:2}" timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/ab2/$1.json 2>> gpurun_out/ab2/err.log || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/ab2/$1.json')); print('$1', d['ms_per_step'], json.dumps(d['stage_ms']))" | tee -a gpurun_out/ab2/ab.log
}
L=$PWD/music-analyst-ai_amd/variants
for r in 1 2 3; do
  b base$r X=1
  b prev_$r MSA_LIB=$L/libmsa_hip_prev.so
done
