# round-3 experiment: text.csv gather variants (slot map vs binary search, slots per batch) (run ON the GPU box)
set -o pipefail
mkdir -p gpurun_out/ab3
L=$PWD/music-analyst-ai_amd/variants
for v in cgbs cgb3 cgb1; do
  MSA_LIB=$L/libmsa_hip_$v.so timeout -k 10 300 python -u -m pytest -q -x tests/test_gpu_parity.py -k "torture or medium or golden" --timeout 120 --timeout-method thread > gpurun_out/ab3/tests_$v.log 2>&1 || { echo "$v parity failed"; tail -20 gpurun_out/ab3/tests_$v.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/ab3/tests_$v.log)" | tee -a gpurun_out/ab3/ab.log
done
b() {  # tag env...
  env "${@:2}" timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/ab3/$1.json 2>> gpurun_out/ab3/err.log || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/ab3/$1.json')); print('$1', d['ms_per_step'], json.dumps(d['stage_ms']))" | tee -a gpurun_out/ab3/ab.log
}
for r in 1 2; do
  b base$r X=1
  for v in cgbs cgb3 cgb1; do b ${v}_$r MSA_LIB=$L/libmsa_hip_$v.so; done
done
