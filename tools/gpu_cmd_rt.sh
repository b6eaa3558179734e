# round-3 experiment: small-table ranking kernels and a CU-masked side stream (run ON the GPU box)
set -o pipefail
mkdir -p gpurun_out/rt
b() {  # tag env...
  env "${@:2}" timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/rt/$1.json 2>> gpurun_out/rt/err.log || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/rt/$1.json')); print('$1', d['ms_per_step'], json.dumps(d['stage_ms']))" | tee -a gpurun_out/rt/ab.log
}
L=$PWD/music-analyst-ai_amd/variants
for r in 1 2; do
  b base$r X=1
  b rc0_$r MSA_LIB=$L/libmsa_hip_rc0.so
  b rt1k_$r MSA_LIB=$L/libmsa_hip_rt1k.so
  b free8_$r MSA_SIDE_FREE=8
  b free16_$r MSA_SIDE_FREE=16
done
