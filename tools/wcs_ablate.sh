# Timing of k_wcs_rows with parts switched off (MSA_WCS_ABLATE, results wrong by design).
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/abl
for v in 0 1 4; do
  MSA_WCS_ABLATE=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/abl/p$v -o run -- python3 tools/bench_wcs.py --songs 2000000 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/abl/b$v.log 2>&1
done
echo done
