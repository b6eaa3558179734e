#!/usr/bin/env bash
# PMC passes (FETCH_SIZE, WRITE_SIZE, SQ) over the row (f) benches, one
# rocprofv3 run per counter group; summarise with tools/pmc_kernels.py.
set -euo pipefail
export TMPDIR=/tmp
OUT=${1:-gpurun_out/pmc_rowf}
mkdir -p "$OUT"
W=(python3 tools/bench_wcs.py --songs 2000000 --steps 1 --warmup 1 --no-cpu-baseline)
S=(python3 tools/bench_wcs.py --path split --songs 2000000 --steps 1 --warmup 1 --no-cpu-baseline)
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/wf" -o run -- "${W[@]}" > "$OUT/wf.log" 2>&1
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/ww" -o run -- "${W[@]}" > "$OUT/ww.log" 2>&1
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY --output-format csv -d "$OUT/wsq" -o run -- "${W[@]}" > "$OUT/wsq.log" 2>&1
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/sf" -o run -- "${S[@]}" > "$OUT/sf.log" 2>&1
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/sw" -o run -- "${S[@]}" > "$OUT/sw.log" 2>&1
python3 tools/pmc_kernels.py "$OUT" k_wcs_ > "$OUT/wcs_pmc.txt"
python3 tools/pmc_kernels.py "$OUT" k_csvcol > "$OUT/split_pmc.txt"
echo done
