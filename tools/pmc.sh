#!/usr/bin/env bash
# PMC passes over bench.py (run ON the GPU box, from the repo root), one
# rocprofv3 run per counter group, as MI355X_MICROARCH.md prescribes:
#   pass 1  FETCH_SIZE            (TCC: 3 slots)
#   pass 2  WRITE_SIZE            (TCC: 2 slots)
#   pass 3  SQ counters of K3     (8 SQ slots)
# Then tools/pmc_summary.py folds them into profiles/pmc_scan_main.json.
set -euo pipefail
export TMPDIR=/tmp
OUT=${1:-gpurun_out/pmc}
STEPS=${STEPS:-1}
mkdir -p "$OUT"
B=(python3 bench.py --steps "$STEPS" --warmup 1 --no-cpu-baseline)
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- "${B[@]}" > "$OUT/fetch.log" 2>&1
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- "${B[@]}" > "$OUT/write.log" 2>&1
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY --output-format csv -d "$OUT/sq" -o run -- "${B[@]}" > "$OUT/sq.log" 2>&1
python3 tools/pmc_summary.py "$OUT"
