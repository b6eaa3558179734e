#!/usr/bin/env bash
# SQ/TCC counter passes (one rocprofv3 run each) over a command, summarised
# per kernel: bash tools/pmc_any.sh OUT FILTER -- cmd args...
set -euo pipefail
export TMPDIR=/tmp
OUT=$1; FLT=$2; shift 3
mkdir -p "$OUT"
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY" \
  "SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_INSTS_LDS_ATOMIC GRBM_GUI_ACTIVE" \
  "TCC_ATOMIC_sum TCC_EA0_ATOMIC_sum TA_FLAT_ATOMIC_WAVEFRONTS_sum" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d "$OUT/p$i" -o run -- "$@" > "$OUT/p$i.log" 2>&1
done
python3 tools/pmc_kernels.py "$OUT" "$FLT" > "$OUT/summary.txt"
