#!/usr/bin/env bash
# PMC passes over tools/ablate.py (5M songs), one rocprofv3 run per counter
# group (run ON the GPU box): bash tools/pmc_k3.sh OUT [ablate bits]
set -euo pipefail
export TMPDIR=/tmp
OUT=${1:-gpurun_out/pmck3}
BITS=${2:-0}
mkdir -p "$OUT"
P=(python3 tools/ablate.py 5000000 $BITS)
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" \
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY" \
  "SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_INSTS_LDS_ATOMIC GRBM_GUI_ACTIVE" \
  "TCC_ATOMIC_sum TCC_EA0_ATOMIC_sum TA_FLAT_ATOMIC_WAVEFRONTS_sum TA_BUFFER_ATOMIC_WAVEFRONTS_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d "$OUT/p$i" -o run -- "${P[@]}" > "$OUT/p$i.log" 2>&1
done
python3 tools/pmc_kernels.py "$OUT" > "$OUT/summary.txt"
