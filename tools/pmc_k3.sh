#!/usr/bin/env bash
# SQ/TCC counter passes over tools/ablate.py (5M songs, no ablation), one
# rocprofv3 run per pass (run ON the GPU box): bash tools/pmc_k3.sh OUT
set -euo pipefail
export TMPDIR=/tmp
OUT=${1:-gpurun_out/pmck3}
mkdir -p "$OUT"
P=(python3 tools/ablate.py 5000000 0)
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" \
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY" \
  "SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d "$OUT/p$i" -o run -- "${P[@]}" > "$OUT/p$i.log" 2>&1
done
python3 tools/pmc_kernels.py "$OUT" > "$OUT/summary.txt"
