#!/usr/bin/env bash
# PMC passes over the configs[4]-scale bench (tools/highcard_bench.py, 4.1 M
# songs, seed 4), one rocprofv3 run per counter group as tools/pmc.sh does
# (run ON the GPU box from the repo root).  Per-kernel means: tools/pmc_fold.py.
set -euo pipefail
export TMPDIR=/tmp
OUT=${1:-gpurun_out/pmc_hc}
mkdir -p "$OUT"
B=(python3 tools/highcard_bench.py 4100000 --steps 1)
pass() {  # name counters...
  local name=$1; shift
  timeout -s KILL 240 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/$name" -o run -- "${B[@]}" > "$OUT/$name.log" 2>&1
}
pass sq SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY
pass atomic TCC_ATOMIC_sum TCC_EA0_ATOMIC_sum TA_FLAT_ATOMIC_WAVEFRONTS_sum TA_BUFFER_ATOMIC_WAVEFRONTS_sum SQ_INSTS_LDS_ATOMIC
pass sq2 SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY
pass write WRITE_SIZE
pass fetch FETCH_SIZE
