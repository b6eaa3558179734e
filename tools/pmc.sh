#!/usr/bin/env bash
# PMC passes over bench.py (run ON the GPU box, from the repo root), one
# rocprofv3 run per counter group, as MI355X_MICROARCH.md prescribes
# (FETCH_SIZE takes 3 TCC slots, WRITE_SIZE 2: never in one pass):
#   fetch   FETCH_SIZE
#   write   WRITE_SIZE
#   sq      8 SQ counters (waves, cycles, VALU/LDS instructions, LDS bank conflicts, waits)
#   sq2     8 more SQ counters (instruction mix, active / waiting issue cycles)
#   atomic  TCC_ATOMIC_sum TCC_EA0_ATOMIC_sum (L2 / memory-side atomics),
#           TA_FLAT_ATOMIC_WAVEFRONTS_sum TA_BUFFER_ATOMIC_WAVEFRONTS_sum (issued),
#           SQ_INSTS_LDS_ATOMIC
# tools/pmc_summary.py then folds them, per kernel, into $OUT/pmc.json stamped
# with the sha256 of the libmsa_hip.so that ran (copy it to
# profiles/pmc_scan_main.json; bench.py only attaches `traffic` when the stamp
# matches the library it loaded).
set -euo pipefail
export TMPDIR=/tmp
OUT=${1:-gpurun_out/pmc}
STEPS=${STEPS:-1}
mkdir -p "$OUT"
B=(python3 bench.py --steps "$STEPS" --warmup 1 --no-cpu-baseline --no-pcie)
pass() {  # name counters...
  local name=$1; shift
  timeout -s KILL 150 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/$name" -o run -- "${B[@]}" > "$OUT/$name.log" 2>&1
}
pass fetch FETCH_SIZE
pass write WRITE_SIZE
pass sq SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY
pass atomic TCC_ATOMIC_sum TCC_EA0_ATOMIC_sum TA_FLAT_ATOMIC_WAVEFRONTS_sum TA_BUFFER_ATOMIC_WAVEFRONTS_sum SQ_INSTS_LDS_ATOMIC
# instruction mix and issue activity (SALU / scalar memory / vector memory, active VALU cycles)
pass sq2 SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY || true
python3 tools/pmc_summary.py "$OUT"
