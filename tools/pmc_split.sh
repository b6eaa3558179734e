#!/usr/bin/env bash
# PMC passes over the column-splitter bench (tools/bench_wcs.py --path split,
# the full 5M-song corpus), one rocprofv3 run per counter group as tools/pmc.sh
# does; tools/pmc_summary.py --split folds them into $OUT/pmc.json stamped
# with this build id (copy to profiles/pmc_split_main.json: bench_wcs.py
# --path split attaches k_csvcol<1>'s traffic only when the stamp matches).
set -euo pipefail
export TMPDIR=/tmp
OUT=${1:-gpurun_out/pmc_split}
mkdir -p "$OUT"
B=(python3 tools/bench_wcs.py --path split --steps 1 --warmup 1 --no-cpu-baseline)
pass() {  # name counters...
  local name=$1; shift
  timeout -s KILL 150 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/$name" -o run -- "${B[@]}" > "$OUT/$name.log" 2>&1
}
pass fetch FETCH_SIZE
pass write WRITE_SIZE
pass sq SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY
python3 tools/pmc_summary.py "$OUT" --split
