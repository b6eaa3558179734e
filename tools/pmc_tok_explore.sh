# Exploratory PMC passes on the split scan (bench.py 1 step): latency and
# texture-unit counters of k_scan_tokens (run ON the GPU box).
set -o pipefail
export TMPDIR=/tmp
OUT=${1:-gpurun_out/pmc_tok}
mkdir -p "$OUT"
timeout -s KILL 60 rocprofv3 -L > "$OUT/avail.txt" 2>&1 || true
B=(python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-pcie)
pass() {
  local name=$1; shift
  timeout -s KILL 150 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/$name" -o run -- "${B[@]}" > "$OUT/$name.log" 2>&1 || echo "pass $name failed" >> "$OUT/fail.txt"
}
pass lat SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM SQ_INST_LEVEL_LDS SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAVE_CYCLES
pass ta TA_TA_BUSY_sum TA_BUSY_max
pass td TD_TD_BUSY_sum TD_BUSY_max
pass tcp TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum
pass tcc TCC_HIT_sum TCC_MISS_sum
echo done > "$OUT/done.txt"
