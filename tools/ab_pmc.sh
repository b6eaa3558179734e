# The in-tree build against a variant (run ON the GPU box):
#   bash tools/ab_pmc.sh TAG VARIANT [pytest files...]
# parity files with the in-tree build, per build the write / LDS counters of
# the split's kernels (one rocprofv3 pass per group), then alternating bench
# pairs (tools/ab_bench.sh).  Every GPU step has its own time limit.
set -eo pipefail
export TMPDIR=/tmp
T=$1; V=$2; shift 2
D=gpurun_out/$T
mkdir -p $D
F=${*:-tests/test_gpu_parity.py}
timeout -k 10 600 python -u -m pytest $F -x -q --timeout 300 --timeout-method thread > $D/parity.log 2>&1
echo "parity ok" >> $D/summary.txt
for v in base $V; do
  if [ $v = base ]; then LL=$PWD/music-analyst-ai_amd/libmsa_hip.so; else LL=$PWD/music-analyst-ai_amd/variants/libmsa_hip_$v.so; fi
  MSA_LIB=$LL timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $D/pmcw_$v -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-pcie > $D/pmcw_$v.log 2>&1
  MSA_LIB=$LL timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAVE_CYCLES --output-format csv -d $D/pmcq_$v -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-pcie > $D/pmcq_$v.log 2>&1
  echo "== $v" >> $D/summary.txt
  LAST=1 python3 tools/pmc_kernels.py $D/pmcw_$v k_scan_tokens >> $D/summary.txt 2>&1
  LAST=1 python3 tools/pmc_kernels.py $D/pmcw_$v k_miss_agg >> $D/summary.txt 2>&1
  LAST=1 python3 tools/pmc_kernels.py $D/pmcq_$v k_scan_tokens >> $D/summary.txt 2>&1
done
bash tools/ab_bench.sh $T/ab base $V base $V
