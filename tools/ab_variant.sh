# A variant of libmsa_hip against the in-tree build (run ON the GPU box):
#   bash tools/ab_variant.sh TAG VARIANT
# parity subset with the variant (MSA_LIB), the token pass's texture-unit
# counters of both, then alternating bench pairs (tools/ab_bench.sh).
set -o pipefail
export TMPDIR=/tmp
T=$1; V=$2
D=gpurun_out/$T
mkdir -p $D
L=$PWD/music-analyst-ai_amd/variants/libmsa_hip_$V.so
MSA_LIB=$L timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $D/parity_$V.log 2>&1
rc=$?
echo "parity rc=$rc" >> $D/summary.txt
[ $rc -eq 0 ] || exit $rc
for v in base $V; do
  if [ $v = base ]; then LL=$PWD/music-analyst-ai_amd/libmsa_hip.so; else LL=$L; fi
  MSA_LIB=$LL timeout -s KILL 150 rocprofv3 --pmc TD_TD_BUSY_sum TD_BUSY_max TA_TA_BUSY_sum TA_BUSY_max --output-format csv -d $D/pmc_$v -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-pcie > $D/pmc_$v.log 2>&1
  echo "== $v" >> $D/summary.txt
  python3 tools/pmc_kernels.py $D/pmc_$v k_scan >> $D/summary.txt 2>&1
done
bash tools/ab_bench.sh $T/ab base $V base $V
