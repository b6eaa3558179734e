set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/r06_kal
mkdir -p $D
L=$PWD/music-analyst-ai_amd/variants/libmsa_hip_kal.so
MSA_LIB=$L timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $D/parity_kal.log 2>&1
echo "parity rc=$?" >> $D/summary.txt
for v in base kal; do
  if [ $v = base ]; then LL=$PWD/music-analyst-ai_amd/libmsa_hip.so; else LL=$L; fi
  MSA_LIB=$LL timeout -s KILL 150 rocprofv3 --pmc TD_TD_BUSY_sum TD_BUSY_max TA_TA_BUSY_sum TA_BUSY_max --output-format csv -d $D/pmc_$v -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-pcie > $D/pmc_$v.log 2>&1
  python3 tools/pmc_kernels.py $D/pmc_$v k_scan_tokens >> $D/summary.txt 2>&1
done
bash tools/ab_bench.sh r06_kal/ab base kal base kal
