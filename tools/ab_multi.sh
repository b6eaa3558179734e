# Several libmsa_hip variants against the in-tree build (run ON the GPU box):
#   bash tools/ab_multi.sh TAG VARIANT...
# per variant the parity subset (tests/test_gpu_parity.py through MSA_LIB; a
# failing variant is dropped), the texture-unit counters of the split-scan
# kernels, then alternating bench rounds of every surviving build.
set -o pipefail
export TMPDIR=/tmp
T=$1; shift
D=gpurun_out/$T
mkdir -p $D
ok=(base)
for V in "$@"; do
  L=$PWD/music-analyst-ai_amd/variants/libmsa_hip_$V.so
  MSA_LIB=$L timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $D/parity_$V.log 2>&1
  rc=$?
  echo "parity $V rc=$rc" >> $D/summary.txt
  [ $rc -eq 124 ] || [ $rc -eq 137 ] && exit $rc
  [ $rc -eq 0 ] && ok+=($V)
done
for v in "${ok[@]}"; do
  if [ $v = base ]; then LL=$PWD/music-analyst-ai_amd/libmsa_hip.so; else LL=$PWD/music-analyst-ai_amd/variants/libmsa_hip_$v.so; fi
  MSA_LIB=$LL timeout -s KILL 150 rocprofv3 --pmc TD_TD_BUSY_sum TD_BUSY_max TA_TA_BUSY_sum TA_BUSY_max --output-format csv -d $D/pmc_$v -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-pcie > $D/pmc_$v.log 2>&1 || exit $?
  echo "== $v" >> $D/summary.txt
  python3 tools/pmc_kernels.py $D/pmc_$v "k_" 2>&1 | grep -A4 -E "^(k_scan_tokens|k_scan_struct|k_chunk_summary)" >> $D/summary.txt
done
bash tools/ab_bench.sh $T/ab "${ok[@]}" "${ok[@]}"
