# Per-song counter: variants against the in-tree build with the wrows
# kernel's memory-side atomics and writes (run ON the GPU box):
#   bash tools/wcs_ab_pmc.sh TAG variant...
# wcs GPU tests on the in-tree build, one PMC pass per build
# (TCC_EA0_ATOMIC_sum + WRITE_SIZE), then bench_wcs legs alternating twice.
set -eo pipefail
export TMPDIR=/tmp
D=gpurun_out/$1; shift
mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_gpu_wcs.py tests/test_gpu_split.py -x -q --timeout 120 --timeout-method thread > $D/tests.log 2>&1
echo "tests ok" > $D/summary.txt
lib() { if [ "$1" = base ]; then echo $PWD/music-analyst-ai_amd/libmsa_hip.so; else echo $PWD/music-analyst-ai_amd/variants/libmsa_hip_$1.so; fi; }
for v in base "$@"; do
  MSA_LIB=$(lib $v) timeout -s KILL 150 rocprofv3 --pmc TCC_EA0_ATOMIC_sum WRITE_SIZE --output-format csv -d $D/pmc_$v -o run -- python3 tools/bench_wcs.py --steps 1 --warmup 1 --no-cpu-baseline > $D/pmc_$v.log 2>&1
  echo "== $v" >> $D/summary.txt
  LAST=1 python3 tools/pmc_kernels.py $D/pmc_$v k_wcs_wrows >> $D/summary.txt 2>&1
done
for r in 1 2; do
  for v in base "$@"; do
    MSA_LIB=$(lib $v) timeout -k 10 200 python -u tools/bench_wcs.py --no-cpu-baseline > $D/$v.$r.json 2> $D/$v.$r.err
    python3 -c "import json; d=json.load(open('$D/$v.$r.json')); print('$v', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])" >> $D/summary.txt
  done
done
echo done >> $D/summary.txt
