# Column splitter: variants of libmsa_hip against the in-tree build (run ON the GPU box):
#   bash tools/split_ab.sh TAG variant...   -- bench_wcs.py --path split legs, alternating twice,
# plus one WRITE_SIZE pass of k_csvcol<1> per build
set -eo pipefail
export TMPDIR=/tmp
D=gpurun_out/$1; shift
mkdir -p $D
lib() { if [ "$1" = base ]; then echo $PWD/music-analyst-ai_amd/libmsa_hip.so; else echo $PWD/music-analyst-ai_amd/variants/libmsa_hip_$1.so; fi; }
: > $D/summary.txt
for r in 1 2; do
  for v in base "$@"; do
    MSA_LIB=$(lib $v) timeout -k 10 200 python -u tools/bench_wcs.py --path split --no-cpu-baseline > $D/$v.$r.json 2> $D/$v.$r.err
    python3 -c "import json; d=json.load(open('$D/$v.$r.json')); print('$v', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])" >> $D/summary.txt
  done
done
for v in base "$@"; do
  MSA_LIB=$(lib $v) timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $D/pmc_$v -o run -- python3 tools/bench_wcs.py --path split --steps 1 --warmup 1 --no-cpu-baseline > $D/pmc_$v.log 2>&1
  echo "== $v" >> $D/summary.txt
  LAST=1 python3 tools/pmc_kernels.py $D/pmc_$v "k_csvcol<1>" >> $D/summary.txt 2>&1 || true
done
echo done >> $D/summary.txt
