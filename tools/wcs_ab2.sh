# Per-song counter + column splitter: the in-tree build against a variant
# (run ON the GPU box):  bash tools/wcs_ab2.sh TAG VARIANT
# their GPU tests on the in-tree build, then bench_wcs legs (both paths)
# alternating twice.
set -eo pipefail
export TMPDIR=/tmp
D=gpurun_out/$1; V=$2
mkdir -p $D
timeout -k 10 500 python -u -m pytest tests/test_gpu_wcs.py tests/test_gpu_split.py -x -q --timeout 300 --timeout-method thread > $D/tests.log 2>&1
echo "tests ok" > $D/summary.txt
lib() { if [ "$1" = base ]; then echo $PWD/music-analyst-ai_amd/libmsa_hip.so; else echo $PWD/music-analyst-ai_amd/variants/libmsa_hip_$1.so; fi; }
for r in 1 2; do
  for v in base $V; do
    for path in wcs split; do
      MSA_LIB=$(lib $v) timeout -k 10 200 python -u tools/bench_wcs.py --path $path --no-cpu-baseline > $D/$v.$path.$r.json 2> $D/$v.$path.$r.err
      python3 -c "import json; d=json.load(open('$D/$v.$path.$r.json')); print('$v', '$path', d['value'], d['ms_per_step'])" >> $D/summary.txt
    done
  done
done
echo done >> $D/summary.txt
