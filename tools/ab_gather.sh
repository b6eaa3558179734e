# text.csv gather variants (k_col_gather is shared by the counter's text.csv and
# the column splitter): run ON the GPU box:  bash tools/ab_gather.sh TAG VARIANT
# parity (counter + CLI + splitter tests) with the variant, then alternating
# bench.py pairs (tools/ab_bench.sh) and splitter legs (tools/split_ab.sh).
set -eo pipefail
export TMPDIR=/tmp
T=$1; V=$2
D=gpurun_out/$T
mkdir -p $D
MSA_LIB=$PWD/music-analyst-ai_amd/variants/libmsa_hip_$V.so timeout -k 10 600 python -u -m pytest \
    tests/test_gpu_parity.py tests/test_gpu_cli.py tests/test_gpu_split.py -x -q --timeout 300 \
    --timeout-method thread > $D/parity_$V.log 2>&1
tail -1 $D/parity_$V.log > $D/parity.txt
bash tools/ab_bench.sh $T/ab base $V base $V
bash tools/split_ab.sh $T/split $V
