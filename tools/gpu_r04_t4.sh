# per-rank local tables of the failing sharded case: split x3, split without the spans overlap x2
export TMPDIR=/tmp; D=gpurun_out/r04_t4b; mkdir -p $D
for v in s1 s2 s3; do MSA_K3SPLIT=1 timeout -k 10 200 python -u tools/dbg_shards.py $D/$v 5 highcard 6000 5 > $D/$v.log 2>&1 || exit 1; done
for v in n1 n2; do MSA_ABLATE=8192 timeout -k 10 200 python -u tools/dbg_shards.py $D/$v 5 highcard 6000 5 > $D/$v.log 2>&1 || exit 1; done
rm -f $D/*/in.csv
