# round 4: the spans-beside race after the ensure(zero) sync fix
export TMPDIR=/tmp; D=gpurun_out/r04_t6b; mkdir -p $D
run() { local name=$1; shift; env "$@" timeout -k 10 200 python -u tools/dbg_shards.py $D/$name 5 highcard 6000 5 > $D/$name.log 2>&1; }
run b1 MSA_K3SPLIT=1 && run b2 MSA_K3SPLIT=1 && run b3 MSA_K3SPLIT=1 && run b4 MSA_K3SPLIT=1
rm -f $D/*/in.csv
