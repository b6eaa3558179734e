# configs[4] A/B of an environment switch (run ON the GPU box):
#   bash tools/ab_env_hc.sh TAG VAR "val1 val2" [songs]
# tools/highcard_bench.py 3 steps per leg, legs alternating twice.
set -eo pipefail
D=gpurun_out/$1; V=$2; VALS=$3; S=${4:-4100000}
mkdir -p $D
for r in 1 2; do
  for v in $VALS; do
    echo "== $V=$v" >> $D/hc.txt
    env $V=$v timeout -k 10 300 python -u tools/highcard_bench.py $S --steps 3 >> $D/hc.txt 2>&1
  done
done
echo done >> $D/hc.txt
