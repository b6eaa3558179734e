# configs[4]-class corpus through the C host's bench mode (rank processes,
# shm transport on a one-GPU box), dense word entries vs the table path:
#   bash tools/chost_highcard.sh TAG [songs]
set -eo pipefail
export TMPDIR=/tmp
D=gpurun_out/${1:-chost_hc}
mkdir -p $D
S=${2:-4100000}
B=music-analyst-ai_amd/bin/parallel_spotify
run() {  # name procs env...
  local name=$1 np=$2; shift 2
  env "$@" timeout -k 10 300 $B - --synthetic-songs $S --synthetic-mode highcard --synthetic-seed 4 --processes $np \
      --bench-steps 5 --bench-warmup 2 --output-dir /tmp/msa_chost_hc > $D/$name.json 2> $D/$name.err
  python3 -c "import json; d=json.loads([l for l in open('$D/$name.json') if l.startswith('{')][-1]); s=d['seconds']/d['steps']; print('$name', 'ranks', d['ranks'], 'ms/step', round(s*1e3,2), 'GB/s', round(d['bytes_total']/s/1e9,1))" >> $D/summary.txt
}
: > $D/summary.txt
run np1_dense 1 MSA_RANK_PATH=1
run np1_table 1 MSA_RANK_PATH=1 MSA_DENSE=0
run np2_dense 2
run np2_table 2 MSA_DENSE=0
run np2_dense_b 2
run np2_table_b 2 MSA_DENSE=0
echo done >> $D/summary.txt
