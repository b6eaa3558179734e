# configs[4]-scale rank-layer world of one (MSA_RANK_PATH=1): this build
# (self block copied, not sent through RCCL) vs the round-5 build with the
# RCCL / shm transports; the single-context table path (MSA_DENSE=0) vs the oracle.
set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/r06_diag3
mkdir -p $D
W=/tmp/msa_diag; mkdir -p $W
music-analyst-ai_amd/bin/msa_gen $W/hc.csv --songs 4100000 --seed 4 --mode highcard > /dev/null
timeout -k 10 300 oracle/msa_oracle $W/hc.csv --output-dir $W/o > /dev/null
for v in "cur:music-analyst-ai_amd/bin/parallel_spotify:MSA_TRANSPORT=rccl" "r5_shm:music-analyst-ai_amd/variants/r5/bin/parallel_spotify:MSA_TRANSPORT=shm" "cur_shm:music-analyst-ai_amd/bin/parallel_spotify:MSA_TRANSPORT=shm"; do
  name=${v%%:*}; rest=${v#*:}; B=${rest%%:*}; e=${rest#*:}
  rm -rf $W/g
  env MSA_RANK_PATH=1 $e timeout -k 10 200 $B $W/hc.csv --output-dir $W/g > $D/$name.out 2> $D/$name.err
  rc=$?
  echo "$name rc=$rc words=$(cmp -s $W/g/word_counts.csv $W/o/word_counts.csv && echo same || echo DIFF) artists=$(cmp -s $W/g/top_artists.csv $W/o/top_artists.csv && echo same || echo DIFF) $(tail -1 $D/$name.err)" >> $D/diag.txt
done
rm -rf $W
MSA_DENSE=0 timeout -k 10 400 python3 tools/highcard_bench.py 4100000 --oracle --steps 1 > $D/hc_table.txt 2>&1
echo "single-context table path rc=$? $(tail -1 $D/hc_table.txt)" >> $D/diag.txt
echo done >> $D/diag.txt
