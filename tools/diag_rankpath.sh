# Rank-layer (MSA_RANK_PATH=1, world of one) runs of the CLI on a configs[4]
# file, this build vs the round-5 build (variants/r5), against the oracle.
set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/r06_diag2
mkdir -p $D
W=/tmp/msa_diag; mkdir -p $W
music-analyst-ai_amd/bin/msa_gen $W/hc.csv --songs 4100000 --seed 4 --mode highcard > /dev/null
timeout -k 10 300 oracle/msa_oracle $W/hc.csv --output-dir $W/o > /dev/null
for v in "cur:music-analyst-ai_amd/bin/parallel_spotify:" "cur_table:music-analyst-ai_amd/bin/parallel_spotify:MSA_DENSE=0" "r5:music-analyst-ai_amd/variants/r5/bin/parallel_spotify:" "cur_np2:music-analyst-ai_amd/bin/parallel_spotify:NP2"; do
  name=${v%%:*}; rest=${v#*:}; B=${rest%%:*}; e=${rest#*:}
  rm -rf $W/g
  if [ "$e" = NP2 ]; then
    timeout -k 10 200 $B $W/hc.csv --output-dir $W/g --processes 2 > $D/$name.out 2> $D/$name.err
  else
    env MSA_RANK_PATH=1 $e timeout -k 10 200 $B $W/hc.csv --output-dir $W/g > $D/$name.out 2> $D/$name.err
  fi
  rc=$?
  echo "$name rc=$rc words=$(cmp -s $W/g/word_counts.csv $W/o/word_counts.csv && echo same || echo DIFF) artists=$(cmp -s $W/g/top_artists.csv $W/o/top_artists.csv && echo same || echo DIFF) $(tail -1 $D/$name.err)" >> $D/diag.txt
done
echo done >> $D/diag.txt
