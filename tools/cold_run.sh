# One-shot (cold) runs of the drop-in CLI, as the reference's own harness
# times it (run_performance.sh: one `mpirun -np N bin/parallel_spotify` per N,
# performance_metrics.json's total_time).  Run ON the GPU box from the repo root:
#   bash tools/cold_run.sh TAG
# configs[2] (5 M zipf songs, seed 1) and configs[4] (4.1 M highcard songs,
# seed 4) written to files; per file: two fresh processes of
# bin/parallel_spotify (wall clock + total_time), a rocprofv3 kernel + HIP
# runtime trace of one more cold run; the reference (`mpirun -np 2`) on the
# configs[2] file.  Every GPU step has its own time limit.
set -eo pipefail
export TMPDIR=/tmp
D=gpurun_out/${1:-cold}
mkdir -p $D
W=/tmp/msa_cold
rm -rf $W && mkdir -p $W
B=music-analyst-ai_amd/bin
$B/msa_gen $W/c2.csv --songs 5000000 --seed 1 > /dev/null
$B/msa_gen $W/c4.csv --songs 4100000 --seed 4 --mode highcard > /dev/null
ls -l $W/c2.csv $W/c4.csv > $D/files.txt
for cfg in c2 c4; do
  for i in 1 2; do
    rm -rf $W/o_$cfg
    s=$(date +%s.%N)
    timeout -k 10 120 $B/parallel_spotify $W/$cfg.csv --output-dir $W/o_$cfg > $D/${cfg}_run$i.out 2> $D/${cfg}_run$i.err
    e=$(date +%s.%N)
    echo "$cfg run $i wall $(python3 -c "print(round($e - $s, 3))") s" >> $D/cold.txt
    python3 -c "import json; m=json.load(open('$W/o_$cfg/performance_metrics.json')); print('$cfg run $i', 'compute', m['compute_time']['max_seconds'], 'total', m['total_time']['max_seconds'])" >> $D/cold.txt
  done
  cp $W/o_$cfg/performance_metrics.json $D/${cfg}_performance_metrics.json
  rm -rf $W/o_$cfg
  timeout -k 10 180 rocprofv3 --kernel-trace --runtime-trace --stats --output-format csv -d $D/prof_$cfg -o run -- \
      $B/parallel_spotify $W/$cfg.csv --output-dir $W/o_$cfg > $D/prof_$cfg.log 2>&1
  python3 -c "import json; m=json.load(open('$W/o_$cfg/performance_metrics.json')); print('$cfg traced', 'compute', m['compute_time']['max_seconds'], 'total', m['total_time']['max_seconds'])" >> $D/cold.txt
  rm -rf $W/o_$cfg
done
# the reference at np=2 on the configs[2] file (its own total_time excludes its split)
if [ -x oracle/_ref/parallel_spotify ]; then
  s=$(date +%s.%N)
  PATH=/opt/conda/bin:$PATH timeout -k 10 300 mpirun -np 2 oracle/_ref/parallel_spotify $W/c2.csv --output-dir $W/ref_c2 > $D/ref_c2.out 2> $D/ref_c2.err
  e=$(date +%s.%N)
  echo "reference np2 c2 wall $(python3 -c "print(round($e - $s, 3))") s" >> $D/cold.txt
  python3 -c "import json; m=json.load(open('$W/ref_c2/performance_metrics.json')); print('reference np2 c2', 'compute', m['compute_time']['max_seconds'], 'total', m['total_time']['max_seconds'])" >> $D/cold.txt
  cp $W/ref_c2/performance_metrics.json $D/ref_c2_performance_metrics.json
fi
rm -rf $W
echo done >> $D/cold.txt
