# Round measurement set, part 2 of 2 (run ON the GPU box from the repo root):
#   bash tools/gpu_final6b.sh TAG
# the per-song counter's and the column splitter's PMC passes and benches,
# configs[4] stages, one-shot (cold) CLI runs.
set -eo pipefail
export TMPDIR=/tmp
D=gpurun_out/${1:-final6}
mkdir -p $D
bash tools/pmc_wcs.sh $D/pmc_wcs
cp $D/pmc_wcs/pmc.json profiles/pmc_wcs_main.json
cp $D/pmc_wcs/pmc.json $D/pmc_wcs_main.json
timeout -k 10 300 python -u tools/bench_wcs.py > $D/bench_wcs.json 2> $D/bench_wcs.err
bash tools/pmc_split.sh $D/pmc_split
cp $D/pmc_split/pmc.json profiles/pmc_split_main.json
cp $D/pmc_split/pmc.json $D/pmc_split_main.json
timeout -k 10 300 python -u tools/bench_wcs.py --path split > $D/bench_split.json 2> $D/bench_split.err
timeout -k 10 300 python -u tools/highcard_bench.py 4100000 --steps 5 > $D/highcard.txt 2>&1
bash tools/cold_run.sh ${1:-final6}/cold
echo done
