# End-to-end A/B of environment settings on the in-tree build (run ON the GPU box):
#   bash tools/ab_env.sh OUT "NAME:VAR=V VAR2=V" ...   (alternating as given)
set -e
out=gpurun_out/$1; shift
mkdir -p gpurun_out
: > $out.log
for spec in "$@"; do
  name=${spec%%:*}; vars=${spec#*:}
  env $vars timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-pcie > $out.$name.json 2>> $out.err
  python3 -c "import json,sys; d=json.load(open('$out.$name.json')); print('$name', d['ms_per_step'], d['value'], d['roofline']['avg_launch_ms'], json.dumps(d['stage_ms']))" >> $out.log
done
echo done >> $out.log
