# End-to-end A/B: bench.py ms_per_step per library variant, alternating (run ON the GPU box):
#   bash tools/ab_bench.sh OUT variant...   ("base" = the in-tree build; "v@N": with MSA_ABLATE=N -- a -DMSA_DIAG=1 variant build)
set -e
out=gpurun_out/$1; shift
mkdir -p gpurun_out
: > $out.log
for vv in "$@"; do
  v=${vv%@*}; ab=0; [ "$vv" != "$v" ] && ab=${vv#*@}
  if [ "$v" = base ]; then L=$PWD/music-analyst-ai_amd/libmsa_hip.so; else L=$PWD/music-analyst-ai_amd/variants/libmsa_hip_$v.so; fi
  MSA_ABLATE=$ab MSA_LIB=$L timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-pcie > $out.$v.json 2>> $out.err
  python3 -c "import json,sys; d=json.load(open('$out.$v.json')); print('$vv', d['ms_per_step'], d['value'], d['roofline']['avg_launch_ms'], json.dumps(d['stage_ms']))" >> $out.log
done
echo done >> $out.log
