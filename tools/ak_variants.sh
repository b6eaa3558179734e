set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/ak
for v in base akA akB akC; do
  if [ $v = base ]; then L=music-analyst-ai_amd/libmsa_hip.so; else L=var_so/libmsa_hip_$v.so; fi
  MSA_LIB=$L timeout -k 10 200 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/ak/$v.json 2> gpurun_out/ak/$v.err
done
echo done
