set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/wcs1
for v in 0; do
  MSA_WCS_ABLATE=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/wcs1/p$v -o run -- python3 tools/bench_wcs.py --songs 2000000 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/wcs1/b$v.log 2>&1
done
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY --output-format csv -d gpurun_out/wcs1/pmc1 -o run -- python3 tools/bench_wcs.py --songs 2000000 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/wcs1/pmc1.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/wcs1/pmc2 -o run -- python3 tools/bench_wcs.py --songs 2000000 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/wcs1/pmc2.log 2>&1
python3 tools/pmc_kernels.py gpurun_out/wcs1 k_wcs_wrows > gpurun_out/wcs1/summary.txt
echo done
