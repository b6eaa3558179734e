# Quick baseline on the GPU box: bench (no CPU leg) + one kernel-trace timeline.
#   bash tools/gpu_base.sh TAG
set -eo pipefail
export TMPDIR=/tmp
D=gpurun_out/${1:-base}
mkdir -p $D
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-pcie > $D/bench.json 2> $D/bench.err
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $D/prof -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-pcie > $D/prof.log 2>&1
python3 tools/timeline.py $D/prof > $D/timeline.txt
echo done
