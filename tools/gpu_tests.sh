#!/usr/bin/env bash
# GPU test pass + bench + kernel-trace profile (run ON the GPU box from the
# repo root):  bash tools/gpu_tests.sh TAG [pytest -k expr]
set -eo pipefail
export TMPDIR=/tmp
D=gpurun_out/${1:-r02}
mkdir -p $D
K=${2:+-k "$2"}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread $K > $D/gpu_tests.log 2>&1
timeout -k 10 300 python -u bench.py > $D/bench.json 2> $D/bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-pcie > $D/prof.log 2>&1
echo done
