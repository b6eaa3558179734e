# Whole GPU suite, then the quick baseline (bench without the CPU leg + one
# kernel-trace timeline) -- run ON the GPU box from the repo root:
#   bash tools/gpu_check.sh TAG [pytest args...]
# Every GPU step has its own time limit; a crash or time limit ends the script.
set -o pipefail
export TMPDIR=/tmp
T=${1:-check}; shift
D=gpurun_out/$T
mkdir -p $D
s=$(date +%s)
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread "$@" > $D/gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc seconds=$(( $(date +%s) - s ))" | tee -a $D/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_base.sh $T/base
