# bisect test_sharded_gather_corank[5-highcard]: fused vs split scan.
# A failing test (rc 1) lets the next step run; a timeout/abort/segfault ends the script.
export TMPDIR=/tmp; D=gpurun_out/r04_t3; mkdir -p $D
step() {  # name env...
  local name=$1; shift
  env "$@" timeout -k 10 200 python -u -m pytest tests/test_gpu_dist.py -x -q --timeout 150 --timeout-method thread -k "corank" > $D/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc" >> $D/rc.txt
  case $rc in 0|1) return 0;; *) return 1;; esac
}
step fused MSA_K3SPLIT=0 && step split MSA_K3SPLIT=1 && step split_noov MSA_ABLATE=8192
cat $D/rc.txt
