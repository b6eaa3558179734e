#!/bin/bash
# run a gpurun command, retrying only while the pool reports no free slot/box (nothing ran, nothing charged)
# usage: gpu_retry.sh LOG TIMEOUT 'command'
log=$1; to=$2; cmd=$3
for i in 1 2 3 4 5 6 7 8; do
  /usr/local/graft/bin/gpurun --timeout $to -- "$cmd" > $log 2>&1
  if grep -q "status=transient" $log; then sleep 90; continue; fi
  break
done
echo "__done__" >> $log
