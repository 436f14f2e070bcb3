#!/bin/bash
# usage: tools/gpu_retry.sh OUTFILE TIMEOUT 'command'   -- retries only while no box is free (rc 3)
out=$1; to=$2; cmd=$3
for i in $(seq 1 20); do
  /usr/local/graft/bin/gpurun --timeout $to -- "$cmd" > $out 2>&1
  rc=$?
  if [ $rc -ne 3 ] && ! grep -q "status=transient" $out; then break; fi
  sleep 150
done
echo "done rc=$rc" >> $out
