#!/bin/bash
# gpurun with retries ONLY while no box / slot is free (exit 3, nothing ran);
# any other outcome (success, failure, refusal) is final.
# usage: gpurun_retry.sh TIMEOUT 'command'
T=$1; shift
for i in $(seq 1 15); do
  /usr/local/graft/bin/gpurun --timeout $T -- "$@"
  rc=$?
  [ $rc -ne 3 ] && exit $rc
  grep -q "nothing was charged\|no free box" <<< "" ; sleep 120
done
exit 3
