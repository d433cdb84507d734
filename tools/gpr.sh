#!/bin/bash
# gpurun, retried only while no GPU slot is free (status=transient / rc 3: nothing ran, nothing charged)
to=$1; shift
for a in $(seq 1 ${GPR_TRIES:-10}); do
  out=$(/usr/local/graft/bin/gpurun --timeout $to -- "$@" 2>&1); rc=$?
  if echo "$out" | grep -q "status=transient" || [ $rc -eq 3 ]; then sleep ${GPR_SLEEP:-150}; continue; fi
  echo "$out"; exit $rc
done
echo "$out"; exit $rc
