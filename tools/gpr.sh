#!/bin/bash
# gpurun, retried only while no GPU slot is free (status=transient / rc 3: nothing ran, nothing charged)
to=$1; shift
for a in 1 2 3 4 5 6 7 8 9 10; do
  out=$(/usr/local/graft/bin/gpurun --timeout $to -- "$@" 2>&1); rc=$?
  if echo "$out" | grep -q "status=transient" || [ $rc -eq 3 ]; then sleep 150; continue; fi
  echo "$out"; exit $rc
done
echo "$out"; exit $rc
