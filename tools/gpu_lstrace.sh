#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out
LGS_LS_TRACE=1 timeout -k 10 120 python -u tools/ls_trace.py > gpurun_out/lstrace.log 2>&1
rc=$?
grep -c LSTRACE gpurun_out/lstrace.log
tail -60 gpurun_out/lstrace.log
exit $rc
