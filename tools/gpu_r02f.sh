#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r02f_gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
DIAG_STEPS=310 DIAG_SLOW_MS=0.6 timeout -k 10 300 python -u tools/diag_stream.py 4.0,4.0,1.0471976 odo > gpurun_out/r02f_diag.log 2>&1 &&
TAG=r02f STEPS=300 bash tools/gpu_stream.sh
