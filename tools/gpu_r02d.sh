#!/bin/bash
# r02 pass d: -m gpu suite, stream diagnostics, config-4 lines
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r02d_gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python -u tools/diag_stream.py > gpurun_out/r02d_diag_stream.log 2>&1 &&
TAG=r02d STEPS=300 bash tools/gpu_stream.sh
