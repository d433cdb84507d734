#!/bin/bash
# r02 first GPU pass: determinism diagnostics, then the -m gpu suite.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/diag_determinism.py > gpurun_out/r02_det.log 2>&1 &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02_gpu_tests.log 2>&1
