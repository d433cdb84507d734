#!/bin/bash
# tests, then A/B bench lines: gpu_ab.sh <tag> "<bench args A>" "<bench args B>"
set -o pipefail
mkdir -p gpurun_out
TAG=$1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 &&
timeout -k 10 300 python -u bench.py --no-cpu --loop-line 0 $2 > gpurun_out/${TAG}_a.json 2> gpurun_out/${TAG}_a.err &&
timeout -k 10 300 python -u bench.py --no-cpu --loop-line 0 $3 > gpurun_out/${TAG}_b.json 2> gpurun_out/${TAG}_b.err
