#!/bin/bash
# r05 baseline: GPU suite + default bench line
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
tools/gpu_step.sh "gputests|700|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "bench|600|python -u bench.py > gpurun_out/r05a_bench.json 2> gpurun_out/r05a_bench.err"
