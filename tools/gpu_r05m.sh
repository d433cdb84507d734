#!/bin/bash
# r05: seed-quality diagnostic (config 2) and the loop-batch scaling probe with
# the default one chunk per 64 candidates
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
tools/gpu_step.sh "diag_seed|200|python -u tools/diag_seed.py > gpurun_out/diag_seed.log 2>&1" \
  "probe|600|python -u tools/scaling_probe.py --out gpurun_out/r05m_scaling_probe.json > gpurun_out/probe.log 2>&1"
