#!/bin/bash
# r05: loop-batch kernel trace (config 5) and the scaling probe on the final library
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
tools/gpu_step.sh "loop_trace|300|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r05s_loop_trace -o run -- python3 bench.py --workload loop --no-cpu > gpurun_out/r05s_loop_trace.log 2>&1" \
  "probe|600|python -u tools/scaling_probe.py --out gpurun_out/r05s_scaling_probe.json > gpurun_out/probe.log 2>&1"
