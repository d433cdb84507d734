#!/bin/bash
# r05: config-4 host phases (LGS_STEP_TIMING) and a kernel trace of the frontend
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
tools/gpu_step.sh "st_timing|300|LGS_STEP_TIMING=1 python -u bench.py --workload stream --steps 2000 --warmup 100 --no-cpu > gpurun_out/r05j_stream.json 2> gpurun_out/r05j_stream.err" \
  "st_trace|300|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r05j_trace -o run -- python3 bench.py --workload stream --steps 1000 --warmup 50 --no-cpu > gpurun_out/r05j_trace.log 2>&1"
