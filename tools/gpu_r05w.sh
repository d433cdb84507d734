#!/bin/bash
# r05: concurrent contexts per GPU, 3 vs 4 vs 5 (A/B on one box)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
B="python -u bench.py --no-cpu --sub-lines 0 --loop-line 0 --dropin-line 0 --latency-calls 20"
tools/gpu_step.sh "s3|300|$B --streams 3 > gpurun_out/r05w_s3.json 2> gpurun_out/r05w_s3.err" \
  "s4|300|$B --streams 4 > gpurun_out/r05w_s4.json 2> gpurun_out/r05w_s4.err" \
  "s5|300|$B --streams 5 > gpurun_out/r05w_s5.json 2> gpurun_out/r05w_s5.err" \
  "s3b|300|$B --streams 3 > gpurun_out/r05w_s3b.json 2> gpurun_out/r05w_s3b.err" \
  "s4b|300|$B --streams 4 > gpurun_out/r05w_s4b.json 2> gpurun_out/r05w_s4b.err"
