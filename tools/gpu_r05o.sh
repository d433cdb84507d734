#!/bin/bash
# r05: wide seed candidates 8 / 12 / 16 (A/B), parity of the batch tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
B="python -u bench.py --no-cpu --sub-lines 0 --loop-line 0 --dropin-line 0"
tools/gpu_step.sh "k_tests|300|python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_batch.py tests/test_gpu_rtcsm.py tests/test_gpu_loop.py" \
  "w8|300|LGS_CTX_OPTIONS=32=8 $B > gpurun_out/r05o_w8.json 2> gpurun_out/r05o_w8.err" \
  "w12|300|LGS_CTX_OPTIONS=32=12 $B > gpurun_out/r05o_w12.json 2> gpurun_out/r05o_w12.err" \
  "w16|300|$B > gpurun_out/r05o_w16.json 2> gpurun_out/r05o_w16.err" \
  "w8b|300|LGS_CTX_OPTIONS=32=8 $B > gpurun_out/r05o_w8b.json 2> gpurun_out/r05o_w8b.err"
