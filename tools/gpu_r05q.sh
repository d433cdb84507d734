#!/bin/bash
# r05: wide seed on the lone path too -- bench configuration tests, the default bench (p50 of lone calls)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
B="python -u bench.py --no-cpu --sub-lines 0 --loop-line 0 --dropin-line 0"
tools/gpu_step.sh "k_tests|400|python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_benchcfg.py tests/test_gpu_batch.py tests/test_gpu_rtcsm.py" \
  "b_wide|300|$B > gpurun_out/r05q_wide.json 2> gpurun_out/r05q_wide.err" \
  "b_lone_narrow|300|LGS_CTX_OPTIONS=32=0 $B > gpurun_out/r05q_narrow.json 2> gpurun_out/r05q_narrow.err"
