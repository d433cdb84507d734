#!/bin/bash
# r05: seed candidates picked by one wave in the one-launch seed too -- matcher tests, p50 of lone calls, bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
B="python -u bench.py --no-cpu --sub-lines 0 --loop-line 0 --dropin-line 0 --latency-calls 300"
tools/gpu_step.sh "k_tests|400|python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_benchcfg.py tests/test_gpu_batch.py tests/test_gpu_rtcsm.py tests/test_gpu_loop.py tests/test_gpu_bb.py" \
  "b1|300|$B > gpurun_out/r05v_b1.json 2> gpurun_out/r05v_b1.err" \
  "b2|300|$B > gpurun_out/r05v_b2.json 2> gpurun_out/r05v_b2.err"
