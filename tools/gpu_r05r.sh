#!/bin/bash
# r05: one-launch wide seed for lone matches -- matcher tests, p50 A/B (lone wide on / off)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
B="python -u bench.py --no-cpu --sub-lines 0 --loop-line 0 --dropin-line 0 --latency-calls 300"
tools/gpu_step.sh "k_tests|400|python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_benchcfg.py tests/test_gpu_batch.py tests/test_gpu_rtcsm.py tests/test_gpu_frontend.py" \
  "lone_on|300|$B > gpurun_out/r05r_on.json 2> gpurun_out/r05r_on.err" \
  "lone_off|300|LGS_CTX_OPTIONS=33=0 $B > gpurun_out/r05r_off.json 2> gpurun_out/r05r_off.err" \
  "lone_on2|300|$B > gpurun_out/r05r_on2.json 2> gpurun_out/r05r_on2.err" \
  "st_on|300|python -u bench.py --workload stream --steps 2000 --warmup 100 --no-cpu > gpurun_out/r05r_st.json 2> gpurun_out/r05r_st.err"
