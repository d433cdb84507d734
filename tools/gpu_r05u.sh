#!/bin/bash
# r05: k_post sized to the records, supplied coarse maps decimated in one launch -- tests, loop bench + trace, stream
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
tools/gpu_step.sh "k_tests|400|python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_planes.py tests/test_gpu_loop.py tests/test_gpu_benchcfg.py tests/test_gpu_batch.py tests/test_gpu_rtcsm.py tests/test_gpu_frontend.py" \
  "loop|300|python -u bench.py --workload loop --no-cpu > gpurun_out/r05u_loop.json 2> gpurun_out/r05u_loop.err" \
  "stream|300|python -u bench.py --workload stream --steps 2000 --warmup 100 --no-cpu > gpurun_out/r05u_stream.json 2> gpurun_out/r05u_stream.err" \
  "loop_trace|300|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r05u_loop_trace -o run -- python3 bench.py --workload loop --no-cpu > gpurun_out/r05u_loop_trace.log 2>&1"
