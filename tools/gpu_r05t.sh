#!/bin/bash
# r05: k_post with all loads before the stores -- matcher tests, config 2 / 5 / 4 benches, loop trace
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
tools/gpu_step.sh "k_tests|400|python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_benchcfg.py tests/test_gpu_batch.py tests/test_gpu_rtcsm.py tests/test_gpu_loop.py tests/test_gpu_frontend.py" \
  "bench|300|python -u bench.py --no-cpu --sub-lines 0 --loop-line 0 --dropin-line 0 > gpurun_out/r05t_bench.json 2> gpurun_out/r05t_bench.err" \
  "loop|300|python -u bench.py --workload loop --no-cpu > gpurun_out/r05t_loop.json 2> gpurun_out/r05t_loop.err" \
  "stream|300|python -u bench.py --workload stream --steps 2000 --warmup 100 --no-cpu > gpurun_out/r05t_stream.json 2> gpurun_out/r05t_stream.err" \
  "loop_trace|300|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r05t_loop_trace -o run -- python3 bench.py --workload loop --no-cpu > gpurun_out/r05t_loop_trace.log 2>&1"
