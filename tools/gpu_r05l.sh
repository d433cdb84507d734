#!/bin/bash
# r05: cooperative-sort reservations and the map writer by completion words
# (no stream events), host hit points through the four-lane sincos -- the full
# GPU suite, config 4 timing + trace, the default bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
tools/gpu_step.sh "gputests|600|python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests" \
  "st_timing|300|LGS_STEP_TIMING=1 python -u bench.py --workload stream --steps 2000 --warmup 100 --no-cpu > gpurun_out/r05l_timing.json 2> gpurun_out/r05l_timing.err" \
  "st_trace|300|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r05l_trace -o run -- python3 bench.py --workload stream --steps 1000 --warmup 50 --no-cpu > gpurun_out/r05l_trace.log 2>&1" \
  "bench|400|python -u bench.py > gpurun_out/r05l_bench.json 2> gpurun_out/r05l_bench.err"
