#!/bin/bash
# r05: wide seed default (12 candidates) -- the full GPU suite, smoke, the default bench with sub-lines
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
tools/gpu_step.sh "gputests|600|python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests" \
  "smoke|120|python -u -c 'import __graft_entry__ as g; g.smoke()'" \
  "bench|500|python -u bench.py > gpurun_out/r05p_bench.json 2> gpurun_out/r05p_bench.err" \
  "bench_loop|300|python -u bench.py --workload loop --no-cpu > gpurun_out/r05p_loop.json 2> gpurun_out/r05p_loop.err"
