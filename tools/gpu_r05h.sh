#!/bin/bash
# r05: full GPU suite + smoke + default bench line
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
tools/gpu_step.sh "gputests|900|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "smoke|300|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "bench|900|python -u bench.py > gpurun_out/r05h_bench.json 2> gpurun_out/r05h_bench.err"
