#!/bin/bash
# r04 closing check: smoke() and the default bench line (roofline traffic from profiles/pmc_summary.json)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
tools/gpu_step.sh "smoke|300|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "bench|600|python -u bench.py > gpurun_out/r04_close_bench.json 2> gpurun_out/r04_close_bench.err" || exit $?
python3 -c "import json;d=json.loads(open('gpurun_out/r04_close_bench.json').read().strip().splitlines()[-1]);print(d['value'], d['roofline'])"
