#!/bin/bash
# r03 re-entry: full GPU parity suite, smoke, default bench line, then the
# config-5 (loop) profile (tools/gpu_prof_loop.sh).  Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=gpurun_out/r03c; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -10 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -10 $O/bench.err; exit 1; }
tail -c 600 $O/bench.json
bash tools/gpu_prof_loop.sh r03c
