#!/bin/bash
# r03: GPU tests touching the scan pool / stamp-only angle flags, then the config-4 stream line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=gpurun_out/r03h; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_batch.py tests/test_gpu_rtcsm.py tests/test_gpu_latest.py tests/test_gpu_frontend.py tests/test_gpu_loop.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 300 python -u bench.py --workload stream > $O/stream.json 2> $O/stream.err || { tail -5 $O/stream.err; exit 1; }
tail -c 700 $O/stream.json
timeout -k 10 300 python -u bench.py > $O/match.json 2> $O/match.err || { tail -5 $O/match.err; exit 1; }
tail -c 700 $O/match.json
