#!/bin/bash
# r03: two-bank chunk pipelining: parity suites, then config-2 bench lines for
# 1 vs 2 streams and 64/128/256 queries per call (no CPU leg, no side lines).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=gpurun_out/r03e; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_batch.py tests/test_gpu_rtcsm.py \
    tests/test_gpu_loop.py tests/test_gpu_bb.py tests/test_gpu_keysort.py tests/test_gpu_latest.py tests/test_gpu_frontend.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for cfg in "1 128" "1 256" "2 128" "1 64" "2 64"; do
  set -- $cfg
  timeout -k 10 200 python -u bench.py --streams $1 --batch $2 --steps 240 --no-cpu --loop-line 0 --dropin-line 0 --latency-calls 0 > $O/s$1_b$2.json 2> $O/s$1_b$2.err || { tail -5 $O/s$1_b$2.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/s$1_b$2.json').read().strip().splitlines()[-1]);r=d['roofline'];ri=d['roofline_isolated'];print('streams $1 batch $2:', d['value'], r['avg_launch_ms'], r['frac'], ri['avg_launch_ms'], ri['frac'])"
done
