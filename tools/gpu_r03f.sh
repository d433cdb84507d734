#!/bin/bash
# r03: k_coarse_lanes exclusive per device (gate) vs free overlap, 2 streams x
# 128 queries, alternated runs; then the gated default under the kernel trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=gpurun_out/r03f; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_batch.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2 3; do
  for g in 1 0; do
    timeout -k 10 200 python -u bench.py --exclusive-coarse $g --steps 300 --no-cpu --loop-line 0 --dropin-line 0 --latency-calls 0 > $O/g${g}_$i.json 2> $O/g${g}_$i.err || { tail -5 $O/g${g}_$i.err; exit 1; }
    python3 -c "import json;d=json.loads(open('$O/g${g}_$i.json').read().strip().splitlines()[-1]);r=d['roofline'];ri=d['roofline_isolated'];print('gate $g run $i:', d['value'], r['avg_launch_ms'], r['frac'], ri['avg_launch_ms'], ri['frac'])"
  done
done
