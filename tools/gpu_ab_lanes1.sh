#!/bin/bash
# r03 A/B (rejected): k_coarse_lanes with one wave per angle
# (LGS_LANES1=1 selected the variant kernel in the experiment build; the
# variant is not in the library).  Tests with the variant, then alternated
# config-2 and config-5 lines, then a rebuild-workload kernel trace.
cd "${GRAFT_REPO_ROOT}" || exit 2
export TMPDIR=/tmp
O=gpurun_out/ab_lanes1; rm -rf $O; mkdir -p $O
LGS_LANES1=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_batch.py tests/test_gpu_loop.py tests/test_gpu_rtcsm.py > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
for v in 0 1; do
  if [ $v = 1 ]; then export LGS_LANES1=1; else unset LGS_LANES1; fi
  timeout -k 10 300 python -u bench.py --no-cpu --latency-calls 0 --loop-line 0 --dropin-line 0 --steps 100 > $O/m$v.json 2>/dev/null || exit 1
  timeout -k 10 300 python -u bench.py --workload loop --no-cpu > $O/l$v.json 2>/dev/null || exit 1
  python3 - $O $v <<'PY'
import json, sys
o, v = sys.argv[1], sys.argv[2]
m = json.loads([l for l in open(f"{o}/m{v}.json") if l.startswith("{")][-1])
l = json.loads([l for l in open(f"{o}/l{v}.json") if l.startswith("{")][-1])
print("lanes1" if v == "1" else "lanes4", "match", m["value"], "coarse alone ms", m["roofline"]["avg_launch_ms"], "frac", m["roofline"]["frac"],
      "| loop", l["value"], "coarse ms", l["roofline"]["avg_launch_ms"], "frac", l["roofline"]["frac"])
PY
done; done
unset LGS_LANES1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/rb -o run -- python3 bench.py --workload rebuild --no-cpu > $O/rb.log 2>&1 || { tail -3 $O/rb.log; exit 1; }
find $O/rb -name '*kernel_trace.csv' -delete
