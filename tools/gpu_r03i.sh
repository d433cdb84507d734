#!/bin/bash
# r03: whole GPU suite after lazy scan copies / stamp-only angle flags, then
# the config-4 stream and config-2 match lines and a stream kernel trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03i}; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 300 python -u bench.py --workload stream > $O/stream.json 2> $O/stream.err || { tail -5 $O/stream.err; exit 1; }
timeout -k 10 300 python -u bench.py > $O/match.json 2> $O/match.err || { tail -5 $O/match.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --workload stream --steps 2000 --no-cpu > $O/trace.log 2>&1 || { tail -5 $O/trace.log; exit 1; }
find $O/trace -name '*kernel_trace.csv' -delete
TAG=${TAG:-r03i} python3 - <<'PY'
import json, os
for f in ("stream", "match"):
    d = json.loads([l for l in open(os.path.join("gpurun_out", os.environ.get("TAG", "r03i"), f + ".json")) if l.startswith("{")][-1])
    print(f, d["value"], d["ms_per_step"], d.get("breakdown_per_step"), (d.get("roofline") or {}).get("frac"))
PY
