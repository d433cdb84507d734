#!/bin/bash
# r03: the whole -m gpu suite on the work-list build, then the config-5 and
# config-2 lines (roofline = k_coarse_list, coarse_stage = the three passes).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03w}; rm -rf $O; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests > $O/gputests.log 2>&1 || { tail -30 $O/gputests.log; exit 1; }
tail -1 $O/gputests.log
timeout -k 10 300 python -u bench.py --workload loop --no-cpu > $O/loop.json 2>/dev/null || exit 1
python3 -c "import json;d=json.loads([l for l in open('$O/loop.json') if l.startswith('{')][-1]);print('loop', d['value'], d['roofline']['kernel'], d['roofline']['avg_launch_ms'], d['roofline']['frac'], d['coarse_stage'], d['config'].get('found'))"
timeout -k 10 300 python -u bench.py --no-cpu --loop-line 0 --dropin-line 0 > $O/match.json 2>/dev/null || exit 1
python3 -c "import json;d=json.loads([l for l in open('$O/match.json') if l.startswith('{')][-1]);print('match', d['value'], d['roofline']['avg_launch_ms'], d['roofline']['frac'], d['roofline_timed_region']['frac'], d['coarse_stage'], d['p50_scan_match_ms'])"
