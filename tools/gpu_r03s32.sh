#!/bin/bash
# r03: k_super_oct with fp32 partial sums (bound x m32) -- the whole -m gpu
# suite, then the config-5 and config-2 lines twice with the one-stream kernel
# trace of config 5.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03s32}; rm -rf $O; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests > $O/gputests.log 2>&1 || { tail -30 $O/gputests.log; exit 1; }
tail -1 $O/gputests.log
for i in 1 2; do
timeout -k 10 300 python -u bench.py --workload loop --no-cpu > $O/loop$i.json 2>/dev/null || exit 1
timeout -k 10 300 python -u bench.py --no-cpu --latency-calls 0 --loop-line 0 --dropin-line 0 > $O/match$i.json 2>/dev/null || exit 1
python3 -c "
import json
a=json.loads([l for l in open('$O/loop$i.json') if l.startswith('{')][-1]);b=json.loads([l for l in open('$O/match$i.json') if l.startswith('{')][-1])
print('loop', a['value'], 'match', b['value'], b['coarse_blocks_scored_mean'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trl -o run -- python3 bench.py --workload loop --no-cpu > $O/trl.log 2>&1 || { tail -5 $O/trl.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr -o run -- python3 bench.py --steps 40 --warmup 5 --streams 1 --no-cpu --latency-calls 0 --loop-line 0 --dropin-line 0 > $O/tr.log 2>&1 || { tail -5 $O/tr.log; exit 1; }
find $O -name '*kernel_trace.csv' -delete
grep -h "k_super_oct" $O/trl/run_kernel_stats.csv $O/tr/run_kernel_stats.csv | cut -c1-200
