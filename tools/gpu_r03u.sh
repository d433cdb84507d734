#!/bin/bash
# r03: kept-superblock work list (k_keep + k_coarse_list + k_unsafe_list, the
# batched default) -- the matcher's GPU tests, the config-5 and config-2 lines
# (twice each) and a config-5 kernel trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03u}; rm -rf $O; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_loop.py tests/test_gpu_batch.py tests/test_gpu_scans.py tests/test_gpu_planes.py tests/test_gpu_rtcsm.py tests/test_gpu_bb.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
timeout -k 10 300 python -u bench.py --workload loop --no-cpu > $O/loop$i.json 2>/dev/null || exit 1
python3 -c "import json;d=json.loads([l for l in open('$O/loop$i.json') if l.startswith('{')][-1]);print('loop', d['value'], d['roofline']['avg_launch_ms'], d['roofline']['frac'], d['config'].get('found'))"
timeout -k 10 300 python -u bench.py --no-cpu --latency-calls 0 --loop-line 0 --dropin-line 0 > $O/match$i.json 2>/dev/null || exit 1
python3 -c "import json;d=json.loads([l for l in open('$O/match$i.json') if l.startswith('{')][-1]);print('match', d['value'], d['roofline']['avg_launch_ms'], d['roofline']['frac'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --workload loop --no-cpu > $O/trace.log 2>&1 || { tail -5 $O/trace.log; exit 1; }
find $O/trace -name '*kernel_trace.csv' -delete
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace2 -o run -- python3 bench.py --steps 60 --warmup 5 --no-cpu --latency-calls 0 --loop-line 0 --dropin-line 0 > $O/trace2.log 2>&1 || { tail -5 $O/trace2.log; exit 1; }
find $O/trace2 -name '*kernel_trace.csv' -delete
