#!/bin/bash
# r03: K3 sort tests + map tests, the f2 rebuild line and its kernel trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03q}; rm -rf $O; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_keysort.py tests/test_gpu_latest.py tests/test_gpu_raycast.py tests/test_gpu_frontend.py tests/test_gpu_mapbuild.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u bench.py --workload rebuild --no-cpu > $O/rebuild.json 2> $O/rebuild.err || { tail -5 $O/rebuild.err; exit 1; }
python3 -c "import json;d=json.loads([l for l in open('$O/rebuild.json') if l.startswith('{')][-1]);print('rebuild', d['value'], d['unit'], d['ms_per_step'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --workload rebuild --no-cpu > $O/trace.log 2>&1 || { tail -5 $O/trace.log; exit 1; }
find $O/trace -name '*kernel_trace.csv' -delete
