#!/bin/bash
# r02 session 3: correlative-path parity tests + default bench
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r02n}
timeout -k 10 600 python -u -m pytest tests/test_gpu_planes.py tests/test_gpu_rtcsm.py tests/test_gpu_batch.py tests/test_gpu_loop.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_tests.log 2>&1
rc=$?
tail -4 gpurun_out/${T}_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python -u bench.py --steps 200 --warmup 10 --cpu-seconds 2 > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err
rc=$?
python3 -c "
import json; d=json.loads(open('gpurun_out/${T}_bench.json').read().strip().splitlines()[-1])
print('value', d['value'], 'p50', d['p50_scan_match_ms'], 'roof', d['roofline']['avg_launch_ms'], d['roofline']['frac'])
print({k: v['avg_ms'] for k, v in d.get('kernels', {}).items()})"
exit $rc
