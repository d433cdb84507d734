#!/bin/bash
# K1 parity tests, then a default-vs-variant bench A/B (variants: ablib/<name>.so).
# Usage: tools/gpu_ab2.sh <variant> [<variant> ...]
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_planes.py tests/test_gpu_rtcsm.py tests/test_gpu_batch.py tests/test_gpu_loop.py tests/test_gpu_frontend.py} -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/ab2_tests.log 2>&1
rc=$?
tail -4 gpurun_out/ab2_tests.log
[ $rc -ne 0 ] && exit $rc
for v in default "$@"; do
  if [ $v = default ]; then L=""; else L="LGS_LIB=ablib/$v.so"; fi
  env $L timeout -k 10 300 python -u bench.py --steps 100 --warmup 10 --cpu-seconds 1 --loop-line 0 --dropin-line 0 > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err || exit $?
  python3 -c "
import json; d=json.loads(open('gpurun_out/ab_$v.json').read().strip().splitlines()[-1])
print('$v', d['value'], d['coarse_blocks_scored_mean'], {k: v['avg_ms'] for k, v in d.get('kernels', {}).items()})"
done
