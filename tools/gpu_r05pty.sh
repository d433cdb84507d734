#!/bin/bash
# batched precompute tile height (LGS_PTY_BATCH build): parity, then the default bench twice.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out
TAG=${1:-r05pty}
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_batch.py tests/test_gpu_planes.py tests/test_gpu_benchcfg.py \
  > $OUT/${TAG}_tests.log 2>&1 || { tail -30 $OUT/${TAG}_tests.log; exit 1; }
tail -1 $OUT/${TAG}_tests.log
B="bench.py --steps 200 --warmup 10 --no-cpu --loop-line 0 --dropin-line 0 --sub-lines 0"
for arm in 1 2; do
  timeout -k 10 400 python3 $B > $OUT/${TAG}_$arm.json 2> $OUT/${TAG}_$arm.err || exit $?
  python3 -c "import json; d=json.loads(open('$OUT/${TAG}_$arm.json').read().strip().splitlines()[-1]); k=d['kernels']; print('$arm', d['value'], d['p50_scan_match_ms'], d['p50_batch_call_ms'], 'pre', k['k_precompute']['avg_ms'], 'hv', k['k_super_planes']['avg_ms'])"
done
echo done
