#!/bin/bash
# Zero tiles: parity tests, then the default bench with LGS_OPT_ZERO_TILES (33) on/off.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out
TAG=${1:-r05zt}
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_batch.py tests/test_gpu_benchcfg.py tests/test_gpu_planes.py tests/test_gpu_loop.py \
  > $OUT/${TAG}_tests.log 2>&1 || { tail -30 $OUT/${TAG}_tests.log; exit 1; }
tail -2 $OUT/${TAG}_tests.log
B="bench.py --steps 200 --warmup 10 --no-cpu --loop-line 0 --dropin-line 0"
for arm in on off on off; do
  opt=""; [ $arm = off ] && opt="33=0"
  LGS_CTX_OPTIONS="$opt" timeout -k 10 400 python3 $B --sub-lines 0 > $OUT/${TAG}_$arm.json 2> $OUT/${TAG}_$arm.err || exit $?
  python3 -c "import json; d=json.loads(open('$OUT/${TAG}_$arm.json').read().strip().splitlines()[-1]); k=d['kernels']; print('$arm', d['value'], d['p50_scan_match_ms'], d['p50_batch_call_ms'], 'pre', k['k_precompute']['avg_ms'], 'hv', k['k_super_planes']['avg_ms'], d['roofline']['frac'])"
done
for arm in on off; do
  opt=""; [ $arm = off ] && opt="33=0"
  LGS_CTX_OPTIONS="$opt" timeout -k 10 400 python3 bench.py --workload loop --steps 12 --warmup 3 --no-cpu > $OUT/${TAG}_loop_$arm.json 2> $OUT/${TAG}_loop_$arm.err || exit $?
  python3 -c "import json; d=json.loads(open('$OUT/${TAG}_loop_$arm.json').read().strip().splitlines()[-1]); print('loop $arm', d['value'])"
done
echo done
