#!/bin/bash
# GPU-box sweep: HW queues x concurrent streams for the match bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
for cfg in ${CFGS:-4x3 8x6 8x8 16x12 16x16}; do   # queues x streams
  set -- ${cfg/x/ }
  name=streams_q$1_s$2${TAG}
  echo "== $name" | tee -a $OUT/steps.log
  GPU_MAX_HW_QUEUES=$1 timeout -k 10 300 python bench.py --no-cpu --steps ${BENCH_STEPS:-400} --warmup 10 --streams $2 ${BENCH_ARGS} > $OUT/$name.log 2>&1
  rc=$?
  echo "== $name rc=$rc" | tee -a $OUT/steps.log
  python3 -c "import json,sys; d=json.loads(open('$OUT/$name.log').read().strip().splitlines()[-1]); print('$name', d['value'], d['p50_scan_match_ms'], d['p50_scan_match_ms_single_stream'])" || true
  [ $rc -eq 0 ] || exit $rc
done
echo done
