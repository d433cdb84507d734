#!/bin/bash
# GPU-box kernel trace of the match bench (csv), for timeline analysis.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
for cfg in ${CFGS:-4x3 16x16}; do   # queues x streams
  set -- ${cfg/x/ }
  name=trace_q$1_s$2
  echo "== $name" | tee -a $OUT/steps.log
  GPU_MAX_HW_QUEUES=$1 timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $OUT/$name -o run -- \
      python3 bench.py --no-cpu --steps ${BENCH_STEPS:-400} --warmup 10 --streams $2 ${BENCH_ARGS} > $OUT/$name.log 2>&1
  rc=$?
  echo "== $name rc=$rc" | tee -a $OUT/steps.log
  [ $rc -eq 0 ] || exit $rc
done
echo done
