#!/bin/bash
# GPU-box profiling: kernel-trace stats run plus separate PMC passes (FETCH_SIZE,
# WRITE_SIZE, L2 hit/miss) of the same bench command.  Each pass runs under its
# own time limit; the script stops at the first crash/timeout.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out
TAG=${1:-r01}
mkdir -p $OUT
BENCH="bench.py --steps ${STEPS:-200} --warmup ${WARMUP:-10} --no-cpu --latency-calls 0 --loop-line 0 --dropin-line 0 --sub-lines 0"
run() {  # run <name> <rocprofv3 args...>
  local name=$1; shift
  echo "== $name" | tee -a $OUT/steps.log
  timeout -k 10 600 rocprofv3 "$@" --output-format csv -d $OUT/${name}_$TAG -o run -- python3 $BENCH \
      > $OUT/${name}_$TAG.log 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a $OUT/steps.log
  tail -2 $OUT/${name}_$TAG.log
  [ $rc -eq 0 ] || exit $rc
}
run trace --kernel-trace --stats
run pmc_fetch --pmc FETCH_SIZE
run pmc_write --pmc WRITE_SIZE
run pmc_l2 --pmc TCC_HIT_sum TCC_MISS_sum
echo done
