#!/bin/bash
# GPU-box A/B of library builds: bench.py with LGS_LIB=<variant .so> for each
# variant in $VARIANTS (name "base" = the in-tree library).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
for v in ${VARIANTS:-base}; do
  lib=""
  [ "$v" != base ] && lib="tools/exp/ab_$v.so"
  echo "== $v" | tee -a $OUT/steps.log
  LGS_LIB=$lib timeout -k 10 300 python bench.py --no-cpu --steps ${BENCH_STEPS:-40} --warmup 5 ${BENCH_ARGS} > $OUT/ab_$v.log 2>&1
  rc=$?
  echo "== $v rc=$rc" | tee -a $OUT/steps.log
  if [ $rc -ne 0 ]; then tail -5 $OUT/ab_$v.log; exit $rc; fi
done
echo done
