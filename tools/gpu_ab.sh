#!/bin/bash
# GPU-box A/B: parity tests, then the match bench with a given option on/off.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
step() {
  local name=$1 to=$2; shift 2
  echo "== $name: $*" | tee -a $OUT/steps.log
  timeout -k 10 "$to" "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a $OUT/steps.log
  tail -3 $OUT/$name.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
[ -z "$SKIP_TESTS" ] && step pytest_gpu 900 python -m pytest tests -m gpu -x -q ${PYTEST_ARGS}
for v in ${AB_VALUES:-1 0}; do
  step bench_${AB_FLAG:-super-prune}_$v 300 python bench.py --no-cpu --steps ${BENCH_STEPS:-200} --warmup 10 --${AB_FLAG:-super-prune} $v ${BENCH_ARGS}
done
echo done
