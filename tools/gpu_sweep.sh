#!/bin/bash
# GPU-box sweep: parity tests, smoke, then bench.py over (batch, streams)
# combinations (no CPU baseline).  Stops at the first crash/timeout.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
step() {  # step <name> <timeout> <cmd...>
  local name=$1 to=$2; shift 2
  echo "== $name: $*" | tee -a $OUT/steps.log
  timeout -k 10 "$to" "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a $OUT/steps.log
  tail -3 $OUT/$name.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
if [ -z "$NO_TESTS" ]; then
  step pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_ARGS}
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
for bs in ${SWEEP:-1:3 8:2 16:1 16:2 32:1 32:2 64:1 64:2}; do
  b=${bs%%:*}; s=${bs##*:}
  step bench_b${b}_s${s} 300 python bench.py --steps ${BENCH_STEPS:-60} --warmup 5 --no-cpu --batch $b --streams $s
done
echo done
