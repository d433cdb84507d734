#!/bin/bash
# GPU-box check: parity tests, smoke, short bench, rocprof kernel-trace stats.
# Each GPU step has its own time limit; a crash/timeout (rc not in {0,1}) stops
# the script so nothing else touches the GPU after a fault.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
TAG=${1:-r01}
step() {  # step <name> <timeout> <cmd...>
  local name=$1 to=$2; shift 2
  echo "== $name: $*" | tee -a $OUT/steps.log
  timeout -k 10 "$to" "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a $OUT/steps.log
  tail -5 $OUT/$name.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step pytest_gpu 900 python -m pytest tests -m gpu -x -q ${PYTEST_ARGS}
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python bench.py --steps ${BENCH_STEPS:-200} --warmup 10
if [ -n "$PROFILE" ]; then
  step rocprof 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_$TAG -o run -- python bench.py --steps 50 --warmup 5 --no-cpu
fi
echo done
