#!/bin/bash
# GPU-box runner: each argument is one step "name|timeout|command"; every step
# runs under its own time limit, output in gpurun_out/<name>.log.  A crash,
# abort or time limit (rc not in {0,1}) ends the script: nothing else touches
# the GPU after a fault.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
for spec in "$@"; do
  name=${spec%%|*}; rest=${spec#*|}; to=${rest%%|*}; cmd=${rest#*|}
  echo "== $name ($to s): $cmd" | tee -a $OUT/steps.log
  timeout -k 10 "$to" bash -c "$cmd" > $OUT/$name.log 2>&1
  rc=$?
  echo "== $name rc=$rc" | tee -a $OUT/steps.log
  tail -4 $OUT/$name.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
done
echo done
