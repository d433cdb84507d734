#!/bin/bash
# All bench workloads, short runs (each under its own time limit).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=gpurun_out; mkdir -p $OUT
for w in ${WORKLOADS:-match refine loop stream}; do
  echo "== $w"
  timeout -k 10 600 python bench.py --workload $w ${BENCH_ARGS} > $OUT/bench_$w.json 2> $OUT/bench_$w.err
  rc=$?
  echo "== $w rc=$rc"; cat $OUT/bench_$w.json; tail -3 $OUT/bench_$w.err
  [ $rc -eq 0 ] || exit $rc
done
