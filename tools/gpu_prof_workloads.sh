#!/bin/bash
# Kernel trace + separate PMC passes (FETCH_SIZE, WRITE_SIZE, L2 hit/miss) of
# the non-default bench workloads, summarised into profiles/pmc_summary_<w>.json
# (bench.py takes roofline.traffic of workload <w> from it for this library
# build).  Each pass has its own time limit; the script stops at the first
# failure.  Usage: tools/gpu_prof_workloads.sh r03_v10 [loop rebuild ...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out
TAG=${1:-r03_vX}; shift
mkdir -p $OUT
for w in ${@:-loop loop_bb rebuild}; do
  BENCH="bench.py --workload $w --steps ${STEPS:-20} --warmup 2 --no-cpu"
  for pass in "trace --kernel-trace --stats" "pmc_fetch --pmc FETCH_SIZE" "pmc_write --pmc WRITE_SIZE" \
              "pmc_l2 --pmc TCC_HIT_sum TCC_MISS_sum"; do
    set -- $pass; name=$1; shift
    echo "== $w $name" | tee -a $OUT/steps.log
    timeout -k 10 300 rocprofv3 "$@" --output-format csv -d $OUT/${name}_${TAG}_$w -o run -- python3 $BENCH \
        > $OUT/${name}_${TAG}_$w.log 2>&1
    rc=$?
    echo "== $w $name rc=$rc" | tee -a $OUT/steps.log
    tail -2 $OUT/${name}_${TAG}_$w.log
    [ $rc -eq 0 ] || exit $rc
  done
  WORKLOAD=$w python3 tools/pmc_summary.py $OUT/trace_${TAG}_$w $OUT/pmc_fetch_${TAG}_$w $OUT/pmc_write_${TAG}_$w \
      $OUT/pmc_l2_${TAG}_$w $OUT/${TAG}_$w > $OUT/${TAG}_${w}_summary.log 2>&1 || exit $?
  cp $OUT/${TAG}_${w}_pmc.json profiles/pmc_summary_$w.json
  cp $OUT/${TAG}_${w}_pmc.json $OUT/pmc_summary_$w.json
  rm -rf $OUT/pmc_fetch_${TAG}_$w $OUT/pmc_write_${TAG}_$w $OUT/pmc_l2_${TAG}_$w $OUT/trace_${TAG}_$w
  timeout -k 10 300 python -u bench.py --workload $w > $OUT/${TAG}_bench_$w.json 2> $OUT/${TAG}_bench_$w.err || exit $?
  python3 -c "import json;d=json.loads(open('$OUT/${TAG}_bench_$w.json').read().strip().splitlines()[-1]);print('$w', d['value'], d['unit'], d['roofline'])"
done
echo done
