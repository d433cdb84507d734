#!/bin/bash
# Final profile of THIS build: full GPU suite, trace + PMC passes of the match bench
# (pmc_summary.json for this library), the default bench line.
# Usage: PHASES="tests prof bench" tools/gpu_final.sh <tag>   (each phase its own gpurun call if need be);
# then tools/gpu_prof_workloads.sh <tag> loop loop_bb rebuild
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
TAG=${1:-r06_vf}
OUT=gpurun_out
PHASES=${PHASES:-tests prof bench}
mkdir -p $OUT
for ph in $PHASES; do
  case $ph in
  tests)
    tools/gpu_step.sh "gputests|1000|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" || exit $?
    cp $OUT/gputests.log $OUT/${TAG}_gputests.log ;;
  prof)
    STEPS=200 bash tools/gpu_prof.sh $TAG || exit $?
    WORKLOAD=match python3 tools/pmc_summary.py $OUT/trace_$TAG $OUT/pmc_fetch_$TAG $OUT/pmc_write_$TAG $OUT/pmc_l2_$TAG $OUT/$TAG > $OUT/${TAG}_summary.log 2>&1 || exit $?
    cp $OUT/${TAG}_pmc.json profiles/pmc_summary.json
    grep '^{' $OUT/trace_$TAG.log | tail -n 1 > $OUT/${TAG}_trace_run_bench.json
    # the timed region's dispatches: streams (bench default 2) x 10 warm-up calls x 2 chunks before it, the
    # 8-call one-stream pass after (HEAD / TAIL override)
    read ALGO ALGOS < <(python3 -c "import json;d=json.loads(open('$OUT/${TAG}_trace_run_bench.json').read());print(d['roofline']['algo_bytes_per_launch'], d['roofline_super']['algo_bytes_per_launch'])") || exit 1
    TR=$(find $OUT/trace_$TAG -name '*kernel_trace.csv' | head -1)
    python3 tools/trace_coarse.py $TR k_coarse_list $ALGO ${HEAD:-40} ${TAIL:-16} > $OUT/${TAG}_coarse_split.json || exit 1
    python3 tools/trace_coarse.py $TR "k_super_oct<5" $ALGOS ${HEAD:-40} ${TAIL:-16} > $OUT/${TAG}_super_split.json || exit 1
    find $OUT/trace_$TAG -name '*kernel_stats.csv' -exec cp {} $OUT/${TAG}_run_kernel_stats.csv \;
    rm -rf $OUT/pmc_fetch_$TAG $OUT/pmc_write_$TAG $OUT/pmc_l2_$TAG $OUT/trace_$TAG ;;
  bench)
    tools/gpu_step.sh "bench|900|python -u bench.py > $OUT/${TAG}_bench.json 2> $OUT/${TAG}_bench.err" || exit $?
    python3 -c "import json;d=json.loads(open('$OUT/${TAG}_bench.json').read().strip().splitlines()[-1]);print(d['value'], d['roofline']['frac'], d['roofline']['traffic'], [(k, (d.get(k) or {}).get('value')) for k in ('config5_strong_scaling','config4_stream','config3_refine','f2_rebuild','config2_distinct_maps')])" ;;
  esac
done
echo done
