#!/bin/bash
# Profile of THIS build: kernel trace + PMC passes of the match bench (the
# default command without its side lines: no CPU leg, lone-latency calls,
# loop or drop-in lines -- they do not touch the timed region or the isolated
# pass), the PMC summary bench.py reads (library sha256 + workload), the split
# of the dominant kernel's traced dispatches into alone / shared
# (tools/trace_coarse.py), then the default bench line and the other
# workloads' lines.  Usage: tools/gpu_prof_final.sh r03_v2
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
TAG=${1:-r03_vX}
OUT=gpurun_out
mkdir -p $OUT
STEPS=${STEPS:-200} bash tools/gpu_prof.sh $TAG || exit $?
WORKLOAD=match python3 tools/pmc_summary.py $OUT/trace_$TAG $OUT/pmc_fetch_$TAG $OUT/pmc_write_$TAG $OUT/pmc_l2_$TAG $OUT/$TAG > $OUT/${TAG}_summary.log 2>&1 || exit $?
cp $OUT/${TAG}_pmc.json profiles/pmc_summary.json
grep '^{' $OUT/trace_$TAG.log | tail -n 1 > $OUT/${TAG}_trace_run_bench.json
ALGO=$(python3 -c "import json;print(json.loads(open('$OUT/${TAG}_trace_run_bench.json').read())['roofline']['algo_bytes_per_launch'])") || exit 1
TR=$(find $OUT/trace_$TAG -name '*kernel_trace.csv' | head -1)
python3 tools/trace_coarse.py $TR k_coarse_list $ALGO > $OUT/${TAG}_coarse_split.json || exit 1
cat $OUT/${TAG}_coarse_split.json
find $OUT/trace_$TAG -name '*kernel_stats.csv' -exec cp {} $OUT/${TAG}_run_kernel_stats.csv \;
rm -rf $OUT/pmc_fetch_$TAG $OUT/pmc_write_$TAG $OUT/pmc_l2_$TAG $OUT/trace_$TAG
timeout -k 10 600 python -u bench.py > $OUT/${TAG}_bench.json 2> $OUT/${TAG}_bench.err || exit $?
tail -c 1500 $OUT/${TAG}_bench.json
for w in ${WORKLOADS:-refine loop loop_bb stream rebuild}; do
  timeout -k 10 600 python -u bench.py --workload $w > $OUT/${TAG}_bench_$w.json 2> $OUT/${TAG}_bench_$w.err || exit $?
  echo "$w: $(python3 -c "import json;d=json.loads(open('$OUT/${TAG}_bench_$w.json').read().strip().splitlines()[-1]);print(d['value'], d['unit'])")"
done
