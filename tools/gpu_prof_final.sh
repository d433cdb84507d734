#!/bin/bash
# Profile of THIS build: kernel trace + PMC passes of the default bench command
# (tools/gpu_prof.sh), the PMC summary bench.py reads (lib sha256 of this .so),
# then the default bench line (roofline.traffic / frac_hbm_counters filled) and
# the other workloads' lines.  Usage: tools/gpu_prof_final.sh r02_v3
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
TAG=${1:-r02_vX}
OUT=gpurun_out
mkdir -p $OUT
STEPS=${STEPS:-200} bash tools/gpu_prof.sh $TAG || exit $?
python3 tools/pmc_summary.py $OUT/trace_$TAG $OUT/pmc_fetch_$TAG $OUT/pmc_write_$TAG $OUT/pmc_l2_$TAG $OUT/$TAG > $OUT/${TAG}_summary.log 2>&1 || exit $?
cp $OUT/trace_$TAG/run_kernel_stats.csv $OUT/${TAG}_run_kernel_stats.csv 2>/dev/null || find $OUT/trace_$TAG -name "*kernel_stats.csv" -exec cp {} $OUT/${TAG}_run_kernel_stats.csv \;
cp $OUT/${TAG}_pmc.json profiles/r02_pmc_summary.json
rm -rf $OUT/pmc_fetch_$TAG $OUT/pmc_write_$TAG $OUT/pmc_l2_$TAG $OUT/trace_$TAG
timeout -k 10 600 python -u bench.py > $OUT/${TAG}_bench.json 2> $OUT/${TAG}_bench.err || exit $?
tail -c 1200 $OUT/${TAG}_bench.json
for w in ${WORKLOADS:-refine loop loop_bb stream rebuild}; do
  timeout -k 10 600 python -u bench.py --workload $w > $OUT/${TAG}_bench_$w.json 2> $OUT/${TAG}_bench_$w.err || exit $?
  echo "$w: $(python3 -c "import json;d=json.loads(open('$OUT/${TAG}_bench_$w.json').read().strip().splitlines()[-1]);print(d['value'], d['unit'])")"
done
