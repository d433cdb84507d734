#!/bin/bash
# r04 final (part 2): trace + PMC passes of the loop / loop_bb / rebuild workloads
# (profiles/pmc_summary_<w>.json for this library), the config-4 stream kernel trace
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
TAG=${1:-r04_vf}
STEPS=12 bash tools/gpu_prof_workloads.sh $TAG loop loop_bb rebuild || exit $?
tools/gpu_step.sh "stprof|300|rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_st -o run -- python3 bench.py --workload stream --steps 2000 --no-cpu > gpurun_out/${TAG}_stprof.json && mkdir -p gpurun_out/prof_st && cp /tmp/prof_st/*kernel_stats.csv /tmp/prof_st/*kernel_trace.csv gpurun_out/prof_st/" || exit $?
python3 tools/stream_gaps.py gpurun_out/prof_st/run_kernel_trace.csv > gpurun_out/${TAG}_stream_gaps.txt; head -14 gpurun_out/${TAG}_stream_gaps.txt
