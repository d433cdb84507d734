#!/bin/bash
# r04i: config-4 stream kernel trace (step anatomy) + LGS_STEP_TIMING host phases
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
tools/gpu_step.sh "stprof|300|LGS_STEP_TIMING=1 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d /tmp/prof_st -o run -- python3 bench.py --workload stream --steps 2000 --no-cpu > gpurun_out/stprof.json 2> gpurun_out/stprof.err && mkdir -p gpurun_out/prof_st && cp /tmp/prof_st/*stats.csv /tmp/prof_st/*kernel_trace.csv /tmp/prof_st/*memory_copy_trace.csv gpurun_out/prof_st/" || exit $?
python3 tools/stream_gaps.py gpurun_out/prof_st/run_kernel_trace.csv
grep "latest step host" gpurun_out/stprof.err | tail -2
tools/gpu_step.sh "st|200|LGS_STEP_TIMING=1 python bench.py --workload stream --steps 2000 --no-cpu > gpurun_out/st.json 2> gpurun_out/st.err" || exit $?
grep "latest step host" gpurun_out/st.err | tail -2
