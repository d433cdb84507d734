#!/bin/bash
# r04j: config-4 stream with host step timing, kernel trace gaps
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
tools/gpu_step.sh "st|200|LGS_STEP_TIMING=1 python bench.py --workload stream --steps 2000 --no-cpu > gpurun_out/st.json 2> gpurun_out/st.err" || exit $?
grep "latest step host" gpurun_out/st.err | tail -3
python3 -c "import json;d=json.loads(open('gpurun_out/st.json').read().strip().splitlines()[-1]);print(d['value'], d['breakdown_per_step'])"
tools/gpu_step.sh "stprof|300|rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_st -o run -- python3 bench.py --workload stream --steps 2000 --no-cpu > gpurun_out/stprof.json 2> gpurun_out/stprof.err && mkdir -p gpurun_out/prof_st && cp /tmp/prof_st/*stats.csv /tmp/prof_st/*kernel_trace.csv gpurun_out/prof_st/" || exit $?
python3 tools/stream_gaps.py gpurun_out/prof_st/run_kernel_trace.csv | head -14
