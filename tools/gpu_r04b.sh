#!/bin/bash
# r04b: full GPU suite (k_match_small included), default bench, config-4 stream A/B of the
# small-window path (LGS_OPT_SMALL_WINDOW = 25), loop_bb
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
tools/gpu_step.sh "gputests|600|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "bench|400|python bench.py > gpurun_out/bench.json" || exit $?
for r in 1 2; do
  tools/gpu_step.sh "st_small_$r|200|python bench.py --workload stream --steps 2000 --no-cpu > gpurun_out/st_small_$r.json" \
    "st_gen_$r|200|python bench.py --workload stream --steps 2000 --no-cpu --ctx-option 25=0 > gpurun_out/st_gen_$r.json" || exit $?
done
tools/gpu_step.sh "stprof|300|LGS_STEP_TIMING=1 rocprofv3 --kernel-trace --memory-copy-trace --hip-trace --stats --output-format csv -d /tmp/prof_st -o run -- python3 bench.py --workload stream --steps 2000 --no-cpu > gpurun_out/stprof.json && mkdir -p gpurun_out/prof_st && cp /tmp/prof_st/*stats.csv /tmp/prof_st/*kernel_trace.csv /tmp/prof_st/*memory_copy_trace.csv gpurun_out/prof_st/" || exit $?
tools/gpu_step.sh "bb|300|python bench.py --workload loop_bb > gpurun_out/bench_bb.json"
tools/gpu_abn.sh m1 "--steps 100 --warmup 10 --no-cpu --loop-line 0 --dropin-line 0 --sub-lines 0 --timed-events all --streams 1" 2 base flat nochunk || exit $?
tools/gpu_abn.sh lp "--workload loop --steps 20 --warmup 2 --no-cpu" 2 base nooct12 || exit $?
