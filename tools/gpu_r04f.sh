#!/bin/bash
# r04f: GPU suite (device branch-and-bound replay), loop_bb bench x2 with phase timing
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
tools/gpu_step.sh "gputests|600|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" || exit $?
tools/gpu_step.sh "bb1|300|LGS_BB_TIMING=1 python bench.py --workload loop_bb > gpurun_out/bench_bb1.json 2> gpurun_out/bench_bb1.err" \
  "bb2|300|python bench.py --workload loop_bb > gpurun_out/bench_bb2.json" || exit $?
grep "^bb n=" gpurun_out/bench_bb1.err | tail -4
