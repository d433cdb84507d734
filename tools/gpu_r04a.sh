#!/bin/bash
# r04: full GPU suite, default bench, loop_bb, and A/B of library variants
# (ablib/ab_<name>.so: flat gathers, 16-byte units, whole-row coarse list, list grid, chunk size)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
tools/gpu_step.sh "gputests|900|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "bench|400|python bench.py > gpurun_out/bench.json" \
  "bb|300|python bench.py --workload loop_bb > gpurun_out/bench_bb.json" || exit $?
tools/gpu_abn.sh m1 "--steps 100 --warmup 10 --no-cpu --loop-line 0 --dropin-line 0 --sub-lines 0 --timed-events all --streams 1" 2 base flat nochunk lw8k ch128 || exit $?
tools/gpu_abn.sh m3 "--steps 200 --warmup 10 --no-cpu --loop-line 0 --dropin-line 0 --sub-lines 0" 2 base flat nochunk || exit $?
tools/gpu_abn.sh lp "--workload loop --steps 20 --warmup 2 --no-cpu" 2 base flat nooct12 nochunk || exit $?
tools/gpu_abn.sh st "--workload stream --steps 2000 --no-cpu" 2 base flat
