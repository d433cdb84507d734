#!/bin/bash
# r04: full GPU suite, default bench, loop_bb, and A/B of the flat-gather and
# 16-byte-unit variants (ablib/ab_flat.so, ablib/ab_nooct12.so)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
tools/gpu_step.sh "gputests|900|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "bench|400|python bench.py > gpurun_out/bench.json" \
  "bb|300|python bench.py --workload loop_bb > gpurun_out/bench_bb.json" || exit $?
tools/gpu_abn.sh m1 "--steps 100 --warmup 10 --no-cpu --loop-line 0 --dropin-line 0 --sub-lines 0 --timed-events all --streams 1" 2 base flat || exit $?
tools/gpu_abn.sh lp "--workload loop --steps 20 --warmup 2 --no-cpu" 2 base flat nooct12 || exit $?
tools/gpu_abn.sh st "--workload stream --steps 2000 --no-cpu" 2 base flat
