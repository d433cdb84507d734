#!/bin/bash
# r04g: branch-and-bound GPU tests + loop_bb bench (rotation trig tables)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
tools/gpu_step.sh "bbtests|300|python -u -m pytest tests/test_gpu_bb.py tests/test_gpu_loop.py tests/test_cpp_adapter.py -x -q --timeout 120 --timeout-method thread" || exit $?
tools/gpu_step.sh "bb1|300|LGS_BB_TIMING=1 python bench.py --workload loop_bb > gpurun_out/bench_bb1.json 2> gpurun_out/bench_bb1.err" \
  "bb2|300|python bench.py --workload loop_bb > gpurun_out/bench_bb2.json" || exit $?
grep "^bb n=" gpurun_out/bench_bb1.err | tail -3
python3 -c "import json;d=json.loads(open('gpurun_out/bench_bb2.json').read().strip().splitlines()[-1]);print(d['value'], d['step_spread'], d['kernels'])"
