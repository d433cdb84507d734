#!/bin/bash
# r05: k_super_hv (flat) + priority tail: parity, the default bench line (all sub-lines), A/B without the priority stream
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
tools/gpu_step.sh "t_planes|300|python -u -m pytest tests/test_gpu_planes.py -x -q --timeout 120 --timeout-method thread" \
  "t_more|600|python -u -m pytest tests/test_gpu_rtcsm.py tests/test_gpu_batch.py tests/test_gpu_benchcfg.py tests/test_gpu_bb.py tests/test_gpu_loop.py tests/test_gpu_small.py -x -q --timeout 120 --timeout-method thread" \
  "bench|900|python -u bench.py > gpurun_out/r05d_bench.json 2> gpurun_out/r05d_bench.err" \
  "bench_np|600|LGS_CTX_OPTIONS=28=0 python -u bench.py --sub-lines 0 --loop-line 0 --dropin-line 0 > gpurun_out/r05d_bench_np.json 2> gpurun_out/r05d_bench_np.err"
