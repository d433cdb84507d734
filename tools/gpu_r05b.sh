#!/bin/bash
# r05: fused planes kernel -- targeted parity, then the default bench (fused on) and an A/B line (fused off)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
tools/gpu_step.sh "t_planes|300|python -u -m pytest tests/test_gpu_planes.py -x -q --timeout 120 --timeout-method thread" \
  "t_more|600|python -u -m pytest tests/test_gpu_rtcsm.py tests/test_gpu_batch.py tests/test_gpu_benchcfg.py tests/test_gpu_bb.py tests/test_gpu_loop.py -x -q --timeout 120 --timeout-method thread" \
  "bench|600|python -u bench.py --sub-lines 0 --loop-line 0 --dropin-line 0 > gpurun_out/r05b_bench.json 2> gpurun_out/r05b_bench.err" \
  "bench_off|600|LGS_CTX_OPTIONS=27=0 python -u bench.py --sub-lines 0 --loop-line 0 --dropin-line 0 --latency-calls 0 > gpurun_out/r05b_bench_off.json 2> gpurun_out/r05b_bench_off.err"
