#!/bin/bash
# r05: k_super_hv<2> (whole units) vs <1> (halves)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
tools/gpu_step.sh "t_planes|300|python -u -m pytest tests/test_gpu_planes.py tests/test_gpu_benchcfg.py -x -q --timeout 120 --timeout-method thread" \
  "bench_full|600|LGS_CTX_OPTIONS=29=1 python -u bench.py --sub-lines 0 --loop-line 0 --dropin-line 0 > gpurun_out/r05e_full.json 2> gpurun_out/r05e_full.err" \
  "bench_half|600|LGS_CTX_OPTIONS=29=0 python -u bench.py --sub-lines 0 --loop-line 0 --dropin-line 0 > gpurun_out/r05e_half.json 2> gpurun_out/r05e_half.err" \
  "bench_full2|600|LGS_CTX_OPTIONS=29=1 python -u bench.py --sub-lines 0 --loop-line 0 --dropin-line 0 --latency-calls 0 > gpurun_out/r05e_full2.json 2> gpurun_out/r05e_full2.err"
