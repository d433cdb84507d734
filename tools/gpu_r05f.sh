#!/bin/bash
# r05: branch-free k_super_hv A/B (whole units vs halves), loop tests, f2 host timing, scaling probe
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
tools/gpu_step.sh "t_sel|400|python -u -m pytest tests/test_gpu_planes.py tests/test_gpu_benchcfg.py tests/test_gpu_loop.py tests/test_gpu_batch.py -x -q --timeout 120 --timeout-method thread" \
  "bench_half|600|python -u bench.py --sub-lines 0 --dropin-line 0 > gpurun_out/r05f_half.json 2> gpurun_out/r05f_half.err" \
  "bench_full|600|LGS_CTX_OPTIONS=29=1 python -u bench.py --sub-lines 0 --loop-line 0 --dropin-line 0 --latency-calls 0 > gpurun_out/r05f_full.json 2> gpurun_out/r05f_full.err" \
  "f2t|300|LGS_F2_TIMING=1 python -u bench.py --workload rebuild --steps 10 --warmup 2 --no-cpu > gpurun_out/r05f_f2.json 2> gpurun_out/r05f_f2.err" \
  "probe|600|python -u tools/scaling_probe.py --out gpurun_out/r05_scaling_probe.json > gpurun_out/probe.log 2>&1"
