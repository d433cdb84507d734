#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_rtcsm.py tests/test_gpu_batch.py tests/test_gpu_loop.py > gpurun_out/abh_tests.log 2>&1 &&
for i in 1 2; do
timeout -k 10 200 python bench.py --steps 100 --no-cpu --latency-calls 20 --timed-events all > gpurun_out/abh_hex_$i.json 2>&1 &&
timeout -k 10 200 python bench.py --steps 100 --no-cpu --latency-calls 20 --timed-events all --super-hex 0 > gpurun_out/abh_quad_$i.json 2>&1 || exit 1
done
rc=$?; tail -2 gpurun_out/abh_tests.log; exit $rc
