#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
LGS_LIB=tools/exp/ab_hp16.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_batch.py > gpurun_out/abhp_tests.log 2>&1 &&
for i in 1 2; do for v in base hp16 hp4; do
  lib=""; [ $v != base ] && lib=tools/exp/ab_$v.so
  LGS_LIB=$lib timeout -k 10 200 python bench.py --steps 100 --no-cpu --latency-calls 10 --timed-events all > gpurun_out/abhp_${v}_$i.json 2>&1 || exit 1
done; done
rc=$?; tail -1 gpurun_out/abhp_tests.log; exit $rc
