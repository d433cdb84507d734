#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
LGS_LIB=tools/exp/ab_rb11.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_mapbuild.py tests/test_gpu_raycast.py > gpurun_out/abs11_tests.log 2>&1 &&
for v in base rb11; do
  lib=""; [ $v != base ] && lib=tools/exp/ab_$v.so
  LGS_LIB=$lib timeout -k 10 200 python bench.py --workload rebuild --no-cpu > gpurun_out/abr_$v.json 2>&1 || exit 1
  LGS_LIB=$lib timeout -k 10 200 python bench.py --workload stream --no-cpu > gpurun_out/abr_s_$v.json 2>&1 || exit 1
done
rc=$?; tail -1 gpurun_out/abs11_tests.log; exit $rc
