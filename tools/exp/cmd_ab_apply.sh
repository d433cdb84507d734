#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_mapbuild.py tests/test_gpu_raycast.py > gpurun_out/f2_tests.log 2>&1 &&
timeout -k 10 200 python bench.py --workload rebuild --no-cpu > gpurun_out/ab_base.json 2>&1 &&
LGS_LIB=tools/exp/ab_nomath.so timeout -k 10 200 python bench.py --workload rebuild --no-cpu > gpurun_out/ab_nomath.json 2>&1
rc=$?; tail -1 gpurun_out/f2_tests.log; exit $rc
