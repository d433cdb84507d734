#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_frontend.py tests/test_gpu_mapbuild.py tests/test_cpp_adapter.py > gpurun_out/f3_tests.log 2>&1 &&
timeout -k 10 300 python bench.py --workload stream > gpurun_out/f3_stream.json 2> gpurun_out/f3_stream.err &&
timeout -k 10 240 python bench.py --workload stream --interp 0 --no-cpu > gpurun_out/f3_stream_raw.json 2>> gpurun_out/f3_stream.err
rc=$?; tail -3 gpurun_out/f3_tests.log; exit $rc
