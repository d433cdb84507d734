#!/bin/bash
# r05: merged window/long apply, in-place strips + two unit columns per thread
# for the superblock units -- parity (latest map, planes, matcher), the default
# bench, A/B with the one-column pass, config 4 A/B (merged on / off)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
tools/gpu_step.sh "k_tests|300|python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_latest.py tests/test_gpu_raycast.py tests/test_gpu_frontend.py tests/test_gpu_mapbuild.py tests/test_gpu_planes.py tests/test_gpu_rtcsm.py tests/test_gpu_keysort.py" \
  "bench|400|python -u bench.py --no-cpu > gpurun_out/r05k_bench.json 2> gpurun_out/r05k_bench.err" \
  "bench_1col|300|LGS_CTX_OPTIONS=33=0 python -u bench.py --no-cpu --sub-lines 0 > gpurun_out/r05k_bench_1col.json 2> gpurun_out/r05k_bench_1col.err" \
  "st_on|300|python -u bench.py --workload stream --steps 2000 --warmup 100 --no-cpu > gpurun_out/r05k_on.json" \
  "st_off|300|LGS_CTX_OPTIONS=32=0 python -u bench.py --workload stream --steps 2000 --warmup 100 --no-cpu > gpurun_out/r05k_off.json"
tools/gpu_step.sh "st_timing|300|LGS_STEP_TIMING=1 python -u bench.py --workload stream --steps 2000 --warmup 100 --no-cpu > gpurun_out/r05k_timing.json 2> gpurun_out/r05k_timing.err" \
  "st_trace|300|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r05k_trace -o run -- python3 bench.py --workload stream --steps 1000 --warmup 50 --no-cpu > gpurun_out/r05k_trace.log 2>&1"
