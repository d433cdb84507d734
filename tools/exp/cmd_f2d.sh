#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_mapbuild.py tests/test_gpu_raycast.py > gpurun_out/f2_tests.log 2>&1 &&
timeout -k 10 240 python bench.py --workload rebuild --no-cpu > gpurun_out/f2_rebuild.json 2> gpurun_out/f2_rebuild.err &&
timeout -k 10 240 python bench.py --workload stream --no-cpu > gpurun_out/f2_stream.json 2> gpurun_out/f2_stream.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_rebuild -o run -- \
  python3 bench.py --workload rebuild --no-cpu --steps 10 > gpurun_out/prof_rebuild.log 2>&1
rc=$?
tail -2 gpurun_out/f2_tests.log
exit $rc
