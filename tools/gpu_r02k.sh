#!/bin/bash
# r02 session 3: f4 (MapSaver / patch allocation) GPU parity + the ray-cast and map-build suites
export TMPDIR=/tmp
mkdir -p gpurun_out
T=r02k
timeout -k 10 600 python -u -m pytest tests/test_gpu_io.py tests/test_gpu_raycast.py tests/test_gpu_mapbuild.py tests/test_gpu_frontend.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_tests.log 2>&1
rc=$?
tail -15 gpurun_out/${T}_tests.log
exit $rc
