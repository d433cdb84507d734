#!/bin/bash
# r05: device hit points for map rebuilds -- parity, then the f2 line with and without
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
tools/gpu_step.sh "t_map|400|python -u -m pytest tests/test_gpu_mapbuild.py tests/test_gpu_raycast.py tests/test_gpu_latest.py tests/test_gpu_io.py -x -q --timeout 120 --timeout-method thread" \
  "f2_dev|300|LGS_F2_TIMING=1 python -u bench.py --workload rebuild --steps 20 --warmup 3 > gpurun_out/r05g_f2_dev.json 2> gpurun_out/r05g_f2_dev.err" \
  "f2_host|300|LGS_CTX_OPTIONS=31=0 python -u bench.py --workload rebuild --steps 20 --warmup 3 --no-cpu > gpurun_out/r05g_f2_host.json 2> gpurun_out/r05g_f2_host.err"
