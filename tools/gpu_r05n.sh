#!/bin/bash
# r05: wide seed (16 candidate superblocks' best members) -- matcher parity,
# seed diagnostic, bench A/B (wide on / off)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
tools/gpu_step.sh "k_tests|400|python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_batch.py tests/test_gpu_rtcsm.py tests/test_gpu_planes.py tests/test_gpu_loop.py tests/test_gpu_frontend.py" \
  "diag_seed|200|python -u tools/diag_seed.py > gpurun_out/diag_seed_wide.log 2>&1" \
  "bench_wide|300|python -u bench.py --no-cpu --sub-lines 0 --loop-line 0 --dropin-line 0 > gpurun_out/r05n_wide.json 2> gpurun_out/r05n_wide.err" \
  "bench_narrow|300|LGS_CTX_OPTIONS=32=0 python -u bench.py --no-cpu --sub-lines 0 --loop-line 0 --dropin-line 0 > gpurun_out/r05n_narrow.json 2> gpurun_out/r05n_narrow.err" \
  "bench_wide2|300|python -u bench.py --no-cpu --sub-lines 0 --loop-line 0 --dropin-line 0 > gpurun_out/r05n_wide2.json 2> gpurun_out/r05n_wide2.err"
