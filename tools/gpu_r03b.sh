#!/bin/bash
# r03: K1 changes (octet superblock bounds for up to 9 rows, edge-beam list in
# k_coarse_lanes): parity suites, then the config-5 and config-2 bench lines.
set -o pipefail
O=gpurun_out/r03b; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_loop.py \
    tests/test_gpu_rtcsm.py tests/test_gpu_batch.py tests/test_gpu_frontend.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 200 python -u bench.py --workload loop --no-cpu > $O/loop.json 2> $O/loop.err || exit 1
timeout -k 10 200 python -u bench.py --no-cpu --loop-line 0 --dropin-line 0 > $O/match.json 2> $O/match.err || exit 1
