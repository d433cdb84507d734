#!/bin/bash
# r03: HIP API + kernel trace of a short config-4 stream run (host timeline per step).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=gpurun_out/r03j; rm -rf $O; mkdir -p $O
timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --memory-copy-trace --output-format csv -d $O/trace -o run -- python3 bench.py --workload stream --steps 300 --warmup 20 --no-cpu > $O/trace.log 2>&1 || { tail -5 $O/trace.log; exit 1; }
ls -la $O/trace
