#!/bin/bash
# r03: config 4 (stream) and f2 (rebuild) after the K3 sort + incremental latest map:
# bench lines, then a kernel trace of a 2000-step stream run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=gpurun_out/r03d; mkdir -p $O
timeout -k 10 300 python -u bench.py --workload stream > $O/stream.json 2> $O/stream.err || { tail -5 $O/stream.err; exit 1; }
tail -c 900 $O/stream.json
timeout -k 10 300 python -u bench.py --workload rebuild --no-cpu > $O/rebuild.json 2> $O/rebuild.err || { tail -5 $O/rebuild.err; exit 1; }
tail -c 600 $O/rebuild.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --workload stream --steps 2000 --no-cpu > $O/trace.log 2>&1 || { tail -5 $O/trace.log; exit 1; }
find $O/trace -name '*kernel_trace.csv' -delete
echo done
