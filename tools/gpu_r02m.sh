#!/bin/bash
# r02 session 3: full GPU suite after the linsolve restructure + refine bench
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r02m}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_tests.log 2>&1
rc=$?
tail -5 gpurun_out/${T}_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --workload refine --cpu-seconds 5 > gpurun_out/${T}_refine.json 2> gpurun_out/${T}_refine.err
rc2=$?
tail -c 600 gpurun_out/${T}_refine.json
exit $(( rc > rc2 ? rc : rc2 ))
