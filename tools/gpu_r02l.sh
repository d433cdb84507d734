#!/bin/bash
# r02 session 3: linsolve (config 3) restructure -- parity tests + refine bench
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r02l}
timeout -k 10 600 python -u -m pytest tests/test_gpu_linsolve.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_ls_tests.log 2>&1
rc=$?
tail -5 gpurun_out/${T}_ls_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --workload refine --cpu-seconds 5 > gpurun_out/${T}_refine.json 2> gpurun_out/${T}_refine.err
rc2=$?
tail -c 1500 gpurun_out/${T}_refine.json
exit $(( rc > rc2 ? rc : rc2 ))
