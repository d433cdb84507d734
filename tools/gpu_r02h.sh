#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T=r02h
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python -u bench.py --workload stream --cpu-seconds 8 > gpurun_out/${T}_stream_json.json 2> gpurun_out/${T}_stream_json.err &&
timeout -k 10 400 python -u bench.py --workload stream --fused 0 --steps 3000 --no-cpu > gpurun_out/${T}_stream_json_unfused.json 2> gpurun_out/${T}_stream_json_unfused.err &&
timeout -k 10 400 python -u bench.py --workload stream --window config2 --cpu-seconds 8 > gpurun_out/${T}_stream_c2.json 2> gpurun_out/${T}_stream_c2.err
