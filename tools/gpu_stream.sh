#!/bin/bash
# config-4 frontend lines (both windows) with the per-phase breakdown
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-s}
timeout -k 10 400 python -u bench.py --workload stream --steps ${STEPS:-500} --cpu-seconds 5 > gpurun_out/${T}_stream_json.json 2> gpurun_out/${T}_stream_json.err &&
timeout -k 10 400 python -u bench.py --workload stream --window config2 --steps ${STEPS:-500} --cpu-seconds 5 > gpurun_out/${T}_stream_c2.json 2> gpurun_out/${T}_stream_c2.err
