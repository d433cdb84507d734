#!/bin/bash
# kernel + HIP API trace of the config-4 frontend (C++ driver); keeps the stats tables only
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 rocprofv3 --kernel-trace --hip-trace --stats --output-format csv -d /tmp/prof_stream -o run -- python3 bench.py --workload stream --steps ${STEPS:-2000} --cpu-seconds 1 > gpurun_out/prof_stream.log 2>&1
rc=$?
mkdir -p gpurun_out/prof_stream
cp /tmp/prof_stream/*stats.csv gpurun_out/prof_stream/ 2>/dev/null
head -25 gpurun_out/prof_stream/run_kernel_stats.csv | cut -d, -f1-8
head -25 gpurun_out/prof_stream/run_hip_api_stats.csv | cut -d, -f1-8
exit $rc
