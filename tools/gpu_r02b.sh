#!/bin/bash
# r02 pass b: -m gpu suite, default bench (config 2 + config-5 sub-line), the
# rank-spawn path rehearsed on one GPU, then the profile of the default command.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02b_gpu_tests.log 2>&1 &&
timeout -k 10 600 python -u bench.py > gpurun_out/r02b_bench.json 2> gpurun_out/r02b_bench.err &&
LGS_BENCH_REHEARSE=1 timeout -k 10 300 python -u bench.py --gpus 2 --steps 10 --warmup 2 --no-cpu --latency-calls 5 --loop-line 1 > gpurun_out/r02b_bench_g2.json 2> gpurun_out/r02b_bench_g2.err &&
STEPS=100 WARMUP=5 bash tools/gpu_prof.sh r02b
