#!/bin/bash
# torch-first runtime sharing (forced RCCL group at world 1) + f2 bench lines
set -o pipefail
mkdir -p gpurun_out
export LGS_BENCH_DIST=1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 \
  bench.py --workload match --steps 100 --no-cpu > gpurun_out/td_match.json 2> gpurun_out/td_match.err &&
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29512 \
  bench.py --workload loop --steps 2 --no-cpu > gpurun_out/td_loop.json 2> gpurun_out/td_loop.err &&
unset LGS_BENCH_DIST &&
timeout -k 10 240 python bench.py --workload match --steps 100 --no-cpu > gpurun_out/nd_match.json 2> gpurun_out/nd_match.err &&
timeout -k 10 240 python bench.py --workload rebuild > gpurun_out/f2_rebuild.json 2> gpurun_out/f2_rebuild.err &&
timeout -k 10 240 python bench.py --workload stream --no-cpu > gpurun_out/f2_stream.json 2> gpurun_out/f2_stream.err
