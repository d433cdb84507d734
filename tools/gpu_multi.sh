#!/bin/bash
# multi-rank rehearsal on one GPU: 2 ranks (gloo collectives, both on GPU 0) and the RCCL group at world 1
export TMPDIR=/tmp
mkdir -p gpurun_out
[ -n "$SKIP_REHEARSE" ] || LGS_BENCH_REHEARSE=1 timeout -k 10 400 python -u bench.py --gpus 2 --steps 20 --warmup 3 --cpu-seconds 1 > gpurun_out/multi2.json 2> gpurun_out/multi2.err
rc=$?
echo "rehearse rc=$rc"; tail -c 400 gpurun_out/multi2.json; tail -3 gpurun_out/multi2.err
[ $rc -ne 0 ] && exit $rc
LGS_BENCH_DIST=1 timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr=127.0.0.1 --master-port=29511 bench.py --gpus 1 --steps 20 --warmup 3 --cpu-seconds 1 --dropin-line 0 > gpurun_out/dist1.json 2> gpurun_out/dist1.err
rc=$?
echo "dist1 rc=$rc"; tail -c 300 gpurun_out/dist1.json; tail -3 gpurun_out/dist1.err
exit $rc
