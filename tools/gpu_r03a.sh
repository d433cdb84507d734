#!/bin/bash
# r03: config-3 refine after the bit-exact K4, and the batch-64 vs batch-128 A/B
set -o pipefail
O=gpurun_out/r03a; mkdir -p $O
timeout -k 10 200 python -u bench.py --workload refine --no-cpu > $O/refine.json 2> $O/refine.err || exit 1
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --batch 64 --steps 400 --no-cpu --loop-line 0 --dropin-line 0 --latency-calls 0 > $O/b64_$i.json 2> $O/b64_$i.err || exit 1
  timeout -k 10 200 python -u bench.py --batch 128 --steps 200 --no-cpu --loop-line 0 --dropin-line 0 --latency-calls 0 > $O/b128_$i.json 2> $O/b128_$i.err || exit 1
done
