#!/bin/bash
# Lone-scan (batch 1) latency A/B: default build vs ablib variants; per-kernel
# one-stream event times of the lone path.  Usage: tools/gpu_lone_ab.sh <variant> ...
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in default "$@"; do
  if [ $v = default ]; then L=""; else L="LGS_LIB=ablib/$v.so"; fi
  env $L timeout -k 10 300 python -u bench.py --batch 1 --streams 1 --steps 400 --no-cpu --loop-line 0 --dropin-line 0 > gpurun_out/lone_$v.json 2> gpurun_out/lone_$v.err || exit $?
  python3 -c "
import json; d=json.loads(open('gpurun_out/lone_$v.json').read().strip().splitlines()[-1])
print('$v', d['value'], 'p50', d['p50_scan_match_ms'], 'p90', d['p90_scan_match_ms'], {k: v['avg_ms'] for k, v in d['kernels'].items()})"
done
