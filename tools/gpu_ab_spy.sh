#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in default ab_noinv ab_rows16 ab_rows4; do
  if [ $v = default ]; then L=""; else L="LGS_LIB=ablib/$v.so"; fi
  env $L timeout -k 10 300 python -u bench.py --steps 100 --warmup 10 --cpu-seconds 1 --loop-line 0 --dropin-line 0 > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err || exit $?
  python3 -c "
import json; d=json.loads(open('gpurun_out/ab_$v.json').read().strip().splitlines()[-1])
print('$v', d['value'], {k: v['avg_ms'] for k, v in d.get('kernels', {}).items() if k in ('k_super_planes','k_project','k_super','k_coarse')})"
done
