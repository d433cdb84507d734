#!/bin/bash
# Bench A/B over environment settings of the same build.
# Usage: tools/gpu_envab.sh "" "LGS_SET_GROUP=8" ...   ("" = defaults)
export TMPDIR=/tmp
mkdir -p gpurun_out
i=0
for e in "$@"; do
  i=$((i+1))
  env $e timeout -k 10 300 python -u bench.py --steps ${STEPS:-100} --warmup 10 --cpu-seconds 1 --loop-line 0 --dropin-line 0 ${BENCH_ARGS} > gpurun_out/envab_$i.json 2> gpurun_out/envab_$i.err || exit $?
  python3 -c "
import json; d=json.loads(open('gpurun_out/envab_$i.json').read().strip().splitlines()[-1])
print(repr('$e'), d['value'], {k: (v['launches'], v['avg_ms']) for k, v in d.get('kernels', {}).items() if k in ('k_precompute','k_super_planes','k_coarse','k_super')})"
done
