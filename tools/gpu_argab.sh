#!/bin/bash
# Bench A/B over bench.py argument sets of the same build.
# Usage: tools/gpu_argab.sh "--streams 1" "--streams 2 --batch 128" ...
export TMPDIR=/tmp
mkdir -p gpurun_out
i=0
for a in "$@"; do
  i=$((i+1))
  timeout -k 10 300 python -u bench.py --steps ${STEPS:-100} --warmup 10 --cpu-seconds 1 --loop-line 0 --dropin-line 0 $a > gpurun_out/argab_$i.json 2> gpurun_out/argab_$i.err || exit $?
  python3 -c "
import json; d=json.loads(open('gpurun_out/argab_$i.json').read().strip().splitlines()[-1])
r=d['roofline']
print(repr('$a'), d['value'], d['ms_per_step'], 'coarse_event_ms', r.get('avg_launch_ms'), 'frac', r.get('frac'))"
done
