#!/bin/bash
# A/B of k_super_oct<9>'s load-pipeline depth (LGS_OCT_PIPE9) on the config-5 batch.
mkdir -p gpurun_out
for v in p8 p4 p12 p16 p8; do
  LGS_LIB=ablib/ab_$v.so timeout -k 10 240 python -u bench.py --workload loop --no-cpu > gpurun_out/pipe9_$v.json 2> gpurun_out/pipe9_$v.err || exit $?
  python3 -c "import json;d=json.loads(open('gpurun_out/pipe9_$v.json').read().strip().splitlines()[-1]);print('$v', d['value'], d['roofline_super']['avg_launch_ms'], d['roofline']['avg_launch_ms'])" | tee -a gpurun_out/pipe9.txt
done
