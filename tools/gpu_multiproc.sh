#!/bin/bash
# Aggregate match throughput of P concurrent bench processes on one GPU
# (per-process host limits vs device limits).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=gpurun_out; mkdir -p $OUT
P=${P:-2}
pids=()
for i in $(seq 1 $P); do
  timeout -k 10 300 python bench.py --no-cpu --steps ${BENCH_STEPS:-1500} --warmup 10 --streams ${S:-3} > $OUT/mp_$i.log 2>&1 &
  pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait $p || rc=$?; done
for i in $(seq 1 $P); do python3 -c "import json; d=json.loads(open('$OUT/mp_$i.log').read().strip().splitlines()[-1]); print('proc $i', d['value'], d['p50_scan_match_ms'])"; done
exit $rc
