#!/bin/bash
# quick A/B of bench variants (no CPU baseline), after the GPU parity tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for v in "$@"; do
  echo "== variant: $v"
  timeout -k 10 300 python bench.py --steps 200 --warmup 10 --no-cpu $v > gpurun_out/ab.log 2>&1 || { tail -20 gpurun_out/ab.log; exit 3; }
  python - <<'PY'
import json
l=[x for x in open('gpurun_out/ab.log') if x.startswith('{')][-1]
d=json.loads(l)
print('value', d['value'], 'p50', d['p50_scan_match_ms'], 'roof', d['roofline']['achieved'], d['roofline']['frac'])
print({k: v['avg_ms'] for k, v in d['kernels'].items()})
PY
done
