#!/bin/bash
# r04k: small-window tests, k_match_small probes, config-4 stream
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
tools/gpu_step.sh "tests|300|python -u -m pytest tests/test_gpu_small.py tests/test_gpu_frontend.py tests/test_gpu_rtcsm.py -x -q --timeout 120 --timeout-method thread" || exit $?
tools/gpu_step.sh "probe|120|LGS_LIB=$PWD/ablib/ab_probe.so python tools/probe_small.py 12 > gpurun_out/probe.out 2>&1" || exit $?
grep "probe match_small" gpurun_out/probe.out | tail -3
for r in 1 2; do
tools/gpu_step.sh "st$r|200|python bench.py --workload stream --steps 2000 --no-cpu > gpurun_out/st$r.json" || exit $?
python3 -c "import json;d=json.loads(open('gpurun_out/st$r.json').read().strip().splitlines()[-1]);print(d['value'], d['breakdown_per_step'])"
done
