#!/bin/bash
# r04e: GPU suite (k_post default on), k_match_small (barrier-free) probes, config-4 stream A/B of k_post
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
tools/gpu_step.sh "gputests|600|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" || exit $?
tools/gpu_step.sh "probe|120|LGS_LIB=$PWD/ablib/ab_probe.so python tools/probe_small.py 12 > gpurun_out/probe.out 2>&1" || exit $?
grep "probe match_small" gpurun_out/probe.out | tail -3
for r in 1 2; do
  tools/gpu_step.sh "st_$r|200|python bench.py --workload stream --steps 2000 --no-cpu > gpurun_out/st_$r.json" \
    "st_nopost_$r|200|python bench.py --workload stream --steps 2000 --no-cpu --ctx-option 26=0 > gpurun_out/st_nopost_$r.json" || exit $?
done
tools/gpu_step.sh "bench|400|python bench.py > gpurun_out/bench.json"
