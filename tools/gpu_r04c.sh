#!/bin/bash
# r04c: GPU suite, config-4 stream (small window, post records A/B), k_match_small phase probes
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
tools/gpu_step.sh "gputests|600|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" || exit $?
tools/gpu_step.sh "probe|120|LGS_LIB=$PWD/ablib/ab_probe.so python tools/probe_small.py 20 > gpurun_out/probe.out 2>&1" || exit $?
grep "probe match_small" gpurun_out/probe.out | tail -5
for r in 1 2; do
  tools/gpu_step.sh "st_$r|200|python bench.py --workload stream --steps 2000 --no-cpu > gpurun_out/st_$r.json" \
    "st_post_$r|200|python bench.py --workload stream --steps 2000 --no-cpu --ctx-option 26=1 > gpurun_out/st_post_$r.json" || exit $?
done
