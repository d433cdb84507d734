#!/bin/bash
# r04d: k_match_small phase probes: base, no gathers, no sums (timing-only variants)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
for v in probe probe_ng probe_ns; do
  tools/gpu_step.sh "$v|120|LGS_LIB=$PWD/ablib/ab_$v.so python tools/probe_small.py 12 > gpurun_out/$v.out 2>&1" || exit $?
  grep "probe match_small" gpurun_out/$v.out | tail -3
done
