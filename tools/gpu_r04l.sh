#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
tools/gpu_step.sh "probe|120|LGS_LIB=$PWD/ablib/ab_probe.so python tools/probe_small.py 12 > gpurun_out/probe.out 2>&1" || exit $?
grep "probe match_small" gpurun_out/probe.out | tail -4
