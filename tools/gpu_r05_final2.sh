#!/bin/bash
# r05 final (2): the final script's passes, then the other workloads' PMC summaries for the same library
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
TAG=${1:-r05_vf4}
tools/gpu_r05_final.sh $TAG || exit $?
tools/gpu_prof_workloads.sh $TAG loop loop_bb rebuild || exit $?
