#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
B=tools/exp/dispatch
for args in "1 20000 1 64" "4 20000 1 64" "16 20000 1 64" "1 20000 421 256" "4 20000 421 256" "16 20000 421 256" "4 20000 1 64 1" "16 20000 1 64 1" "16 20000 421 256 1"; do
  set -- $args
  q=4; [ "$1" -ge 8 ] && q=16
  GPU_MAX_HW_QUEUES=$q timeout -k 10 60 $B $args || exit $?
done
