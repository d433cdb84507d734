#!/bin/bash
# r03: config 4 with superblock pruning for every window (default) vs only for
# windows of >= 2 superblocks (LGS_OPT_PRUNE_MIN_SUPER 2: the frontend's json
# window then scores its 1 block per angle densely); alternated runs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=gpurun_out/r03g; mkdir -p $O
for i in 1 2; do
  for v in 1 2; do
    timeout -k 10 200 python -u bench.py --workload stream --no-cpu --ctx-option 21=$v > $O/p${v}_$i.json 2> $O/p${v}_$i.err || { tail -5 $O/p${v}_$i.err; exit 1; }
    python3 -c "import json;d=json.loads(open('$O/p${v}_$i.json').read().strip().splitlines()[-1]);print('min_super $v run $i:', d['value'], d['breakdown_per_step'])"
  done
done
