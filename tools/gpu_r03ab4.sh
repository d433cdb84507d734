#!/bin/bash
# r03: config-4 frontend with superblock pruning (default) vs every coarse
# block scored (--ctx-option 9=0, LGS_OPT_SUPER_PRUNE), alternated on one box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03ab4}; rm -rf $O; mkdir -p $O
uptime
for i in 1 2 3; do
for v in prune dense; do
opt=""; [ $v = dense ] && opt="${ALT:---ctx-option 9=0}"
timeout -k 10 300 python -u bench.py --workload stream --no-cpu $opt > $O/s_$v$i.json 2> $O/s_$v$i.err || { tail -5 $O/s_$v$i.err; exit 1; }
python3 -c "import json;d=json.loads([l for l in open('$O/s_$v$i.json') if l.startswith('{')][-1]);print('$v', d['value'], d['ms_per_step'])"
done
done
