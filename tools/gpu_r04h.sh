#!/bin/bash
# r04h: kernel trace of loop_bb (replay-kernel duration spread)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
tools/gpu_step.sh "bbtests|300|python -u -m pytest tests/test_gpu_bb.py tests/test_gpu_loop.py -x -q --timeout 120 --timeout-method thread" "bbtrace|300|rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_bb -o run -- python3 bench.py --workload loop_bb --no-cpu > gpurun_out/bbtrace.json && mkdir -p gpurun_out/prof_bb && cp /tmp/prof_bb/*kernel_stats.csv /tmp/prof_bb/*kernel_trace.csv gpurun_out/prof_bb/" || exit $?
python3 - <<'PY'
import csv
rows=[r for r in csv.DictReader(open('gpurun_out/prof_bb/run_kernel_trace.csv'))]
for name in ('k_bb_replay','k_bb_score','k_bb_rescore','k_bb_trig','k_bb_expand'):
    d=[(int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3 for r in rows if name in r['Kernel_Name']]
    if d: print(name, len(d), 'min %.1f med %.1f max %.1f us' % (min(d), sorted(d)[len(d)//2], max(d)), [round(x) for x in d[-14:]] if name=='k_bb_replay' else '')
PY
