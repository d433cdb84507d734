#!/bin/bash
# r03: SQ counters of the f2 rebuild kernels (k_apply, k_emit, k_runmask, K3 sort passes).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=gpurun_out/pmc_rebuild; rm -rf $O; mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-include-regex "k_apply\b|k_emit|k_runmask|k_sort_down|k_sort_up" --output-format csv -d $O/p1 -o run -- python3 bench.py --workload rebuild --steps 10 --no-cpu > $O/p1.log 2>&1 || { tail -5 $O/p1.log; exit 1; }
python3 - <<'PY'
import csv, glob, collections
f = glob.glob("gpurun_out/pmc_rebuild/p1/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"].split("(")[0][-40:]
    acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
    n[(k, r["Counter_Name"])] += 1
for k, d in acc.items():
    c = n[(k, "SQ_WAVES")]
    print(k, {kk: round(v / max(1, c)) for kk, v in sorted(d.items())})
PY
