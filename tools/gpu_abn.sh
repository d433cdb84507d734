#!/bin/bash
# Alternated A/B bench runs of library variants: gpu_abn.sh <tag> "<bench args>" <rounds> base name1 name2 ...
# ("base" = the in-tree liblgs_hip.so, others = ablib/ab_<name>.so); one JSON line per run in
# gpurun_out/<tag>_<name>_<round>.json.  Every run has its own time limit; a crash stops the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
tag=$1; args=$2; rounds=$3; shift 3
for r in $(seq 1 $rounds); do
  for v in "$@"; do
    if [ "$v" = base ]; then lib=""; else lib="$PWD/ablib/ab_$v.so"; fi
    LGS_LIB=$lib timeout -k 10 300 python -u bench.py $args > gpurun_out/${tag}_${v}_$r.json 2> gpurun_out/${tag}_${v}_$r.err
    rc=$?
    echo "$v round $r rc=$rc $(python3 -c "import json,sys; d=json.load(open('gpurun_out/${tag}_${v}_$r.json')); print(d['value'], {k: v['avg_ms'] for k, v in d.get('kernels', {}).items()})" 2>/dev/null)"
    if [ $rc -ne 0 ]; then tail -5 gpurun_out/${tag}_${v}_$r.err; exit $rc; fi
  done
done
