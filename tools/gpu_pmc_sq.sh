#!/bin/bash
# SQ / TCP counters of the K1 kernels (separate passes; no tracing domains).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
B="bench.py --steps 30 --warmup 3 --no-cpu"
i=0
while read -r counters; do
  [ -z "$counters" ] && continue
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $counters --output-format csv -d $OUT/sq$i -o run -- python3 $B > $OUT/sq$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/sq$i.log; exit 1; }
  echo "pass $i ok: $counters"
done <<LIST
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY
SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM
TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum
SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS
LIST
