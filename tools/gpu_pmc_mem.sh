#!/bin/bash
# Memory-system counters per kernel, single-stream match bench (separate passes).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
B="bench.py --steps 30 --warmup 3 --no-cpu --streams 1 ${BENCH_ARGS}"
i=0
while read -r counters; do
  [ -z "$counters" ] && continue
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $counters --output-format csv -d $OUT/mem$i -o run -- python3 $B > $OUT/mem$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/mem$i.log; exit 1; }
  echo "pass $i ok: $counters"
done <<LIST
TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum
TCC_REQ_sum TCC_HIT_sum TCC_MISS_sum
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES
SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_SMEM
FETCH_SIZE
WRITE_SIZE
LIST
python3 tools/pmc_table.py $(ls -d $OUT/mem*/) > $OUT/mem_table.csv
echo done
