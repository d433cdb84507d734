#!/bin/bash
# Pipeline counters of the K1 kernels (one pass per counter group, no tracing
# domains), summarised per kernel into gpurun_out/k1_pmc.csv.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
B="bench.py --steps 30 --warmup 3 --no-cpu --latency-calls 0 --loop-line 0 --dropin-line 0 --sub-lines 0 --streams 1"
i=0; dirs=""
while read -r counters; do
  [ -z "$counters" ] && continue
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $counters --output-format csv -d $OUT/k1_$i -o run -- python3 $B > $OUT/k1_$i.log 2>&1 \
      || { echo "pass $i failed: $counters"; tail -5 $OUT/k1_$i.log; exit 1; }
  echo "pass $i ok: $counters"; dirs="$dirs $OUT/k1_$i"
done <<LIST
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_SALU
TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum
TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE GRBM_COUNT
TD_BUSY_avr TD_TC_STALL_sum TCC_HIT_sum TCC_MISS_sum
LIST
python3 tools/pmc_table.py $dirs > $OUT/k1_pmc.csv && cat $OUT/k1_pmc.csv
find $OUT -path "$OUT/k1_*" -name '*.csv' -size +20M -delete
echo done
