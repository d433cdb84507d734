#!/bin/bash
# Config-5 (--workload loop) profile: kept-superblock statistics, the bench
# line, a kernel-trace pass and separate PMC passes (HBM bytes, L2, pipeline
# counters) of the same command.  Every step has its own time limit; the
# script stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
TAG=${1:-r03}
OUT=gpurun_out/loop_$TAG; mkdir -p $OUT
B="bench.py --workload loop --steps ${STEPS:-4} --warmup 1 --no-cpu"
timeout -k 10 120 python3 tools/diag_loop_kept.py > $OUT/kept.txt 2>&1 || { tail -5 $OUT/kept.txt; exit 1; }
timeout -k 10 120 python3 $B > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $B \
    > $OUT/trace.log 2>&1 || { tail -5 $OUT/trace.log; exit 1; }
i=0
while read -r counters; do
  [ -z "$counters" ] && continue
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $counters --output-format csv -d $OUT/pmc_$i -o run -- python3 $B \
      > $OUT/pmc_$i.log 2>&1 || { echo "pass $i failed: $counters"; tail -5 $OUT/pmc_$i.log; exit 1; }
  echo "pass $i ok: $counters"
done <<LIST
FETCH_SIZE
WRITE_SIZE
TCC_HIT_sum TCC_MISS_sum
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_SALU
TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum
TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE GRBM_COUNT
LIST
find $OUT -name '*.csv' -size +20M -delete
echo done
