#!/bin/bash
# Whole-run memory-system counters of the match bench at two concurrency levels.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
i=0
for cfg in ${CFGS:-4x1 16x16}; do
  set -- ${cfg/x/ }
  while read -r counters; do
    [ -z "$counters" ] && continue
    i=$((i+1))
    GPU_MAX_HW_QUEUES=$1 timeout -k 10 300 rocprofv3 --pmc $counters --output-format csv -d $OUT/conc_q$1_s$2_$i -o run -- \
        python3 bench.py --steps 300 --warmup 5 --no-cpu --streams $2 > $OUT/conc_q$1_s$2_$i.log 2>&1 \
        || { echo "pass failed: $cfg $counters"; tail -5 $OUT/conc_q$1_s$2_$i.log; exit 1; }
    echo "ok $cfg: $counters"
  done <<LIST
TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum
TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_REQUEST_sum
TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum
TA_BUSY_avr TCC_BUSY_avr GRBM_GUI_ACTIVE
LIST
done
echo done
