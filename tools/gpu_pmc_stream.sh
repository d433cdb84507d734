#!/bin/bash
# Pipeline counters of the config-4 (stream) kernels: one PMC pass per counter
# group over a 1500-step run, summarised per kernel.  Usage: tools/gpu_pmc_stream.sh TAG
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
TAG=${1:-r03}
OUT=gpurun_out/pmc_stream_$TAG; mkdir -p $OUT
B="bench.py --workload stream --steps 1500 --no-cpu"
i=0; dirs=""
while read -r counters; do
  [ -z "$counters" ] && continue
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --pmc $counters --output-format csv -d $OUT/p$i -o run -- python3 $B > $OUT/p$i.log 2>&1 \
      || { echo "pass $i failed: $counters"; tail -5 $OUT/p$i.log; exit 1; }
  echo "pass $i ok: $counters"; dirs="$dirs $OUT/p$i"
done <<LIST
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_SALU
TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum
SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAIT_ANY SQ_INSTS_SMEM GRBM_GUI_ACTIVE GRBM_COUNT
FETCH_SIZE
WRITE_SIZE
LIST
python3 tools/pmc_table.py $dirs > $OUT/table.csv && grep -E "^(kernel|k_apply|k_sort|k_emit|k_run)" $OUT/table.csv
find $OUT -name '*.csv' -size +20M -delete
echo done
