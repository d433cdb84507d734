#!/bin/bash
# LDS counters of the config-2 kernels (one pass, no tracing domains).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
B="bench.py --steps 30 --warmup 3 --no-cpu --latency-calls 0 --loop-line 0 --dropin-line 0 --streams 1"
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAVES --output-format csv -d $OUT/lds_1 -o run -- python3 $B > $OUT/lds_1.log 2>&1 || { tail -5 $OUT/lds_1.log; exit 1; }
python3 tools/pmc_table.py $OUT/lds_1 > $OUT/lds_pmc.csv && cat $OUT/lds_pmc.csv
find $OUT -path "$OUT/lds_1*" -name '*.csv' -size +20M -delete
