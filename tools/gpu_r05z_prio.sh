#!/bin/bash
# A/B of LGS_OPT_PRIORITY_TAIL (28) on the default config-2 bench: bench lines
# with the option off/on, then one kernel trace with it on (k_cost in trace).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out
TAG=${1:-r05z}
mkdir -p $OUT
B="bench.py --steps 200 --warmup 10 --no-cpu --loop-line 0 --dropin-line 0 --sub-lines 0"
for arm in off on off on; do
  opt=""; [ $arm = on ] && opt="28=1"
  LGS_CTX_OPTIONS="$opt" timeout -k 10 300 python3 $B > $OUT/${TAG}_$arm.json 2> $OUT/${TAG}_$arm.err || exit $?
  python3 -c "import json,sys; d=json.loads(open('$OUT/${TAG}_$arm.json').read().strip().splitlines()[-1]); print('$arm', d['value'], d['p50_scan_match_ms'], d['p50_batch_call_ms'], d['kernels']['k_cost'])"
done
LGS_CTX_OPTIONS="28=1" timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${TAG}_trace -o run -- \
  python3 bench.py --steps 200 --warmup 10 --no-cpu --latency-calls 0 --loop-line 0 --dropin-line 0 --sub-lines 0 \
  > $OUT/${TAG}_trace.log 2>&1 || exit $?
f=$(find $OUT/${TAG}_trace -name '*kernel_stats.csv' | head -1)
grep -E "k_cost|k_coarse_list|k_fine_regs|k_seed" $f
echo done
