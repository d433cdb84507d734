#!/bin/bash
# Device-throughput share of each stage: 16-stream match bench with one stage skipped.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=gpurun_out; mkdir -p $OUT
for sk in none k_precompute,k_super_planes k_project k_super k_seed k_coarse k_select,k_fine,k_replay k_cost "k_project,k_super,k_seed,k_coarse,k_select,k_fine,k_replay,k_cost,k_precompute,k_super_planes"; do
  a=""; [ "$sk" != none ] && a="--skip-kernels $sk"
  timeout -k 10 300 python bench.py --no-cpu --steps 800 --warmup 10 --streams ${S:-8} $a > $OUT/skip.log 2>&1 || { tail -5 $OUT/skip.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/skip.log').read().strip().splitlines()[-1]); print('skip %-40s %9.1f scans/s  p50 %.4f ms' % ('$sk'[:40], d['value'], d['p50_scan_match_ms']))"
done
