#!/usr/bin/env python3
"""One line per bench JSON log: value, latencies, roofline frac, per-kernel ms."""
import json
import sys

for f in sys.argv[1:]:
    lines = [x for x in open(f) if x.startswith("{")]
    if not lines:
        print(f, "no json")
        continue
    d = json.loads(lines[-1])
    r = d.get("roofline") or {}
    print(f"{f}: value={d['value']} p50={d.get('p50_scan_match_ms')} batch_ms={d.get('p50_batch_call_ms')} "
          f"frac={r.get('frac')} coarse={d.get('coarse_blocks_scored_mean')} fine={d.get('fine_blocks_refined_mean')}")
    print("   ", {k: round(v["avg_ms"], 4) for k, v in (d.get("kernels") or {}).items()})
