#!/usr/bin/env python3
"""Summarise rocprofv3 CSV output of tools/gpu_prof.sh into per-kernel stats.

    python tools/pmc_summary.py <trace_dir> <pmc_fetch_dir> <pmc_write_dir> <pmc_l2_dir> <out_prefix>

    [<liblgs_hip.so profiled>]   (env WORKLOAD: the bench workload profiled, default "match")

Writes <out_prefix>_kernel_stats.md (kernel-trace durations) and
<out_prefix>_pmc.json = {"lib_sha256": the profiled library's hash, "kernels":
{name: dispatches, avg duration, FETCH_SIZE / WRITE_SIZE per dispatch}};
bench.py takes roofline.traffic from it only for the same library build.  gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE
counts 64 B per 128-B request of wide coalesced reads, so the reported value is
doubled for those; our gathers are 8-B per lane, an access width the guide
lists as uncalibrated, so both the raw and the x2 figure are recorded and the
raw figure is the one reported as traffic (a lower bound)."""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def short(name: str) -> str:
    name = name.replace("(anonymous namespace)::", "")
    if "rocprim" in name:
        for k in ("partition", "lookback", "transform", "radix", "sort", "scan"):
            if k in name:
                return "rocprim::" + k
        return "rocprim::kernel"
    name = re.sub(r"^void ", "", name)
    return name.split("(")[0]


def one(d, pat):
    f = glob.glob(os.path.join(d, "**", pat), recursive=True)
    if not f:
        raise SystemExit(f"no {pat} under {d}")
    return f[0]


def counters(d):
    agg = defaultdict(lambda: defaultdict(list))
    for r in csv.DictReader(open(one(d, "*counter_collection.csv"))):
        agg[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return agg


def main():
    trace, fetch, write, l2, prefix = sys.argv[1:6]
    lib = sys.argv[6] if len(sys.argv) > 6 else os.path.join(os.path.dirname(os.path.dirname(
        os.path.abspath(__file__))), "my-lidar-graph-slam_amd", "lgs_amd", "liblgs_hip.so")
    rows = list(csv.DictReader(open(one(trace, "*kernel_trace.csv"))))
    dur = defaultdict(list)
    for r in rows:
        dur[short(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    total = sum(sum(v) for v in dur.values())
    lines = ["| kernel | calls | total_us | avg_us | min_us | max_us | % |", "|---|---|---|---|---|---|---|"]
    for k, v in sorted(dur.items(), key=lambda kv: -sum(kv[1])):
        lines.append(f"| {k} | {len(v)} | {sum(v):.1f} | {sum(v)/len(v):.3f} | {min(v):.3f} | {max(v):.3f} | "
                     f"{100*sum(v)/total:.1f} |")
    open(prefix + "_kernel_stats.md", "w").write("\n".join(lines) + "\n")
    print("\n".join(lines))
    cf, cw, cl = counters(fetch), counters(write), counters(l2)
    out = {}
    for k in sorted(dur):
        e = {"dispatches": len(dur[k]), "avg_us": round(sum(dur[k]) / len(dur[k]), 3)}
        if k in cf and cf[k].get("FETCH_SIZE"):
            v = cf[k]["FETCH_SIZE"]
            e["fetch_kb_per_dispatch"] = round(sum(v) / len(v), 1)
        if k in cw and cw[k].get("WRITE_SIZE"):
            v = cw[k]["WRITE_SIZE"]
            e["write_kb_per_dispatch"] = round(sum(v) / len(v), 1)
        if k in cl and cl[k].get("TCC_HIT_sum"):
            h, m = sum(cl[k]["TCC_HIT_sum"]), sum(cl[k].get("TCC_MISS_sum", [0]))
            e["l2_hit_rate"] = round(h / max(1.0, h + m), 4)
        if "fetch_kb_per_dispatch" in e:
            e["fetch_bytes_per_launch"] = round(1024.0 * e["fetch_kb_per_dispatch"])
        if "write_kb_per_dispatch" in e:
            e["write_bytes_per_launch"] = round(1024.0 * e["write_kb_per_dispatch"])
        out[k] = e
    import hashlib
    doc = {"lib_sha256": hashlib.sha256(open(lib, "rb").read()).hexdigest(),
           "workload": os.environ.get("WORKLOAD", "match"),
           "note": "rocprofv3 FETCH_SIZE / WRITE_SIZE (separate --pmc passes) per dispatch; gfx950 FETCH_SIZE counts "
                   "half the bytes of wide coalesced reads (MI355X_MICROARCH.md HBM section): bench.py doubles it",
           "kernels": out}
    json.dump(doc, open(prefix + "_pmc.json", "w"), indent=1)
    print(json.dumps(out.get("k_coarse_list", {}), indent=1))


if __name__ == "__main__":
    main()
