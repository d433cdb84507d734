#!/usr/bin/env python3
"""Why a streaming kernel slows down under two streams: for each dispatch of
the named kernel that another dispatch overlapped, sum the HBM bytes of every
dispatch over the interval (PMC counter bytes per launch from a
pmc_summary-style JSON -- 2 x FETCH_SIZE (gfx950) + WRITE_SIZE -- spread
uniformly over each dispatch's duration) and report the kernel's own rate,
the aggregate rate of everything running beside it, and which kernels it
shared the GPU with.

    python tools/overlap_bw.py <run_kernel_trace.csv> <pmc.json> <kernel_substring>"""
import csv
import json
import sys
from collections import Counter


def short(name):
    return name.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0].strip()


def main():
    trace, pmc, name = sys.argv[1], sys.argv[2], sys.argv[3]
    kb = json.load(open(pmc))["kernels"]
    bytes_of = {}
    for k, v in kb.items():
        bytes_of[k.split("<")[0]] = 2.0 * v["fetch_bytes_per_launch"] + v["write_bytes_per_launch"]
    rows = []
    for r in csv.DictReader(open(trace)):
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        rows.append((s, e, short(r["Kernel_Name"])))
    rows.sort()

    def nbytes(k):
        return bytes_of.get(k.split("<")[0], 0.0)

    out = {"kernel": name, "bytes_per_launch": None, "alone": None, "shared": None, "shared_with": {}}
    alone, shared = [], []
    partners = Counter()
    for i, (s, e, k) in enumerate(rows):
        if name not in k:
            continue
        out["bytes_per_launch"] = nbytes(k)
        agg = nbytes(k)
        ov = False
        for j in range(max(0, i - 64), min(len(rows), i + 64)):
            if j == i:
                continue
            s2, e2, k2 = rows[j]
            lo, hi = max(s, s2), min(e, e2)
            if hi > lo:
                ov = True
                agg += nbytes(k2) * (hi - lo) / max(1, e2 - s2)
                partners[k2] += (hi - lo) / 1e3
        dur = (e - s) / 1e9
        (shared if ov else alone).append((dur, nbytes(k) / dur, agg / dur))
    for tag, v in (("alone", alone), ("shared", shared)):
        if v:
            n = len(v)
            out[tag] = {"dispatches": n, "avg_us": round(1e6 * sum(x[0] for x in v) / n, 1),
                        "own_TBps": round(sum(x[1] for x in v) / n / 1e12, 2),
                        "aggregate_TBps": round(sum(x[2] for x in v) / n / 1e12, 2)}
    tot = sum(partners.values())
    out["shared_with"] = {k: round(t / tot, 3) for k, t in partners.most_common(6)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
