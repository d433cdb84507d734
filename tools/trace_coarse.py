#!/usr/bin/env python3
"""Split a rocprofv3 kernel trace's dispatches of one kernel into those that
ran alone on the GPU (no other dispatch overlapped them in time) and those
that shared it, and report each group's average duration -- the two figures
bench.py reports as `roofline_isolated` (the one-stream pass after the timed region)
and `roofline` (the timed region, several streams).

    python tools/trace_coarse.py <run_kernel_trace.csv> [kernel_substring] [algo_bytes_per_launch]
                                 [head_dispatches tail_dispatches]

Prints one JSON object; with the algorithmic bytes per launch (the bench
line's roofline.algo_bytes_per_launch) it adds the achieved GB/s and the
fraction of the 8 TB/s HBM peak for every group.  r06: also every dispatch
("all", what a whole-trace average -- pmc_summary's avg_us -- reports) and,
given the number of the kernel's dispatches before the timed region (the
warm-up calls, one stream at a time) and after it (the one-stream pass),
the timed region's own dispatches ("timed"): the same launches the line's
device-timed roofline averages, rocprof's duration of which also counts the
time a dispatch waits for CUs held by the other streams' kernels."""
import csv
import json
import sys


def main():
    path = sys.argv[1]
    name = sys.argv[2] if len(sys.argv) > 2 else "k_coarse_list"
    algo = float(sys.argv[3]) if len(sys.argv) > 3 else None
    head = int(sys.argv[4]) if len(sys.argv) > 4 else None
    tail = int(sys.argv[5]) if len(sys.argv) > 5 else 0
    rows = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], int(r["Stream_Id"]))
            for r in csv.DictReader(open(path))]
    rows.sort()
    # for each dispatch: does any other dispatch overlap [start, end)?
    alone, shared, every = [], [], []
    for i, (s, e, k, st) in enumerate(rows):
        if name not in k:
            continue
        overl = False
        for j in range(i - 1, -1, -1):        # earlier starts still running at s
            if rows[j][1] > s:
                overl = True
                break
            if s - rows[j][0] > 50_000_000:    # 50 ms back is enough
                break
        if not overl and i + 1 < len(rows) and rows[i + 1][0] < e:   # a later start before e
            overl = True
        (shared if overl else alone).append((e - s) / 1e3)
        every.append((e - s) / 1e3)
    out = {"kernel": name, "dispatches": len(alone) + len(shared)}
    groups = [("all", every), ("alone", alone), ("shared", shared)]
    if head is not None:
        groups.append(("timed", every[head:len(every) - tail]))
    for tag, v in groups:
        if not v:
            out[tag] = None
            continue
        avg = sum(v) / len(v)
        d = {"dispatches": len(v), "avg_us": round(avg, 3), "min_us": round(min(v), 3), "max_us": round(max(v), 3)}
        if algo:
            gbs = algo / (avg * 1e-6) / 1e9
            d["achieved_GBps"] = round(gbs, 1)
            d["frac_of_8TBps"] = round(gbs / 8000.0, 4)
        out[tag] = d
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
