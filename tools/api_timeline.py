#!/usr/bin/env python3
"""Host/device timeline of one config-4 frontend step from a rocprofv3
--hip-trace --kernel-trace run: HIP API calls of the driving thread (runs of
the same call folded) interleaved with kernel execution, times in us relative
to the step's first k_project launch call.

    python tools/api_timeline.py <trace_dir> [step_index]"""
import csv
import sys
from collections import Counter


def main():
    d = sys.argv[1]
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 150
    api = [r for r in csv.DictReader(open(f"{d}/run_hip_api_trace.csv"))]
    kern = [r for r in csv.DictReader(open(f"{d}/run_kernel_trace.csv"))]
    corr = {r["Correlation_Id"]: r for r in kern}
    proj = [r for r in kern if "k_project" in r["Kernel_Name"]]
    t0 = int(corr[proj[k]["Correlation_Id"]]["Start_Timestamp"])
    a0 = [r for r in api if r["Correlation_Id"] == proj[k]["Correlation_Id"]][0]
    t0 = int(a0["Start_Timestamp"])
    t1 = int([r for r in api if r["Correlation_Id"] == proj[k + 1]["Correlation_Id"]][0]["Start_Timestamp"])
    tid = a0["Thread_Id"]
    ev = []
    for r in api:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if r["Thread_Id"] == tid and t0 <= s < t1:
            ev.append((s, "api", r["Function"], e - s, r["Correlation_Id"]))
    for r in kern:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if t0 <= s < t1:
            ev.append((s, "gpu", r["Kernel_Name"].split("(")[0].replace("(anonymous namespace)::", "")[:40], e - s, ""))
    ev.sort()
    fold = []
    for s, kind, name, dur, c in ev:
        if fold and fold[-1][1] == kind == "api" and fold[-1][2] == name:
            fold[-1][3] += dur
            fold[-1][5] += 1
            continue
        fold.append([s, kind, name, dur, c, 1])
    for s, kind, name, dur, c, n in fold:
        ind = "" if kind == "api" else " " * 50
        print(f"{(s - t0) / 1e3:8.1f} {ind}{name:40s} {dur / 1e3:7.1f}" + (f" x{n}" if n > 1 else ""))
    print(f"step {(t1 - t0) / 1e3:.1f} us")
    tot = Counter()
    cnt = Counter()
    for s, kind, name, dur, c in ev:
        if kind == "api":
            tot[name] += dur
            cnt[name] += 1
    for name, v in tot.most_common(12):
        print(f"  {name:40s} {v / 1e3:7.1f} us  x{cnt[name]}")


if __name__ == "__main__":
    main()
