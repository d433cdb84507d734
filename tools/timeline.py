"""Kernel-trace timeline analysis (rocprofv3 --kernel-trace csv): GPU busy
fraction (union of kernel intervals) over the densest window, per-kernel
average duration, and gaps between consecutive kernels of one queue."""
import csv
import sys
from collections import defaultdict


def load(path):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name,
                         r.get("Queue_Id", r.get("Stream_Id", "0"))))
    rows.sort()
    return rows


def main(path, skip_frac=0.3, take_frac=0.4):
    rows = load(path)
    # the timed bench region: take the middle of the match kernels
    ks = [r for r in rows if r[2].startswith("k_")]
    n = len(ks)
    sel = ks[int(n * skip_frac): int(n * (skip_frac + take_frac))]
    t0, t1 = sel[0][0], max(r[1] for r in sel)
    busy, cur_s, cur_e = 0, None, None
    for s, e, _, _ in sel:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    print(f"window {1e-3 * (t1 - t0):.1f} us, kernels {len(sel)}, busy {100.0 * busy / (t1 - t0):.1f}%")
    dur = defaultdict(list)
    for s, e, k, _ in sel:
        dur[k].append(e - s)
    nscan = len(dur.get("k_replay", [1]))
    for k, v in sorted(dur.items(), key=lambda kv: -sum(kv[1])):
        print(f"  {k[-40:]:40s} n={len(v):5d} avg={1e-3 * sum(v) / len(v):8.2f} us  total/scan={1e-3 * sum(v) / max(1, nscan):8.2f} us")
    print(f"scans in window ~{nscan}, window/scan {1e-3 * (t1 - t0) / max(1, nscan):.2f} us")


if __name__ == "__main__":
    main(sys.argv[1])


def per_queue(path, skip_frac=0.3, take_frac=0.4):
    """Per hardware queue: kernels, busy fraction and mean gap between
    consecutive kernels (in-order queue: gaps are host/launch time)."""
    rows = load(path)
    ks = [r for r in rows if r[2].startswith("k_")]
    n = len(ks)
    sel = ks[int(n * skip_frac): int(n * (skip_frac + take_frac))]
    t0, t1 = sel[0][0], max(r[1] for r in sel)
    q = defaultdict(list)
    for r in sel:
        q[r[3]].append(r)
    for qid, rs in sorted(q.items()):
        rs.sort()
        busy = sum(e - s for s, e, _, _ in rs)
        gaps = [rs[i + 1][0] - rs[i][1] for i in range(len(rs) - 1)]
        big = [g for g in gaps if g > 20000]
        print(f"queue {qid}: kernels {len(rs)} busy {100.0 * busy / (t1 - t0):.1f}% "
              f"mean gap {1e-3 * sum(gaps) / max(1, len(gaps)):.2f} us, gaps>20us {len(big)} "
              f"(mean {1e-3 * sum(big) / max(1, len(big)):.1f} us)")
