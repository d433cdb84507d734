"""Config-4 step anatomy from a rocprofv3 kernel trace (csv): per kernel name,
its mean duration and the mean idle gap before it (the end of the previous
kernel to its start: host time on the dependency chain), over the middle of
the run.  Usage: stream_gaps.py run_kernel_trace.csv [skip_frac take_frac]"""
import sys
from collections import defaultdict

from timeline import load


def main(path, skip_frac=0.3, take_frac=0.4):
    rows = [r for r in load(path) if r[2].startswith("k_")]
    n = len(rows)
    sel = rows[int(n * skip_frac): int(n * (skip_frac + take_frac))]
    t0, t1 = sel[0][0], max(r[1] for r in sel)
    dur, gap = defaultdict(list), defaultdict(list)
    for i, (s, e, k, _) in enumerate(sel):
        dur[k].append(e - s)
        if i:
            gap[k].append(max(0, s - max(r[1] for r in sel[max(0, i - 4): i])))
    steps = max(1, len(dur.get("k_cost<1>", dur.get("k_cost", [1]))))
    busy = sum(sum(v) for v in dur.values())
    print(f"window {1e-3 * (t1 - t0):.0f} us, steps ~{steps}, step {1e-3 * (t1 - t0) / steps:.1f} us, "
          f"kernel time/step {1e-3 * busy / steps:.1f} us, idle/step {1e-3 * (t1 - t0 - busy) / steps:.1f} us")
    print(f"{'kernel':44s} {'n/step':>7s} {'dur us':>8s} {'gap us':>8s} {'dur/step':>9s} {'gap/step':>9s}")
    for k, v in sorted(dur.items(), key=lambda kv: -sum(kv[1])):
        g = gap.get(k, [0])
        print(f"{k[-44:]:44s} {len(v) / steps:7.2f} {1e-3 * sum(v) / len(v):8.2f} {1e-3 * sum(g) / len(g):8.2f} "
              f"{1e-3 * sum(v) / steps:9.2f} {1e-3 * sum(g) / steps:9.2f}")


if __name__ == "__main__":
    main(sys.argv[1], *(float(a) for a in sys.argv[2:4]))
