"""Print a few consecutive config-4 steps from a rocprofv3 kernel trace:
start (us, relative to a k_match_small), duration, the gap since the previous
kernel ended, and the kernel -- where the step's device idle time sits."""
import csv
import sys


def main(path, steps=3):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            n = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "")
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), n.split("(")[0][:40]))
    rows.sort()
    i = len(rows) // 2
    while "match_small" not in rows[i][2]:
        i += 1
    t0, prev, seen = rows[i][0], rows[i - 1][1], 0
    for s, e, n in rows[i:]:
        if "match_small" in n:
            seen += 1
            if seen > steps:
                break
        print(f"{(s - t0) / 1000:8.1f} {(e - s) / 1000:6.1f} gap {(s - prev) / 1000:6.1f}  {n}")
        prev = e


if __name__ == "__main__":
    main(sys.argv[1], *(int(a) for a in sys.argv[2:3]))
