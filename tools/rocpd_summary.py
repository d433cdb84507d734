#!/usr/bin/env python3
"""Summarise a rocprofv3 rocpd database (kernel trace) into a per-kernel stats
table: calls, total/avg/min/max duration (us), share.  Usage:
    python tools/rocpd_summary.py <results.db> [out.md]"""
import re
import sqlite3
import sys


def short(name: str) -> str:
    if name.startswith("void "):
        name = name[len("void "):]
    if name.startswith("(anonymous namespace)::"):
        name = name[len("(anonymous namespace)::"):]
    if "rocprim" in name:
        m = re.search(r"detail::(\w+?_kernel|trampoline_kernel<rocprim::\S+?::detail::wrapped_(\w+)_config)", name)
        return "rocprim::" + (m.group(2) or m.group(1) if m else "kernel")
    return name.split("(")[0]


def main():
    db, out = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else None)
    c = sqlite3.connect(db)
    rows = c.execute("select name, count(*), sum(duration), avg(duration), min(duration), max(duration) "
                     "from kernels group by name order by sum(duration) desc").fetchall()
    total = sum(r[2] for r in rows)
    lines = ["| kernel | calls | total_us | avg_us | min_us | max_us | % |", "|---|---|---|---|---|---|---|"]
    for name, n, tot, avg, mn, mx in rows:
        lines.append(f"| {short(name)} | {n} | {tot/1e3:.1f} | {avg/1e3:.3f} | {mn/1e3:.3f} | {mx/1e3:.3f} | "
                     f"{100*tot/total:.1f} |")
    text = "\n".join(lines)
    print(text)
    if out:
        open(out, "w").write(text + "\n")


if __name__ == "__main__":
    main()
