#!/usr/bin/env python3
"""Per-kernel mean of every counter found in rocprofv3 --pmc csv passes.

    python tools/pmc_table.py <pass_dir> [<pass_dir> ...]"""
import sys
from collections import defaultdict

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from pmc_summary import counters  # noqa: E402

agg = defaultdict(dict)
for d in sys.argv[1:]:
    for k, cs in counters(d).items():
        for c, v in cs.items():
            agg[k][c] = sum(v) / len(v)
cols = sorted({c for v in agg.values() for c in v})
print("kernel," + ",".join(cols))
for k, v in sorted(agg.items()):
    print(k + "," + ",".join(f"{v.get(c, float('nan')):.4g}" for c in cols))
