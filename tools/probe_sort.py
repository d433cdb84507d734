#!/usr/bin/env python3
"""Phase timings of the K3 sort on ray-like keys (probe build: make -C
my-lidar-graph-slam_amd/csrc probe; run with
LGS_LIB=my-lidar-graph-slam_amd/lgs_amd/liblgs_hip_probe.so).  Block 0
prints its per-phase wall-clock deltas (us)."""
import sys

import numpy as np

sys.path.insert(0, "my-lidar-graph-slam_amd")
from lgs_amd import abi  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 160_000
    bits = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    rng = np.random.default_rng(1)
    keys = (rng.integers(0, 1 << bits, n, dtype=np.int64) << 5 | rng.integers(0, 32, n)).astype(np.uint32)
    keys = np.sort(keys.reshape(-1, 100), axis=1).ravel()   # runs of nearby cells, as rays emit them
    ctx = abi.Context(0)
    for _ in range(6):
        got = ctx.debug_keysort(keys, 5, bits)
    f = (keys >> np.uint32(5)) & np.uint32((1 << bits) - 1)
    assert np.array_equal(got, keys[np.argsort(f, kind="stable")])
    print("ok", n, bits, flush=True)


if __name__ == "__main__":
    main()
