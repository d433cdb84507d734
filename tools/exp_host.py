#!/usr/bin/env python3
"""Experiment: host-path ceiling.  A tiny match (40x40 map, 16 beams, 3x3x3
window) costs almost no GPU time, so calls/s here is the host + launch path
of optimize_pose_query: 1 thread vs S threads (one context each)."""
import os, sys, threading, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "my-lidar-graph-slam_amd"))
from lgs_amd import abi, scene
if os.environ.get("EXP_SEGV"):
    import ctypes
    ctypes.CDLL(os.path.join(ROOT, "tools", "exp", "libsegv.so"))

cells = np.random.default_rng(0).uniform(0, 1, (40, 40))
ang = scene.beam_angles(16)
r = np.full(16, 0.5)
P = abi.RtcsmParams(5, 0.1, 0.1, 0.05, 20.0)
cost = abi.CostGEParams(0.01, 20.0, 0.075, 0.1, 1, 0.05, 1.0)
for S in [int(x) for x in os.environ.get("EXP_S", "1,2,4,8,16").split(",")]:
    ctxs = [abi.Context(0) for _ in range(S)]
    grids = [c.grid_from_array(cells, -1.0, -1.0, 0.05) for c in ctxs]
    ds = [c.scan(r, ang) for c in ctxs]
    n = 2000 // S
    def work(i):
        for _ in range(n):
            ctxs[i].optimize_pose_query(grids[i], P, cost, ds[i], (0.0, 0.0, 0.0))
    for i in range(S):
        work_one = ctxs[i].optimize_pose_query(grids[i], P, cost, ds[i], (0.0, 0.0, 0.0))
    th = [threading.Thread(target=work, args=(i,)) for i in range(S)]
    t0 = time.perf_counter()
    for t in th: t.start()
    for t in th: t.join()
    el = time.perf_counter() - t0
    # pure-Python share: the same loop without the C call
    t1 = time.perf_counter()
    for _ in range(2000):
        abi.RtcsmSummary()
    py = time.perf_counter() - t1
    print(f"threads {S}: {S * n / el:.0f} calls/s ({1e6 * el / n:.1f} us per call per thread); "
          f"summary alloc {1e6 * py / 2000:.2f} us", flush=True)
    for c in ctxs:
        c.close()
