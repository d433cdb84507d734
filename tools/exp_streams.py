#!/usr/bin/env python3
"""Experiment: aggregate config-2 scans/s with S contexts (HIP streams) driven
from S host threads (ctypes releases the GIL during each C-ABI call)."""
import os, sys, threading, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "my-lidar-graph-slam_amd")); sys.path.insert(0, ROOT)
from lgs_amd import abi, scene
import bench

world = scene.make_world(); ang = scene.beam_angles(1081)
cells, mx, my = bench.bench_map(world, ang)
rng = np.random.default_rng(1000)
scans, inits, _ = bench.random_scans(world, ang, rng, 128)
P, cost = abi.RtcsmParams(*bench.PARAMS), abi.CostGEParams(*bench.COST)
for S in [1, 2, 3, 4, 6, 8]:
    ctxs = [abi.Context(0) for _ in range(S)]
    grids = [c.grid_from_array(cells, mx, my, 0.05) for c in ctxs]
    ds = [[c.scan(r, ang) for r in scans] for c in ctxs]
    n_per = 120
    def work(i):
        c, g = ctxs[i], grids[i]
        for k in range(n_per):
            c.optimize_pose_query(g, P, cost, ds[i][(k * S + i) % len(scans)], inits[(k * S + i) % len(scans)])
    for i in range(S):  # warm
        ctxs[i].optimize_pose_query(grids[i], P, cost, ds[i][0], inits[0])
    th = [threading.Thread(target=work, args=(i,)) for i in range(S)]
    t0 = time.perf_counter()
    for t in th: t.start()
    for t in th: t.join()
    el = time.perf_counter() - t0
    print(f"streams {S}: {S * n_per / el:.0f} scans/s  ({1e3 * el / n_per:.3f} ms per scan per stream)", flush=True)
    for c in ctxs: c.close()
