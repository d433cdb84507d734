#!/usr/bin/env python3
"""Run a few config-2 matches through the probe build (make -C csrc probe):
kernels print per-phase wall-clock deltas from block 0."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "my-lidar-graph-slam_amd")); sys.path.insert(0, ROOT)
from lgs_amd import abi, scene
import numpy as np
abi.load(os.path.join(ROOT, "my-lidar-graph-slam_amd", "lgs_amd", "liblgs_hip_probe.so"))
import bench
world = scene.make_world(); ang = scene.beam_angles(1081)
cells, mx, my = bench.bench_map(world, ang)
scans, inits, _ = bench.random_scans(world, ang, np.random.default_rng(1000), 8)
ctx = abi.Context(0)
g = ctx.grid_from_array(cells, mx, my, 0.05)
P, cost = abi.RtcsmParams(*bench.PARAMS), abi.CostGEParams(*bench.COST)
for k in range(int(os.environ.get("N", "3"))):
    out = ctx.optimize_pose_query(g, P, cost, ctx.scan(scans[k], ang), inits[k])
    ctx.synchronize()
    print(f"--- scan {k}: coarse_blocks {out.coarse_blocks} fine_blocks {out.fine_blocks}", flush=True)
