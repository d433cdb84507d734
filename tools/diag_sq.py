#!/usr/bin/env python3
"""Find beams whose device CostSquareError term differs from the oracle's."""
import ctypes as C, math, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "my-lidar-graph-slam_amd")); sys.path.insert(0, os.path.join(ROOT, "tests"))
from lgs_amd import abi, scene
import oracle_bind as ob
world = scene.make_world()
ang = scene.beam_angles(361)
m = ob.OMap(0.05, 100, 600, 600)
for p in scene.arc_poses(6):
    m.integrate(p, ob.OScan(scene.ray_cast(world, p, ang), ang), ob.BuilderParams(0.01, 20.0, 0.6, 0.45))
cells, mx, my = m.cells(), m.m.min_x, m.m.min_y
ctx = abi.Context(0)
g = ctx.grid_from_array(cells, mx, my, 0.05)
og = ob.OGrid(cells, mx, my, 0.05)
rng = np.random.default_rng(1)
for k in range(5):
    p = (rng.uniform(-1.5, 1.5), rng.uniform(-1.5, 1.5), rng.uniform(-3, 3))
    r = scene.ray_cast(world, p, ang)
    for i in range(len(r)):
        rr, aa = r[i:i+1].copy(), ang[i:i+1].copy()
        c = ctx.cost_square_error(g, 0.01, 20.0, ctx.scan(rr, aa), p)
        oc = ob.lib().orc_sq_cost(C.byref(og.g), 0.01, 20.0, C.byref(ob.OScan(rr, aa).s), ob.Pose(*p))
        if c != oc:
            th = p[2] + aa[0]
            fx = (p[0] + rr[0] * math.cos(th) - mx) / 0.05
            fy = (p[1] + rr[0] * math.sin(th) - my) / 0.05
            print(f"pose {k} beam {i}: dev {c!r} orc {oc!r} fx {fx!r} fy {fy!r}")
