"""Diagnostics: end-to-end deviation of config-3 refines (device vs the
oracle's own 50-iteration loop) over many seeds."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "my-lidar-graph-slam_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import oracle_bind as ob  # noqa: E402
from lgs_amd import abi, scene  # noqa: E402

CONFIG3 = (50, 0.0, 0.01, 20.0, 1e-3, 1e-3, 0.01, 20.0)
ctx = abi.Context(0)
world = scene.make_world()
ang = scene.beam_angles(1081)
w, h, mx, my = scene.map_geometry(1000, 100, 0.05)
cells = scene.approx_occupancy_map(world, scene.arc_poses(10), ang, w, h, mx, my, 0.05)
g = ctx.grid_from_array(cells, mx, my, 0.05)
og = ob.OGrid(cells, mx, my, 0.05)
split = int(sys.argv[1]) if len(sys.argv) > 1 else 1
ctx.set_option(abi.LGS_OPT_LINSOLVE_SPLIT, split)
devs = []
for seed in range(int(os.environ.get("SEEDS", 24))):
    rng = np.random.default_rng(300 + seed)
    true = (rng.uniform(-1.2, 1.2), rng.uniform(-1.2, 1.2), rng.uniform(-3, 3))
    r = scene.ray_cast(world, true, ang)
    init = (true[0] + rng.uniform(-0.05, 0.05), true[1] + rng.uniform(-0.05, 0.05), true[2] + rng.uniform(-0.03, 0.03))
    d = ctx.linsolve(g, abi.LinsolveParams(*CONFIG3), ctx.scan(r, ang), init)
    o = ob.Summary()
    traj = (ob.Pose * 50)()
    ob.lib().orc_linsolve_optimize_pose(C.byref(og.g), C.byref(ob.LinsolveParams(*CONFIG3)),
                                        C.byref(ob.OScan(r, ang).s), ob.Pose(*init), C.byref(o), traj)
    de, oe = d.estimated_pose, o.estimated_pose
    dev = max(abs(de.x - oe.x), abs(de.y - oe.y), abs(de.theta - oe.theta))
    devs.append(dev)
    print(f"seed {seed}: dev {dev:.3e} iters {d.iterations}/{o.best_win[0]} cost {d.normalized_cost:.9f} "
          f"{o.normalized_cost:.9f}", flush=True)
devs = np.array(devs)
print(f"split={split}: max {devs.max():.3e} median {np.median(devs):.3e} frac<=1e-5 {np.mean(devs <= 1e-5):.2f}")
