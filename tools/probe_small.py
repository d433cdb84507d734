"""Lone JSON-window matches (k_match_small) on the config-2 bench map through
abi.Context (LGS_LIB selects the library: an LGS_PROBE build prints the
kernel's phase times from workgroup 0)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "my-lidar-graph-slam_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from lgs_amd import abi, scene  # noqa: E402
import bench  # noqa: E402

world = scene.make_world()
ang = np.ascontiguousarray(scene.beam_angles(1081))
cells, mx, my = bench.bench_map(world, ang)
ctx = abi.Context(0)
g = ctx.grid_from_array(cells, mx, my, 0.05)
P = abi.RtcsmParams(5, 0.2, 0.2, 0.5, 20.0)
cost = abi.CostGEParams(*bench.COST)
rng = np.random.default_rng(1)
for k in range(int(sys.argv[1]) if len(sys.argv) > 1 else 20):
    t = (rng.uniform(-2, 2), rng.uniform(-2, 2), rng.uniform(-3, 3))
    sc = ctx.scan(scene.ray_cast(world, t, ang), ang)
    out = ctx.optimize_pose_query(g, P, cost, sc, (t[0] + 0.03, t[1] - 0.02, t[2] + 0.05))
    print(k, out.pose_found, list(out.best_win), out.score_max, flush=True)
ctx.close()
