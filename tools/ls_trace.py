"""Phase stamps of one split refine on config 3 (LGS_LS_TRACE=1 makes the
library print 'LSTRACE pass k: axes smoothed published consumed solved | next'
in microseconds from the pass start, workgroup 0)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "my-lidar-graph-slam_amd")]
import numpy as np  # noqa: E402

from lgs_amd import abi, scene  # noqa: E402

world = scene.make_world()
ang = scene.beam_angles(1081)
w, h, mx, my = scene.map_geometry(1000, 100, 0.05)
cells = scene.approx_occupancy_map(world, scene.arc_poses(10), ang, w, h, mx, my, 0.05)
ctx = abi.Context(0)
g = ctx.grid_from_array(cells, mx, my, 0.05)
true = (0.3, -0.2, 0.5)
sc = ctx.scan(scene.ray_cast(world, true, ang), ang)
lp = abi.LinsolveParams(50, 0.0, 0.01, 20.0, 1e-3, 1e-3, 0.01, 20.0)
for _ in range(3):
    ctx.linsolve(g, lp, sc, (0.32, -0.18, 0.51))
