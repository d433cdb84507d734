"""Diagnostic: query path vs supplied-coarse path with fp16 superblock planes
(coarse_blocks and results), each path run twice."""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "my-lidar-graph-slam_amd"))
import numpy as np
from lgs_amd import abi, scene
from conftest import launcher_cost
from test_gpu_rtcsm import build_map
ctx = abi.Context(0)
world = scene.make_world()
for low_res, n_cells in [(5, 400), (4, 400)]:
    cells, mx, my = build_map(world, n_cells, 0.05, 100, scene.arc_poses(5), n_beams=541)
    rng = np.random.default_rng(low_res)
    ang = scene.beam_angles(541)
    qs = []
    for _ in range(4):
        true = (rng.uniform(-1, 1), rng.uniform(-1, 1), rng.uniform(-np.pi, np.pi))
        r = scene.ray_cast(world, true, ang)
        qs.append((r, (true[0] + rng.uniform(-.3, .3), true[1] + rng.uniform(-.3, .3), true[2] + rng.uniform(-.2, .2))))
    P, cost = abi.RtcsmParams(low_res, 1.0, 1.0, 0.5, 20.0), launcher_cost()
    g = ctx.grid_from_array(cells, mx, my, 0.05)
    cg = ctx.precompute_max(g, low_res)
    for j, (r, init) in enumerate(qs):
        sc = ctx.scan(r, ang)
        a = [ctx.optimize_pose_query(g, P, cost, sc, init) for _ in range(2)]
        b = [ctx.optimize_pose(g, cg, P, cost, sc, init, 2.2250738585072014e-308) for _ in range(2)]
        print(low_res, j, [x.coarse_blocks for x in a], [x.coarse_blocks for x in b],
              [list(x.best_win) for x in a + b] , [x.score_max for x in a + b], flush=True)
