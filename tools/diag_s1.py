import ctypes as C, sys
import numpy as np
sys.path.insert(0, "my-lidar-graph-slam_amd"); sys.path.insert(0, "tests")
from lgs_amd import abi, scene
import oracle_bind as ob
world = scene.make_world()
ang = scene.beam_angles(361)
m = ob.OMap(0.05, 100, 600, 600)
for p in scene.arc_poses(6):
    m.integrate(p, ob.OScan(scene.ray_cast(world, p, ang), ang), ob.BuilderParams(0.01, 20.0, 0.6, 0.45))
cells, mx, my = m.cells(), m.m.min_x, m.m.min_y
ctx = abi.Context(0)
g = ctx.grid_from_array(cells, mx, my, 0.05); og = ob.OGrid(cells, mx, my, 0.05)
for seed in (1, 2):
    rng = np.random.default_rng(100 + seed)
    true = (rng.uniform(-1, 1), rng.uniform(-1, 1), rng.uniform(-3, 3))
    r = scene.ray_cast(world, true, ang)
    init = (true[0] + rng.uniform(-0.05, 0.05), true[1] + rng.uniform(-0.05, 0.05), true[2] + rng.uniform(-0.03, 0.03))
    lp = (50, 0.0, 0.01, 20.0, 1e-3, 1e-3, 0.01, 20.0) if seed % 2 == 0 else (100, 1e-3, 0.01, 20.0, 1e-3, 1e-3, 0.01, 20.0)
    d, traj = ctx.linsolve(g, abi.LinsolveParams(*lp), ctx.scan(r, ang), init, trajectory=True)
    osc = ob.OScan(r, ang); olp = ob.LinsolveParams(*lp)
    prev = (d.sensor_pose.x, d.sensor_pose.y, d.sensor_pose.theta)
    for k, t in enumerate(traj):
        o = ob.lib().orc_linsolve_step(C.byref(og.g), C.byref(olp), C.byref(osc.s), ob.Pose(*prev))
        oc = ob.lib().orc_sq_cost(C.byref(og.g), 0.01, 20.0, C.byref(osc.s), ob.Pose(*t))
        dc = ctx.cost_square_error(g, 0.01, 20.0, ctx.scan(r, ang), t)
        dev = max(abs(o.x - t[0]), abs(o.y - t[1]), abs(o.theta - t[2]))
        print(f"seed {seed} step {k+1}: stepdev {dev:.2e} ocost {oc!r} dcost {dc!r}")
        prev = t
    print("device iterations", d.iterations, "cost", d.cost)
