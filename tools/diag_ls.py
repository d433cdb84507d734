#!/usr/bin/env python3
"""K4 diagnostic: device Gauss-Newton refine vs the oracle on config-3 style
inputs (1081 beams, 50 iterations, 1000x1000 @ 5 cm).  Prints per-seed pose /
cost / covariance deviations and timings.  Run on the GPU box."""
import ctypes as C
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "my-lidar-graph-slam_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from lgs_amd import abi, scene  # noqa: E402
import oracle_bind as ob  # noqa: E402

LP = (50, 0.0, 0.01, 20.0, 1e-3, 1e-3, 0.01, 20.0)


def main():
    nseed = int(sys.argv[1]) if len(sys.argv) > 1 else 12
    world = scene.make_world()
    ang = scene.beam_angles(1081)
    w, h, mx, my = scene.map_geometry(1000, 100, 0.05)
    cells = scene.approx_occupancy_map(world, scene.arc_poses(10), ang, w, h, mx, my, 0.05)
    ctx = abi.Context(0)
    g = ctx.grid_from_array(cells, mx, my, 0.05)
    og = ob.OGrid(cells, mx, my, 0.05)
    rng = np.random.default_rng(11)
    # single-pose cost parity
    cd = []
    for _ in range(40):
        p = (rng.uniform(-1, 1), rng.uniform(-1, 1), rng.uniform(-3, 3))
        r = scene.ray_cast(world, p, ang)
        dc = ctx.cost_square_error(g, 0.01, 20.0, ctx.scan(r, ang), p)
        oc = ob.lib().orc_sq_cost(C.byref(og.g), 0.01, 20.0, C.byref(ob.OScan(r, ang).s), ob.Pose(*p))
        cd.append(abs(dc - oc) / max(1e-300, abs(oc)))
    cd = np.array(cd)
    print(f"sq_cost rel diff: max {cd.max():.3e} median {np.median(cd):.3e} exact {np.sum(cd == 0)}/{len(cd)}")
    lp = abi.LinsolveParams(*LP)
    olp = ob.LinsolveParams(*LP)
    worst = 0.0
    tg, tc = [], []
    for s in range(nseed):
        true = (rng.uniform(-1.2, 1.2), rng.uniform(-1.2, 1.2), rng.uniform(-3, 3))
        r = scene.ray_cast(world, true, ang)
        init = (true[0] + rng.uniform(-0.05, 0.05), true[1] + rng.uniform(-0.05, 0.05),
                true[2] + rng.uniform(-0.03, 0.03))
        sc = ctx.scan(r, ang)
        t0 = time.perf_counter()
        d = ctx.linsolve(g, lp, sc, init)
        tg.append(time.perf_counter() - t0)
        out = ob.Summary()
        t0 = time.perf_counter()
        ob.lib().orc_linsolve_optimize_pose(C.byref(og.g), C.byref(olp), C.byref(ob.OScan(r, ang).s),
                                            ob.Pose(*init), C.byref(out), None)
        tc.append(time.perf_counter() - t0)
        de, oe = d.estimated_pose, out.estimated_pose
        dp = max(abs(de.x - oe.x), abs(de.y - oe.y), abs(de.theta - oe.theta))
        dcst = abs(d.normalized_cost - out.normalized_cost) / abs(out.normalized_cost)
        dcov = max(abs(d.covariance[i] - out.covariance[i]) / max(1e-12, abs(out.covariance[i])) for i in range(9))
        worst = max(worst, dp)
        print(f"seed {s}: dpose {dp:.3e} dcost_rel {dcst:.3e} dcov_rel {dcov:.3e} it {d.iterations}/{out.best_win[0]}"
              f" err_vs_truth {max(abs(oe.x-true[0]), abs(oe.y-true[1])):.4f}")
    print(f"worst dpose {worst:.3e}; gpu {1e3*np.median(tg):.3f} ms/solve, oracle {1e3*np.median(tc):.1f} ms/solve")
    # batch throughput
    scans, inits = [], []
    for s in range(64):
        true = (rng.uniform(-1.2, 1.2), rng.uniform(-1.2, 1.2), rng.uniform(-3, 3))
        scans.append(ctx.scan(scene.ray_cast(world, true, ang), ang))
        inits.append((true[0] + 0.03, true[1] - 0.02, true[2] + 0.01))
    ctx.linsolve_batch(g, lp, scans, inits)
    t0 = time.perf_counter()
    ctx.linsolve_batch(g, lp, scans, inits)
    print(f"batch of 64: {1e3*(time.perf_counter()-t0):.3f} ms")


if __name__ == "__main__":
    main()


def per_step():
    """Device trajectory step k vs oracle OptimizeStep from the device's pose k-1."""
    world = scene.make_world()
    ang = scene.beam_angles(1081)
    w, h, mx, my = scene.map_geometry(1000, 100, 0.05)
    cells = scene.approx_occupancy_map(world, scene.arc_poses(10), ang, w, h, mx, my, 0.05)
    ctx = abi.Context(0)
    g = ctx.grid_from_array(cells, mx, my, 0.05)
    og = ob.OGrid(cells, mx, my, 0.05)
    olp = ob.LinsolveParams(*LP)
    rng = np.random.default_rng(5)
    for s in range(4):
        true = (rng.uniform(-1.2, 1.2), rng.uniform(-1.2, 1.2), rng.uniform(-3, 3))
        r = scene.ray_cast(world, true, ang)
        init = (true[0] + 0.03, true[1] - 0.02, true[2] + 0.01)
        d, traj = ctx.linsolve(g, abi.LinsolveParams(*LP), ctx.scan(r, ang), init, trajectory=True)
        osc = ob.OScan(r, ang)
        prev = init
        devs = []
        for k, t in enumerate(traj):
            o = ob.lib().orc_linsolve_step(C.byref(og.g), C.byref(olp), C.byref(osc.s), ob.Pose(*prev))
            devs.append(max(abs(o.x - t[0]), abs(o.y - t[1]), abs(o.theta - t[2])))
            prev = t
        devs = np.array(devs)
        print(f"per-step seed {s}: max {devs.max():.3e} median {np.median(devs):.3e} n>1e-12 {np.sum(devs > 1e-12)}")


if __name__ == "__main__" and os.environ.get("PER_STEP"):
    per_step()
