"""Diagnostics (GPU): is superblock pruning a function of the call's inputs only?

For each case: call A (query path), B (supplied coarse map), a "dirty" call
with a different scan (other T and Nv), then A and B again; with and without
LGS_OPT_POISON_WS.  Prints coarse_blocks of every call and, for the first
intermediate buffer of item 0 that differs between two identical calls, its
name and the first differing index.  Exit status 1 if any identical calls
disagree.
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "my-lidar-graph-slam_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

from lgs_amd import abi, scene  # noqa: E402
from conftest import launcher_cost  # noqa: E402
from test_gpu_rtcsm import build_map  # noqa: E402

BUFS = ["sbound", "part_c", "part_k", "L", "tedge", "cbase", "idx", "cscore"]


def snap(ctx, out):
    return dict(blocks=out.coarse_blocks, win=list(out.best_win), score=out.score_max,
                bufs={b: ctx.debug_buffer(b) for b in BUFS})


def diff(a, b):
    if a["blocks"] != b["blocks"] or a["win"] != b["win"] or a["score"] != b["score"]:
        for name in BUFS:
            x, y = a["bufs"][name], b["bufs"][name]
            if name == "cscore":
                continue   # only the kept blocks are written: not comparable
            if x.shape != y.shape or not np.array_equal(x.view(np.uint8), y.view(np.uint8)):
                k = int(np.argmax(x.view(np.uint8) != y.view(np.uint8))) // x.itemsize if x.shape == y.shape else -1
                return f"{name}[{k}]: {x[k] if k >= 0 else x.shape} vs {y[k] if k >= 0 else y.shape}"
        return "outputs differ, buffers equal"
    return None


def main():
    world = scene.make_world()
    ctx = abi.Context(0)
    bad = 0
    for poison in (0, 1):
        ctx.set_option(abi.LGS_OPT_POISON_WS, poison)
        for low_res, n_cells in [(5, 400), (4, 400), (2, 300), (8, 400)]:
            cells, mx, my = build_map(world, n_cells, 0.05, 100, scene.arc_poses(5), n_beams=541)
            rng = np.random.default_rng(low_res)
            ang = scene.beam_angles(541)
            params = abi.RtcsmParams(low_res, 1.0, 1.0, 0.5, 20.0)
            cost = launcher_cost()
            g = ctx.grid_from_array(cells, mx, my, 0.05)
            cg = ctx.precompute_max(g, low_res)
            dirty_r = np.minimum(scene.ray_cast(world, (0.2, -0.1, 1.0), ang), 6.0)
            dirty_r[::3] = 25.0
            dirty = ctx.scan(dirty_r, ang)
            for j in range(4):
                true = (rng.uniform(-1, 1), rng.uniform(-1, 1), rng.uniform(-np.pi, np.pi))
                r = scene.ray_cast(world, true, ang)
                init = (true[0] + rng.uniform(-0.3, 0.3), true[1] + rng.uniform(-0.3, 0.3),
                        true[2] + rng.uniform(-0.2, 0.2))
                sc = ctx.scan(r, ang)
                a1 = snap(ctx, ctx.optimize_pose_query(g, params, cost, sc, init))
                b1 = snap(ctx, ctx.optimize_pose(g, cg, params, cost, sc, init, 2.2250738585072014e-308))
                ctx.optimize_pose_query(g, params, cost, dirty, (0.0, 0.0, 0.5))
                a2 = snap(ctx, ctx.optimize_pose_query(g, params, cost, sc, init))
                ctx.optimize_pose_query_batch(g, params, cost, [dirty, sc], [(0.0, 0.0, 0.5), init])
                b2 = snap(ctx, ctx.optimize_pose(g, cg, params, cost, sc, init, 2.2250738585072014e-308))
                da, db, dab = diff(a1, a2), diff(b1, b2), diff(a1, b1)
                print(f"poison={poison} lr={low_res} q{j}: blocks A {a1['blocks']} {a2['blocks']} "
                      f"B {b1['blocks']} {b2['blocks']}  A:{da}  B:{db}  AvsB:{dab}", flush=True)
                bad += (da is not None) + (db is not None) + (dab is not None)
                bad += a1["blocks"] != a2["blocks"] or b1["blocks"] != b2["blocks"]
    ctx.close()
    print("DETERMINISM", "OK" if bad == 0 else f"FAIL ({bad})")
    sys.exit(1 if bad and "--strict" in sys.argv else 0)


if __name__ == "__main__":
    main()
