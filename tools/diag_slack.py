"""Diagnostics (GPU): how sensitive the superblock pruning is to a looser
bound.  For one 64-query batch of the bench workload: superblocks kept with
the shipped bound (bound > thr and bound >= L) and with every bound raised by
an absolute slack s (what a coarser superblock-plane encoding would add: an
8-bit round-up of values in [0, 1] adds up to Nv / 255 ~ 4.2 per 1081-beam
bound, about half that on average), the coarse blocks those superblocks
would make the coarse stage score, and the angles that keep anything."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "my-lidar-graph-slam_amd"))
import bench  # noqa: E402
from lgs_amd import abi, scene  # noqa: E402

ctx = abi.Context(0)
world = scene.make_world()
ang = scene.beam_angles(1081)
cells, mx, my = bench.bench_map(world, ang)
scans, inits, _ = bench.random_scans(world, ang, np.random.default_rng(1000), 64)
g = ctx.grid_from_array(cells, mx, my, 0.05)
ds = [ctx.scan(r, ang) for r in scans]
P, cost = abi.RtcsmParams(*bench.PARAMS), abi.CostGEParams(*bench.COST)
outs = ctx.optimize_pose_query_batch(g, P, cost, ds, inits)
lr = bench.PARAMS[0]
slacks = (0.0, 0.5, 1.0, 2.0, 4.0, 8.0, 16.0)
rows = []
for j, o in enumerate(outs):
    sb = ctx.debug_buffer("sbound", j)
    L = float(np.max(ctx.debug_buffer("L", j)[8:12]))
    thr = o.score_threshold
    wx, wy = o.win[0], o.win[1]
    ncx, ncy = 2 * wx // lr + 1, 2 * wy // lr + 1
    nsbx, nsby = (ncx + 3) // 4, (ncy + 3) // 4
    members = np.array([min(4, ncx - 4 * (i % nsbx)) * min(4, ncy - 4 * (i // nsbx)) for i in range(nsbx * nsby)])
    sbm = sb.reshape(-1, nsbx * nsby)
    r = dict(L=L, best=o.score_max, T=int(sbm.shape[0]), coarse_blocks=int(o.coarse_blocks))
    for s in slacks:
        kept = (sbm + s > thr) & (sbm + s >= L)
        r[f"kept_{s}"] = int(kept.sum())
        r[f"blocks_{s}"] = int((kept * members[None, :]).sum())
        r[f"angles_{s}"] = int(kept.any(axis=1).sum())
    # the bound's margin below L of the superblocks just missed (how close the field is)
    below = np.sort((L - sbm[sbm < L]).ravel())[:20]
    r["closest_below_L"] = [round(float(x), 3) for x in below[:5]]
    rows.append(r)
mean = {k: float(np.mean([r[k] for r in rows])) for k in rows[0] if k != "closest_below_L"}
print(json.dumps(mean, indent=1))
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
with open(os.path.join(ROOT, "gpurun_out", "diag_slack.json"), "w") as f:
    json.dump(dict(mean=mean, items=rows), f, indent=1)
