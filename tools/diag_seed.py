"""Diagnostics (GPU): how much of the config-2 coarse work the seed leaves.
For one 64-query batch of the bench workload: the seed's lower bound L (max of
k_seed_super's candidates), the final score, the superblocks kept with L (bound
>= L) and with the final score as L (the best any seed could do), and the
coarse blocks actually scored."""
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
rng = np.random.default_rng(1000)
scans, inits, _ = bench.random_scans(world, ang, rng, 64)
g = ctx.grid_from_array(cells, mx, my, 0.05)
ds = [ctx.scan(r, ang) for r in scans]
P, cost = abi.RtcsmParams(*bench.PARAMS), abi.CostGEParams(*bench.COST)
outs = ctx.optimize_pose_query_batch(g, P, cost, ds, inits)
rows = []
for j, o in enumerate(outs):
    sb = ctx.debug_buffer("sbound", j)
    Lb = ctx.debug_buffer("L", j)
    L = float(np.max(Lb[8:12]))
    Lbest_b = int(np.argmax(Lb[8:12]))   # which of the 4 fine-scored members gave L (wide seed: by coarse rank)
    best = o.score_max
    thr = o.score_threshold
    keep_L = int(np.sum((sb > thr) & (sb >= L)))
    keep_best = int(np.sum((sb > thr) & (sb >= best)))
    # the best pose's superblock and its rank among all superblocks by bound
    wx, wy, wt = o.win[0], o.win[1], o.win[2]
    lr = bench.PARAMS[0]
    ncx, ncy = 2 * wx // lr + 1, 2 * wy // lr + 1
    nsbx, nsby = (ncx + 3) // 4, (ncy + 3) // 4
    jx, jy, tt = (o.best_win[0] + wx) // lr, (o.best_win[1] + wy) // lr, o.best_win[2] + wt
    k = tt * nsbx * nsby + (jy // 4) * nsbx + (jx // 4)
    rank = int(np.sum(sb > sb[k]))
    # the best per-angle superblock ranks (the seed's candidate pool: k_super's per-angle bests)
    per_angle = sb.reshape(-1, nsbx * nsby).max(axis=1)
    arank = int(np.sum(per_angle > per_angle[tt]))
    # the best block's coarse-score rank among its superblock's members
    cs = ctx.debug_buffer("cscore", j)
    P_ = ncx * ncy
    mem = []
    for b_ in range(4):
        for a_ in range(4):
            mx_, my_ = 4 * (jx // 4) + a_, 4 * (jy // 4) + b_
            if mx_ < ncx and my_ < ncy:
                mem.append(cs[tt * P_ + mx_ * ncy + my_])
    cbest = cs[tt * P_ + jx * ncy + jy]
    mrank = int(np.sum(np.array(mem) > cbest))
    rows.append(dict(Lbest_b=Lbest_b, member_rank=mrank, L=L, best=best, thr=thr, superblocks=int(sb.size), kept_L=keep_L, kept_best=keep_best,
                     coarse_blocks=int(o.coarse_blocks), fine_blocks=int(o.fine_blocks), best_sb_rank=rank,
                     best_angle_rank=arank, best_is_angle_max=int(sb[k] >= per_angle[tt])))
a = {k: float(np.mean([r[k] for r in rows])) for k in rows[0]}
a["L_equals_best"] = int(sum(r["L"] >= r["best"] for r in rows))
for n in range(4):
    a[f"L_from_b{n}"] = int(sum(r["Lbest_b"] == n for r in rows))
for n in (1, 2, 3, 4, 6, 8):
    a[f"member_in_top{n}"] = int(sum(r["member_rank"] < n for r in rows))
for n in (4, 8, 16, 32, 64):
    a[f"best_sb_in_top{n}"] = int(sum(r["best_sb_rank"] < n for r in rows))
    a[f"best_angle_in_top{n}"] = int(sum(r["best_angle_rank"] < n for r in rows))
print(json.dumps(a, indent=1))
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
with open(os.path.join(ROOT, "gpurun_out", "diag_seed.json"), "w") as f:
    json.dump(dict(mean=a, items=rows), f, indent=1)
