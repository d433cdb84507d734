"""Config-5 superblock pruning statistics: for the first 64 loop candidates
(one batched launch), the number of kept superblocks of every (item, angle)
workgroup of k_coarse_lanes -- the work each workgroup does -- from the
pruning inputs (lgs_debug_item_buffer: superblock bounds, seed bound L)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "my-lidar-graph-slam_amd"), ROOT]
import numpy as np  # noqa: E402

import bench  # noqa: E402
from lgs_amd import abi, loopbatch, scene  # noqa: E402

ctx = abi.Context(0)
world = scene.make_world()
bp = abi.BuilderParams(*bench.BUILDER)


def build(poses, ang):
    m = ctx.map(0.05, 100, 600, 600)
    m.construct([ctx.scan(scene.ray_cast(world, p, ang), ang) for p in poses], poses, bp)
    cells, _, _ = m.download()
    g = m.geometry()
    return cells, g["min_x"], g["min_y"], 0.05


maps, cands = scene.loop_problem(world, build, n_maps=32, nodes_per_map=16, n_beams=1081, seed=5,
                                 perturb=(2.0, 0.4), arc_scans=10)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 64
fn = loopbatch.hip_detect_fn(ctx, maps, cands[:n], abi.RtcsmParams(*bench.LOOP_PARAMS),
                             abi.CostGEParams(*bench.COST), 0.6)
rec = loopbatch.run_sharded(cands[:n], fn)
thr = 0.6 * 1081
kept_all = []
for item in range(min(n, 64)):
    sb = ctx.debug_buffer("sbound", item)
    L = ctx.debug_buffer("L", item)
    Lc = L[8:12].max()
    T = 401
    nsb2 = len(sb) // T
    s = sb[: T * nsb2].reshape(T, nsb2)
    kept = ((s > thr) & (s >= Lc)).sum(axis=1)
    kept_all.append(kept)
k = np.array(kept_all)
print("nsb2", nsb2, "items", k.shape[0], "angles", k.shape[1])
print("kept superblocks per workgroup: mean %.2f  max %d  total %d" % (k.mean(), k.max(), k.sum()))
hist = np.bincount(k.ravel())
print("histogram (kept: workgroups):", {i: int(c) for i, c in enumerate(hist) if c})
per_item = k.sum(axis=1)
print("per item kept: min %d median %d max %d" % (per_item.min(), np.median(per_item), per_item.max()))
w = np.sort(k.ravel())[::-1]
print("top workgroups:", w[:20].tolist(), " share of work in top 1%%: %.2f" % (w[: len(w) // 100].sum() / w.sum()))
