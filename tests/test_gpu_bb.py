"""GPU parity tests for the branch-and-bound matcher:
lgs_grid_precompute_pyramid, lgs_bb_optimize_pose_query / _batch,
lgs_loop_detect_bb, against the oracle's restatement of
ScanMatcherBranchBound / ScorePixelAccurate / PrecomputeGridMaps.

Bar: pyramid bit-exact; best node (x, y, theta), best score and found flag
bit-exact; the number of nodes the reference's LIFO search visits equal
(the host replay walks the same search); cost and covariance within 1e-5.
"""
import ctypes as C

import numpy as np
import pytest

import oracle_bind as ob
from conftest import launcher_cost
from lgs_amd import abi, scene
from test_gpu_rtcsm import build_map

pytestmark = pytest.mark.gpu
DBL_MIN = 2.2250738585072014e-308
TOL = 1e-5


def oracle_bb(cells, mx, my, res, prm, ranges, angles, init, thr=None):
    g = ob.OGrid(cells, mx, my, res)
    sc = ob.OScan(ranges, angles, (0, 0, 0), 0.0, 30.0)
    P = ob.BBParams(*prm)
    out = ob.Summary()
    cost = launcher_cost(oracle=True)
    if thr is None:
        ob.lib().orc_bb_optimize_pose_query(C.byref(g.g), C.byref(P), C.byref(cost), C.byref(sc.s), ob.Pose(*init),
                                            C.byref(out))
    else:
        keep = [ob.OGrid(m, mx, my, res) for m in ob.precompute_pyramid(cells, prm[0])]
        maps = (ob.Grid * len(keep))(*[k.g for k in keep])
        ob.lib().orc_bb_optimize_pose(C.byref(g.g), maps, C.byref(P), C.byref(cost), C.byref(sc.s), ob.Pose(*init),
                                      thr, C.byref(out))
    return out


def assert_bb_same(gpu, ora, tag=""):
    assert gpu.pose_found == ora.pose_found, tag
    assert list(gpu.win) == list(ora.win), tag
    assert list(gpu.best_win) == list(ora.best_win), (tag, list(gpu.best_win), list(ora.best_win))
    assert gpu.score_max == ora.score_max, (tag, gpu.score_max, ora.score_max)
    assert gpu.fine_blocks == ora.coarse_evals, (tag, gpu.fine_blocks, ora.coarse_evals)   # nodes visited
    assert gpu.coarse_blocks >= gpu.fine_blocks
    assert gpu.estimated_pose.tuple() == (ora.estimated_pose.x, ora.estimated_pose.y, ora.estimated_pose.theta)
    assert abs(gpu.normalized_cost - ora.normalized_cost) <= TOL, tag
    assert np.allclose(list(gpu.covariance), list(ora.covariance), rtol=0, atol=TOL), tag


def test_pyramid_parity(ctx):
    rng = np.random.default_rng(4)
    cells = rng.choice([0.0, 0.0, 0.45, 0.6, 0.9], size=(90, 130)) * rng.uniform(0.5, 1.0, size=(90, 130))
    g = ctx.grid_from_array(cells, -2.0, -3.0, 0.05)
    pyr = ctx.precompute_pyramid(g, 6)
    for h, (d, o) in enumerate(zip(pyr, ob.precompute_pyramid(cells, 6))):
        assert np.array_equal(d.download(), o), h


@pytest.fixture(scope="module")
def small_map(world):
    return build_map(world, 300, 0.05, 100, scene.arc_poses(4), n_beams=361)


@pytest.mark.parametrize("seed", range(4))
def test_bb_query_dbl_min(ctx, world, small_map, seed):
    """OptimizePose(query): threshold DBL_MIN, so the first descent decides the
    expansion threshold of the device superset."""
    cells, mx, my = small_map
    rng = np.random.default_rng(40 + seed)
    ang = scene.beam_angles(361)
    true = (rng.uniform(-0.8, 0.8), rng.uniform(-0.8, 0.8), rng.uniform(-np.pi, np.pi))
    r = scene.ray_cast(world, true, ang)
    init = (true[0] + rng.uniform(-0.2, 0.2), true[1] + rng.uniform(-0.2, 0.2), true[2] + rng.uniform(-0.1, 0.1))
    prm = (3, 1.0, 1.0, 0.4, 20.0, 0.01, 20.0)
    g = ctx.grid_from_array(cells, mx, my, 0.05)
    gpu = ctx.bb_optimize_pose_query(g, abi.BBParams(*prm), launcher_cost(), ctx.scan(r, ang), init)
    assert_bb_same(gpu, oracle_bb(cells, mx, my, 0.05, prm, r, ang, init), f"seed{seed}")


def test_bb_batch_loop_threshold(ctx, world):
    """LoopDetectorBranchBound settings (NodeHeightMax 6, 2.0/2.0/1.0,
    threshold 0.6) on a 600x600 local map with 1081-beam scans."""
    cells, mx, my = build_map(world, 600, 0.05, 100, scene.arc_poses(10), n_beams=1081)
    rng = np.random.default_rng(7)
    ang = scene.beam_angles(1081)
    prm = (6, 2.0, 2.0, 1.0, 20.0, 0.01, 20.0)
    g = ctx.grid_from_array(cells, mx, my, 0.05)
    pyr = ctx.precompute_pyramid(g, 6)
    scans, inits, rs = [], [], []
    for _ in range(5):
        true = (rng.uniform(-1, 1), rng.uniform(-1, 1), rng.uniform(-3, 3))
        r = scene.ray_cast(world, true, ang)
        rs.append(r)
        scans.append(ctx.scan(r, ang))
        inits.append((true[0] + rng.uniform(-0.5, 0.5), true[1] + rng.uniform(-0.5, 0.5),
                      true[2] + rng.uniform(-0.2, 0.2)))
    out = ctx.bb_optimize_pose_batch(g, pyr, abi.BBParams(*prm), launcher_cost(), scans, inits, 0.6)
    for j, o in enumerate(out):
        assert_bb_same(o, oracle_bb(cells, mx, my, 0.05, prm, rs[j], ang, inits[j], thr=0.6), f"cand{j}")


def test_bb_fixups(ctx, world, small_map):
    """Every guarded device cell corrupted (LGS_OPT_INJECT_INDEX): the host
    re-checks them with glibc, re-scores the nodes, and the result is exact."""
    cells, mx, my = small_map
    ang = scene.beam_angles(361)
    true = (0.3, -0.2, 0.7)
    r = scene.ray_cast(world, true, ang)
    init = (0.4, -0.1, 0.75)
    prm = (3, 0.8, 0.8, 0.3, 20.0, 0.01, 20.0)
    g = ctx.grid_from_array(cells, mx, my, 0.05)
    try:
        ctx.set_option(abi.LGS_OPT_GUARD_EPS, 0.01)
        ctx.set_option(abi.LGS_OPT_INJECT_INDEX, 1)
        gpu = ctx.bb_optimize_pose_query(g, abi.BBParams(*prm), launcher_cost(), ctx.scan(r, ang), init)
    finally:
        ctx.set_option(abi.LGS_OPT_INJECT_INDEX, 0)
        ctx.set_option(abi.LGS_OPT_GUARD_EPS, 1e-9)
    assert gpu.fixups == 1 and gpu.guard_hits > 0
    assert_bb_same(gpu, oracle_bb(cells, mx, my, 0.05, prm, r, ang, init), "inject")


@pytest.mark.parametrize("eps", [3e-4, 1e-2])
def test_bb_fixups_batch_small_scans(ctx, world, small_map, eps):
    """A 64-candidate batch of 17-beam scans with injected guard corruption:
    few dirty nodes make the re-score's upload (cells, pointer arrays) smaller
    than the replay's upload that follows it in the same staging buffer -- the
    replay's staging must not overwrite it before the re-score's copy read it
    (ADVICE r04)."""
    cells, mx, my = small_map
    ang = scene.beam_angles(17)
    prm = (3, 0.8, 0.8, 0.3, 20.0, 0.01, 20.0)
    g = ctx.grid_from_array(cells, mx, my, 0.05)
    pyr = ctx.precompute_pyramid(g, 3)
    rng = np.random.default_rng(99)
    scans, inits, rs = [], [], []
    for _ in range(64):
        true = (rng.uniform(-0.8, 0.8), rng.uniform(-0.8, 0.8), rng.uniform(-3, 3))
        r = scene.ray_cast(world, true, ang)
        rs.append(r)
        scans.append(ctx.scan(r, ang))
        inits.append((true[0] + rng.uniform(-0.2, 0.2), true[1] + rng.uniform(-0.2, 0.2), true[2] + 0.05))
    try:
        ctx.set_option(abi.LGS_OPT_GUARD_EPS, eps)
        ctx.set_option(abi.LGS_OPT_INJECT_INDEX, 1)
        out = ctx.bb_optimize_pose_batch(g, pyr, abi.BBParams(*prm), launcher_cost(), scans, inits, 0.3)
    finally:
        ctx.set_option(abi.LGS_OPT_INJECT_INDEX, 0)
        ctx.set_option(abi.LGS_OPT_GUARD_EPS, 1e-9)
    assert sum(o.fixups for o in out) >= 1
    for j, o in enumerate(out):
        assert_bb_same(o, oracle_bb(cells, mx, my, 0.05, prm, rs[j], ang, inits[j], thr=0.3), f"cand{j}")


def test_loop_detect_bb(ctx, world):
    """LoopDetectorBranchBound::Detect over two local maps of different size."""
    maps = [build_map(world, n, 0.05, 100, scene.arc_poses(k), n_beams=541) for n, k in ((300, 4), (400, 6))]
    ang = scene.beam_angles(541)
    prm = (4, 1.0, 1.0, 0.6, 20.0, 0.01, 20.0)
    rng = np.random.default_rng(21)
    grids = [ctx.grid_from_array(c, mx, my, 0.05) for c, mx, my in maps]
    queries, cands, ref = [], [], []
    for q, (c, mx, my) in enumerate(maps):
        first = len(cands)
        for k in range(3):
            true = (rng.uniform(-1, 1), rng.uniform(-1, 1), rng.uniform(-3, 3))
            r = scene.ray_cast(world, true, ang)
            init = (true[0] + rng.uniform(-0.3, 0.3), true[1] + rng.uniform(-0.3, 0.3), true[2] + 0.1)
            cands.append((ctx.scan(r, ang), init, 100 * q + k))
            ref.append(oracle_bb(c, mx, my, 0.05, prm, r, ang, init, thr=0.6))
        queries.append((grids[q], None, (0.1 * q, 0.0, 0.0), q, first, 3))
    res = ctx.loop_detect_bb(abi.BBParams(*prm), launcher_cost(), 0.6, queries, cands)
    for k, (rr, o) in enumerate(zip(res, ref)):
        assert rr.found == o.pose_found, k
        assert rr.end_node_index == cands[k][2]
        assert rr.score == o.score_max, k
        e = rr.estimated_pose
        assert (e.x, e.y, e.theta) == (o.estimated_pose.x, o.estimated_pose.y, o.estimated_pose.theta), k
