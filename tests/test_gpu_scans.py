"""Scan device copies (r03): a scan is copied to the device by the first call
that reads it, from a per-device buffer pool, and joins the match's staging
launch (csrc/lgs_core.hip scans_to_device, k_fetch).  The matcher's results
must not depend on any of that: a scan used on a context other than the one
that copied it (the device-wide wait path), scans destroyed and re-created so
that pooled buffers are handed out again with other contents and sizes, and a
batch whose new scans need several staging launches (more than 8 copies)
all match like the oracle (C/mapping/scan_matcher_real_time_correlative.cpp:31-47)."""
import numpy as np
import pytest

from conftest import launcher_cost
from lgs_amd import abi, scene
from test_gpu_rtcsm import assert_same, build_map, oracle_match

pytestmark = pytest.mark.gpu
PARAMS = (5, 0.6, 0.6, 0.3, 20.0)


def _scene(world, n):
    rng = np.random.default_rng(5)
    cells, mx, my = build_map(world, 500, 0.05, 64, [(0.0, 0.0, 0.0), (0.3, 0.2, 0.4)])
    ang = scene.beam_angles(361)
    truths = [(rng.uniform(-0.5, 0.5), rng.uniform(-0.5, 0.5), rng.uniform(-0.3, 0.3)) for _ in range(n)]
    ranges = [scene.ray_cast(world, t, ang) for t in truths]
    inits = [(t[0] + 0.07, t[1] - 0.05, t[2] + 0.04) for t in truths]
    return cells, mx, my, ang, ranges, inits


def test_scan_used_on_another_context(ctx, world):
    """A scan created (and first copied) on one context, then matched on a
    second context's grid: the second waits for the first's copy once."""
    cells, mx, my, ang, ranges, inits = _scene(world, 3)
    other = abi.Context(0)
    try:
        P, cost = abi.RtcsmParams(*PARAMS), launcher_cost()
        g_a = ctx.grid_from_array(cells, mx, my, 0.05)
        g_b = other.grid_from_array(cells, mx, my, 0.05)
        for r, init in zip(ranges, inits):
            s = ctx.scan(r, ang)
            ref = oracle_match(cells, mx, my, 0.05, PARAMS, r, ang, init)
            assert_same(ctx.optimize_pose_query(g_a, P, cost, s, init), ref, "creating context")
            assert_same(other.optimize_pose_query(g_b, P, cost, s, init), ref, "other context")
            s.close()
        # first use on the other context: the copy is made there
        s = ctx.scan(ranges[0], ang)
        assert_same(other.optimize_pose_query(g_b, P, cost, s, inits[0]),
                    oracle_match(cells, mx, my, 0.05, PARAMS, ranges[0], ang, inits[0]), "first use elsewhere")
        s.close()
    finally:
        other.close()


def test_pooled_buffers_reused(ctx, world):
    """Scans of different beam counts created and destroyed in turn, so the
    pool hands the same buffers out again: every match still equals the
    oracle's (a stale copy would change the scan's points)."""
    cells, mx, my, _, _, _ = _scene(world, 0)
    P, cost = abi.RtcsmParams(*PARAMS), launcher_cost()
    g = ctx.grid_from_array(cells, mx, my, 0.05)
    rng = np.random.default_rng(9)
    for k in range(12):
        nb = (181, 361, 541, 1081)[k % 4]
        ang = scene.beam_angles(nb)
        t = (rng.uniform(-0.4, 0.4), rng.uniform(-0.4, 0.4), rng.uniform(-0.2, 0.2))
        r = scene.ray_cast(world, t, ang)
        init = (t[0] - 0.05, t[1] + 0.06, t[2] - 0.03)
        s = ctx.scan(r, ang)
        assert_same(ctx.optimize_pose_query(g, P, cost, s, init),
                    oracle_match(cells, mx, my, 0.05, PARAMS, r, ang, init), f"cycle {k}")
        s.close()


def test_batch_of_new_scans_several_staging_launches(ctx, world):
    """20 scans never used before in one batched call: their copies join the
    batch's staging launch, 8 segments per launch (3 launches); results equal
    the lone calls' and the oracle's."""
    cells, mx, my, ang, ranges, inits = _scene(world, 20)
    P, cost = abi.RtcsmParams(*PARAMS), launcher_cost()
    g = ctx.grid_from_array(cells, mx, my, 0.05)
    scans = [ctx.scan(r, ang) for r in ranges]
    outs = ctx.optimize_pose_query_batch(g, P, cost, scans, inits)
    for k, (out, r, init) in enumerate(zip(outs, ranges, inits)):
        assert_same(out, oracle_match(cells, mx, my, 0.05, PARAMS, r, ang, init), f"batch item {k}")
    for s in scans:
        s.close()
