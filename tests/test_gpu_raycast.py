"""GPU parity tests for K3: Bresenham ray-cast + ordered binary-Bayes update,
with the reference's GridMap geometry (Expand/Resize, patch quirks).

Bar (north_star): cell indices and hit/miss counts bit-exact; cell values are
bit-exact too (same IEEE operations in the reference's update order)."""
import numpy as np
import pytest

import oracle_bind as ob
from lgs_amd import abi, scene

pytestmark = pytest.mark.gpu
BP = (0.01, 20.0, 0.6, 0.45)


def same_map(gm, om, tag=""):
    g = gm.geometry()
    o = om.geometry()
    assert g == o, (tag, g, o)
    cells, hits, misses = gm.download()
    assert np.array_equal(hits, om.hits()), tag
    assert np.array_equal(misses, om.misses()), tag
    assert np.array_equal(cells, om.cells()), tag
    # Patch::IsAllocated (moved by Resize, kept by Reset) -> ComputeActualMapSize
    assert np.array_equal(gm.patches(), om.patches()), tag
    assert gm.actual_size() == om.actual_size(), tag


def test_fixed_map_ten_scans(ctx, world):
    """Config-2 map: 1000x1000 @ 5 cm, PatchSize 100, 10 scans on an arc."""
    ang = scene.beam_angles(1081)
    gm = ctx.map(0.05, 100, 1000, 1000)
    om = ob.OMap(0.05, 100, 1000, 1000)
    bp = abi.BuilderParams(*BP)
    obp = ob.BuilderParams(*BP)
    for p in scene.arc_poses(10):
        r = scene.ray_cast(world, p, ang)
        gm.update_scan(ctx.scan(r, ang), p, bp)
        om.integrate(p, ob.OScan(r, ang), obp)
    same_map(gm, om)


def test_local_map_growth(ctx, world):
    """A new local map (0x0 cells centred at the first pose, default PatchSize
    64) that Expand()s scan by scan (C/mapping/grid_map_builder.cpp:127-158)."""
    ang = scene.beam_angles(541)
    poses = [(x, 0.3 * np.sin(x), 0.2 * x) for x in np.linspace(-1.5, 1.5, 12)]
    gm = ctx.map(0.05, 64, 0, 0, center=poses[0][:2])
    om = ob.OMap(0.05, 64, 0, 0, center=poses[0][:2])
    bp = abi.BuilderParams(*BP)
    obp = ob.BuilderParams(*BP)
    for k, p in enumerate(poses):
        r = scene.ray_cast(world, p, ang)
        gm.update_scan(ctx.scan(r, ang), p, bp)
        om.integrate(p, ob.OScan(r, ang), obp)
        same_map(gm, om, f"scan{k}")


def test_latest_map_rebuilds(ctx, world):
    """ConstructMapFromScans over a sliding window of 10 scans, re-using one
    map object so Resize is anchored to the previous minPos (latest map)."""
    ang = scene.beam_angles(361)
    poses = [(0.1 * k, 0.05 * k, 0.03 * k) for k in range(16)]
    scans = [scene.ray_cast(world, p, ang) for p in poses]
    gm = ctx.map(0.05, 64, 0, 0)
    om = ob.OMap(0.05, 64, 0, 0)
    bp = abi.BuilderParams(*BP)
    obp = ob.BuilderParams(*BP)
    dscans = [ctx.scan(r, ang) for r in scans]
    oscans = [ob.OScan(r, ang) for r in scans]
    for k in range(len(poses)):
        lo = max(0, k - 9)
        gm.construct(dscans[lo:k + 1], poses[lo:k + 1], bp)
        om.construct(poses[lo:k + 1], oscans[lo:k + 1], obp)
        same_map(gm, om, f"frame{k}")


def test_negative_quadrant_topright_quirk(ctx):
    """All points at negative x/y: topRight starts at DBL_MIN, so the latest
    map still reaches x = y = 0."""
    ang = np.linspace(np.pi, 1.5 * np.pi, 33)
    r = np.full(33, 1.0)
    gm = ctx.map(0.05, 16, 0, 0)
    om = ob.OMap(0.05, 16, 0, 0)
    gm.construct([ctx.scan(r, ang)], [(-3.0, -3.0, 0.0)], abi.BuilderParams(*BP))
    om.construct([(-3.0, -3.0, 0.0)], [ob.OScan(r, ang)], ob.BuilderParams(*BP))
    same_map(gm, om)


def test_zero_length_and_filtered_beams(ctx):
    """Beams inside the sensor cell (zero-length rays: hit only), beams at or
    beyond the usable range limits (skipped)."""
    ang = np.linspace(-np.pi, np.pi, 64, endpoint=False)
    r = np.full(64, 2.0)
    r[::5] = 0.01       # <= usable min: skipped
    r[1::7] = 0.02      # stays in the sensor cell
    r[2::9] = 20.0      # >= usable max: skipped
    gm = ctx.map(0.05, 32, 200, 200)
    om = ob.OMap(0.05, 32, 200, 200)
    for p in [(0.0, 0.0, 0.0), (0.012, -0.013, 0.4), (0.5, 0.5, 1.0)]:
        gm.update_scan(ctx.scan(r, ang), p, abi.BuilderParams(*BP))
        om.integrate(p, ob.OScan(r, ang), ob.BuilderParams(*BP))
    same_map(gm, om)


def test_map_grid_feeds_matcher(ctx, world):
    """The device map is directly usable by the correlative matcher."""
    import ctypes as C
    from conftest import launcher_cost
    ang = scene.beam_angles(361)
    gm = ctx.map(0.05, 100, 400, 400)
    om = ob.OMap(0.05, 100, 400, 400)
    for p in scene.arc_poses(4):
        r = scene.ray_cast(world, p, ang)
        gm.update_scan(ctx.scan(r, ang), p, abi.BuilderParams(*BP))
        om.integrate(p, ob.OScan(r, ang), ob.BuilderParams(*BP))
    r = scene.ray_cast(world, (0.3, 0.2, 0.1), ang)
    params = (5, 0.6, 0.6, 0.3, 20.0)
    gpu = ctx.optimize_pose_query(gm.grid(), abi.RtcsmParams(*params), launcher_cost(), ctx.scan(r, ang),
                                  (0.33, 0.18, 0.12))
    og = ob.OGrid(om.cells(), om.m.min_x, om.m.min_y, 0.05)
    out = ob.Summary()
    ob.lib().orc_rtcsm_optimize_pose_query(C.byref(og.g), C.byref(ob.RtcsmParams(*params)),
                                           C.byref(launcher_cost(oracle=True)), C.byref(ob.OScan(r, ang).s),
                                           ob.Pose(0.33, 0.18, 0.12), C.byref(out))
    assert list(gpu.best_win) == list(out.best_win) and gpu.score_max == out.score_max
