"""GPU-box tests for the frontend's per-scan host remainder:
ScanInterpolator::Interpolate (C/mapping/scan_interpolator.cpp:9-98) as
lgs_scan_interpolate, which writes the interpolated scan straight into a
device scan.  Bar: ranges and angles bit-exact vs the oracle (both use glibc
sincos/atan2/sqrt; the oracle is pinned by the pure-Python KAT,
tests/golden/kat.json "interp_py"), and the interpolated scan matches like the
oracle's scan in OptimizePose(query)."""
import numpy as np
import pytest

import oracle_bind as ob
from lgs_amd import abi, scene
from conftest import launcher_cost
from test_gpu_rtcsm import assert_same, build_map, oracle_match

pytestmark = pytest.mark.gpu


def _check(ctx, r, a, ds=0.05, de=0.25, rel=(0.0, 0.0, 0.0)):
    sc = ctx.scan(r, a, rel_pose=rel, min_range=0.01, max_range=25.0)
    out = ctx.interpolate(sc, ds, de)
    orr, oa = ob.scan_interpolate(r, a, ds, de)
    assert out.ranges.tolist() == orr.tolist()
    assert out.angles.tolist() == oa.tolist()
    assert out.rel_pose == rel and out.min_range == 0.01 and out.max_range == 25.0
    return out


@pytest.mark.parametrize("seed", range(4))
def test_interpolate_scene_scans(ctx, world, seed):
    """1081-beam scans of the synthetic world with the launcher's 0.05 / 0.25."""
    rng = np.random.default_rng(seed)
    ang = scene.beam_angles(1081)
    pose = (rng.uniform(-1, 1), rng.uniform(-1, 1), rng.uniform(-np.pi, np.pi))
    r = scene.ray_cast(world, pose, ang)
    out = _check(ctx, r, ang)
    assert 50 < len(out.ranges) < 3000


@pytest.mark.parametrize("ds,de", [(0.05, 0.25), (0.1, 0.3), (0.02, 0.5), (0.03, 0.06)])
def test_interpolate_parameters_and_edges(ctx, ds, de):
    rng = np.random.default_rng(7)
    a = np.linspace(-2.0, 2.0, 300)
    r = 1.0 + 0.5 * np.sin(3 * a)
    r[rng.integers(0, 300, 20)] *= 3.0          # gaps
    _check(ctx, r, a, ds, de)
    _check(ctx, np.array([1.5]), np.array([0.3]), ds, de)          # one beam
    _check(ctx, np.full(50, 0.5), np.linspace(0, 0.02, 50), ds, de)  # all closer than DistScans
    _check(ctx, np.array([1.0, 1.0]), np.array([0.0, 1e-9]), ds, de)


def test_interpolate_rejects_endless_inputs(ctx):
    """Arguments that would make the reference's walk loop forever are
    LGS_ERR_INVALID_ARG: dist_scans <= 0 or > dist_threshold_empty, non-finite
    distances, NaN/inf points."""
    a = np.linspace(-1.0, 1.0, 20)
    sc = ctx.scan(np.full(20, 2.0), a)
    for ds, de in [(0.0, 0.25), (-0.05, 0.25), (0.3, 0.25), (np.nan, 0.25), (0.05, np.inf)]:
        with pytest.raises(abi.LgsError):
            ctx.interpolate(sc, ds, de)
    for bad in (np.nan, np.inf):
        r = np.full(20, 2.0)
        r[7] = bad
        with pytest.raises(abi.LgsError):
            ctx.interpolate(ctx.scan(r, a), 0.05, 0.25)
    assert len(ctx.interpolate(sc, 0.05, 0.25).ranges) > 20


def test_interpolated_scan_matches_like_the_oracle(ctx, world):
    """Interpolate, then OptimizePose(query) on the device scan == the oracle on
    the oracle's interpolated ranges/angles (the frontend's order)."""
    cells, mx, my = build_map(world, 400, 0.05, 100, scene.arc_poses(5), n_beams=541)
    ang = scene.beam_angles(1081)
    rng = np.random.default_rng(3)
    P, cost = abi.RtcsmParams(5, 0.3, 0.3, 0.4, 20.0), launcher_cost()
    g = ctx.grid_from_array(cells, mx, my, 0.05)
    for k in range(3):
        true = (rng.uniform(-0.5, 0.5), rng.uniform(-0.5, 0.5), rng.uniform(-np.pi, np.pi))
        init = (true[0] + 0.1, true[1] - 0.1, true[2] + 0.05)
        r = scene.ray_cast(world, true, ang)
        isc = ctx.interpolate(ctx.scan(r, ang))
        orr, oa = ob.scan_interpolate(r, ang, 0.05, 0.25)
        got = ctx.optimize_pose_query(g, P, cost, isc, init)
        assert_same(got, oracle_match(cells, mx, my, 0.05, (5, 0.3, 0.3, 0.4, 20.0), orr, oa, init), f"k{k}")


# ------------------------------------------------------------------ chained frontend
def _odometry(rng, last):
    # the true relative motion + noise, composed onto the last estimate (bench.py run_stream)
    d = (0.1 + rng.normal(0, 0.01), rng.normal(0, 0.01), 0.02 + rng.normal(0, 0.005))
    c, s = np.cos(last[2]), np.sin(last[2])
    return (last[0] + c * d[0] - s * d[1], last[1] + s * d[0] + c * d[1], last[2] + d[2])


def _chain(ctx, world, steps, window, n_beams, check_maps_every=10, fused=False):
    """LidarGraphSlamFrontEnd::ProcessScan's per-scan loop
    (C/mapping/lidar_graph_slam_frontend.cpp:78-127) on the device, step for step
    against the same loop through the oracle: ScanInterpolator::Interpolate, the
    latest map rebuilt from the last 10 scans (ConstructMapFromScans), OptimizePose
    (query) from the odometry guess, and the local-map insert (UpdateGridMap).
    Every step's scan, match summary and (every few steps) both maps must agree."""
    from test_gpu_raycast import same_map
    ang = scene.beam_angles(n_beams)
    n = steps + 1
    truths = [(5.0 * np.cos(0.02 * k), 5.0 * np.sin(0.02 * k), 0.02 * k + np.pi / 2) for k in range(n)]
    ranges = [scene.ray_cast(world, t, ang) for t in truths]
    BP = (0.01, 20.0, 0.6, 0.45)
    bp, obp = abi.BuilderParams(*BP), ob.BuilderParams(*BP)
    params = (5, *window, 20.0)
    P, cost = abi.RtcsmParams(*params), launcher_cost()
    local = ctx.map(0.05, 100, 200, 200, center=truths[0][:2])
    latest = ctx.map(0.05, 100, 200, 200, center=truths[0][:2])
    olocal = ob.OMap(0.05, 100, 200, 200, center=truths[0][:2])
    olatest = ob.OMap(0.05, 100, 200, 200, center=truths[0][:2])
    dscans, oscans = [], []
    for k in range(n):
        dscans.append(ctx.interpolate(ctx.scan(ranges[k], ang), 0.05, 0.25))
        orr, oa = ob.scan_interpolate(ranges[k], ang, 0.05, 0.25)
        assert dscans[-1].ranges.tolist() == orr.tolist(), k
        oscans.append(ob.OScan(orr, oa))
    est = [truths[0]]
    if fused:   # GridMapBuilder::AppendScan: insert + latest map in one call
        local.append_scan(latest, dscans[:1], est[:1], bp)
    else:
        local.update_scan(dscans[0], est[0], bp)
    olocal.integrate(est[0], oscans[0], obp)
    rng = np.random.default_rng(7)
    ctx.reset_stats()
    for k in range(1, n):
        guess = _odometry(rng, est[-1])
        lo = max(0, k - 10)
        if not fused:
            latest.construct(dscans[lo:k], est[lo:k], bp)
        olatest.construct(est[lo:k], oscans[lo:k], obp)
        if k % check_maps_every == 1:
            same_map(latest, olatest, f"latest k{k}")
        got = ctx.optimize_pose_query(latest.grid(), P, cost, dscans[k], guess)
        g = olatest.geometry()
        ora = oracle_match(olatest.cells(), g["min_x"], g["min_y"], 0.05, params,
                           oscans[k].r, oscans[k].a, guess)
        assert_same(got, ora, f"step {k}")
        e = got.estimated_pose
        est.append((e.x, e.y, e.theta))
        if fused:
            local.append_scan(latest, dscans[max(0, k - 9):k + 1], est[max(0, k - 9):k + 1], bp)
        else:
            local.update_scan(dscans[k], est[-1], bp)
        olocal.integrate(est[-1], oscans[k], obp)
    same_map(local, olocal, "local map")
    return est, truths, ctx.match_counters()


def test_frontend_chain_json_window(ctx, world):
    """60 chained frontend steps with the launcher's frontend window (0.2 m / 0.2 m / 0.5 rad)."""
    est, truths, _ = _chain(ctx, world, 60, (0.2, 0.2, 0.5), 1081)
    assert abs(est[-1][0] - truths[-1][0]) < 0.2 and abs(est[-1][1] - truths[-1][1]) < 0.2


def test_frontend_chain_append_scan(ctx, world):
    """The same loop with GridMapBuilder::AppendScan as one call
    (lgs_map_append_scan: local insert + latest rebuild in one device pass)."""
    est, truths, _ = _chain(ctx, world, 30, (0.2, 0.2, 0.5), 1081, check_maps_every=3, fused=True)
    assert abs(est[-1][0] - truths[-1][0]) < 0.2 and abs(est[-1][1] - truths[-1][1]) < 0.2


def test_frontend_chain_config2_window(ctx, world):
    """Chained steps with the config-2 window (+-2 m / +-30 deg) against the
    10-scan latest map: the scan's hits sit at the map's low edges, so many
    blocks are 'unsafe' (coarse reads left of / below the map).  The superblock
    bounds also bound their fine scores (clamped strip): the
    pruned search must stay exact AND skip most blocks."""
    _, _, cnt = _chain(ctx, world, 12, (4.0, 4.0, 1.0471976), 541, check_maps_every=4)
    assert cnt["matches"] == 12 and cnt["pruned"] == 12, cnt
    assert cnt["coarse_blocks"] < 0.5 * cnt["coarse_blocks_dense"], cnt
