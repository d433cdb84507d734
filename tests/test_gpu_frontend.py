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
