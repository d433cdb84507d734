"""GPU parity tests for the one-launch small-window search (k_match_small,
DESIGN.md §4.1c): windows whose coarse lattice holds ONE block per angle
(2 winX < LowRes and 2 winY < LowRes -- the launcher JSON frontend window).

The kernel derives every coarse value from the fine map (the max of the
LowRes x LowRes cells a beam's block covers, SlidingWindowMax's clamped last
window at the high edges, 0 outside the map) instead of reading a precomputed
coarse map, scores every angle's block and fine poses, and replays the
reference's walk (scan_matcher_real_time_correlative.cpp:88-112) on the last
workgroup.  Bar: bit-exact against the oracle for the argmax window, every
score, the found flag and the refined-block count (fine_blocks is the
reference's exact count here: nothing is pruned); cost and covariance within
1e-5 (north_star), as for every match.
"""
import numpy as np
import pytest

from conftest import launcher_cost
from lgs_amd import abi, scene
from test_gpu_rtcsm import assert_same, build_map, oracle_match

pytestmark = pytest.mark.gpu


def _match(ctx, cells, mx, my, res, params, r, ang, init, small=True):
    try:
        ctx.set_option(abi.LGS_OPT_SMALL_WINDOW, 1 if small else 0)
        ctx.set_option(abi.LGS_OPT_PROFILE, 1)
        ctx.reset_stats()
        g = ctx.grid_from_array(cells, mx, my, res)
        sc = ctx.scan(r, ang)
        out = ctx.optimize_pose_query(g, abi.RtcsmParams(*params), launcher_cost(), sc, init)
        launches = ctx.kernel_stats().get("k_match_small", {}).get("launches", 0)
    finally:
        ctx.set_option(abi.LGS_OPT_PROFILE, 0)
        ctx.set_option(abi.LGS_OPT_SMALL_WINDOW, 1)
    return out, launches


def _exact(gpu, ora, tag):
    assert_same(gpu, ora, tag)
    assert gpu.fine_blocks == ora.fine_blocks, (tag, gpu.fine_blocks, ora.fine_blocks)
    assert gpu.coarse_blocks == (2 * gpu.win[2] + 1), tag   # K = T x 1 block: every block scored


@pytest.fixture(scope="module")
def room(world):
    return build_map(world, 400, 0.05, 100, scene.arc_poses(5), n_beams=541)


@pytest.mark.parametrize("low_res", [2, 3, 4, 5, 6, 7, 8])
def test_small_window_low_resolutions(ctx, world, room, low_res):
    """Every LowRes the kernel is built for (2..7: the adder wave holds the
    LowRes^2 pose chains and the coarse one), with the widest one-block window
    (winX = winY = (LowRes - 1) // 2); LowRes 8 takes the general path."""
    cells, mx, my = room
    ang = scene.beam_angles(541)
    rng = np.random.default_rng(40 + low_res)
    true = (rng.uniform(-1, 1), rng.uniform(-1, 1), rng.uniform(-np.pi, np.pi))
    r = scene.ray_cast(world, true, ang)
    init = (true[0] + 0.03, true[1] - 0.02, true[2] + 0.05)
    # winX = ceil(0.5 rangeX / stepX) = (LowRes - 1) // 2 (a hair under the
    # exact multiple: 0.5 * 0.3 / 0.05 rounds above 3)
    rng_xy = max(0.0, (2 * ((low_res - 1) // 2) - 0.01) * 0.05)
    params = (low_res, rng_xy, rng_xy, 0.5, 20.0)
    gpu, n = _match(ctx, cells, mx, my, 0.05, params, r, ang, init)
    assert n == (1 if low_res <= 7 else 0), n
    ora = oracle_match(cells, mx, my, 0.05, params, r, ang, init)
    if n:
        _exact(gpu, ora, f"lr{low_res}")
    else:
        assert_same(gpu, ora, f"lr{low_res}")


@pytest.mark.parametrize("seed", range(6))
def test_small_window_json_frontend(ctx, world, room, seed):
    """The launcher JSON window (LowRes 5, 0.2/0.2/0.5, 20 m), 1081 beams, and
    the general path (LGS_OPT_SMALL_WINDOW 0) agrees on every result field."""
    cells, mx, my = room
    ang = scene.beam_angles(1081)
    rng = np.random.default_rng(70 + seed)
    true = (rng.uniform(-1.5, 1.5), rng.uniform(-1.5, 1.5), rng.uniform(-np.pi, np.pi))
    r = scene.ray_cast(world, true, ang)
    init = (true[0] + rng.uniform(-0.08, 0.08), true[1] + rng.uniform(-0.08, 0.08), true[2] + rng.uniform(-0.2, 0.2))
    params = (5, 0.2, 0.2, 0.5, 20.0)
    on, n_on = _match(ctx, cells, mx, my, 0.05, params, r, ang, init)
    off, n_off = _match(ctx, cells, mx, my, 0.05, params, r, ang, init, small=False)
    assert n_on == 1 and n_off == 0
    _exact(on, oracle_match(cells, mx, my, 0.05, params, r, ang, init), f"json{seed}")
    assert list(on.best_win) == list(off.best_win) and on.score_max == off.score_max
    assert on.pose_found == off.pose_found and on.normalized_cost == off.normalized_cost
    assert list(on.covariance) == list(off.covariance)


@pytest.mark.parametrize("corner", ["low", "high"])
def test_small_window_map_edges(ctx, world, corner):
    """Crops that put the scan's hits against the map's low or high edges:
    beams whose block starts outside the map (coarse value 0 while fine reads
    land inside) and beams in SlidingWindowMax's repeated last window."""
    cells, mx, my = build_map(world, 600, 0.05, 100, scene.arc_poses(5), n_beams=541)
    sub = cells[40:360, 40:360].copy() if corner == "low" else cells[240:560, 240:560].copy()
    off = 40 if corner == "low" else 240
    smx, smy = mx + off * 0.05, my + off * 0.05
    ang = scene.beam_angles(541)
    rng = np.random.default_rng(3 if corner == "low" else 4)
    for k in range(3):
        true = (rng.uniform(-1, 0), rng.uniform(-1, 0), rng.uniform(-3, 3)) if corner == "low" else \
            (rng.uniform(0, 1), rng.uniform(0, 1), rng.uniform(-3, 3))
        r = scene.ray_cast(world, true, ang)
        init = (true[0] + 0.05, true[1] - 0.05, true[2] + 0.1)
        params = (5, 0.2, 0.2, 0.5, 20.0)
        gpu, n = _match(ctx, sub, smx, smy, 0.05, params, r, ang, init)
        assert n == 1
        _exact(gpu, oracle_match(sub, smx, smy, 0.05, params, r, ang, init), f"{corner}{k}")


@pytest.mark.parametrize("shape", [(3, 200), (200, 5), (200, 4), (2, 3)])
def test_small_window_maps_narrower_than_window(ctx, shape):
    """Maps thinner than LowRes: SlidingWindowMax pads with 0 past the end, so
    a row of negative cells still has coarse value 0.  Maps narrower (in x)
    than LowRes take the general path (k_match_small's clamped row runs need
    W >= LowRes), with the same result."""
    rng = np.random.default_rng(shape[0] * 7 + shape[1])
    cells = rng.choice([-0.3, 0.0, 0.4, 0.8], size=shape) * rng.uniform(0.5, 1.0, size=shape)
    ang = scene.beam_angles(181)
    r = rng.uniform(0.05, 0.4, size=181)
    init = (0.05, 0.05, 0.1)
    params = (5, 0.2, 0.2, 0.3, 20.0)
    gpu, n = _match(ctx, cells, 0.0, 0.0, 0.05, params, r, ang, init)
    assert n == (1 if shape[1] >= 5 else 0), n
    ora = oracle_match(cells, 0.0, 0.0, 0.05, params, r, ang, init)
    if n:
        _exact(gpu, ora, f"narrow{shape}")
    else:
        assert_same(gpu, ora, f"narrow{shape}")


@pytest.mark.parametrize("seed", range(3))
def test_small_window_noise_and_negative_cells(ctx, seed):
    """Dense random map with negative cells: many near-equal sums and maxima
    that are not the window's first cell."""
    rng = np.random.default_rng(1300 + seed)
    cells = rng.choice([-0.5, 0.0, 0.3, 0.5, 0.7, 0.9], size=(240, 260)) * rng.uniform(0.9, 1.0, size=(240, 260))
    ang = scene.beam_angles(361)
    r = rng.uniform(0.5, 4.0, size=361)
    init = (rng.uniform(-1, 1), rng.uniform(-1, 1), rng.uniform(-3, 3))
    params = (5, 0.2, 0.2, 0.4, 20.0)
    gpu, n = _match(ctx, cells, -6.0, -6.5, 0.05, params, r, ang, init)
    assert n == 1
    _exact(gpu, oracle_match(cells, -6.0, -6.5, 0.05, params, r, ang, init), f"noise{seed}")


def test_small_window_ties_and_empty(ctx):
    """A uniform map (every pose ties: the first in (t, x, y) order wins), an
    empty map (nothing beats the threshold: the window corner), and a scan
    with no beam below ScanRangeMax (Nv = 0)."""
    ang = scene.beam_angles(91)
    params = (5, 0.2, 0.2, 0.2, 20.0)
    cases = [("ties", np.full((160, 160), 0.5), np.full(91, 1.0)),
             ("empty", np.zeros((160, 160)), np.full(91, 1.0)),
             ("nv0", np.full((160, 160), 0.5), np.full(91, 25.0))]
    for tag, cells, r in cases:
        gpu, n = _match(ctx, cells, -4.0, -4.0, 0.05, params, r, ang, (0.0, 0.0, 0.0))
        assert n == 1
        _exact(gpu, oracle_match(cells, -4.0, -4.0, 0.05, params, r, ang, (0.0, 0.0, 0.0)), tag)


def test_small_window_guard_fixups(ctx, world, room):
    """Corrupted guarded indices (k_patch + a mode-1 rerun that reads the
    patched rows) and a full host re-projection (uploaded rows)."""
    cells, mx, my = room
    ang = scene.beam_angles(361)
    r = scene.ray_cast(world, (0.3, 0.3, 1.0), ang)
    params = (5, 0.2, 0.2, 0.4, 20.0)
    init = (0.32, 0.29, 1.01)
    ora = oracle_match(cells, mx, my, 0.05, params, r, ang, init)
    try:
        ctx.set_option(abi.LGS_OPT_GUARD_EPS, 0.02)
        ctx.set_option(abi.LGS_OPT_INJECT_INDEX, 1)
        gpu, n = _match(ctx, cells, mx, my, 0.05, params, r, ang, init)
        assert n == 2 and gpu.guard_hits > 0 and gpu.fixups == 1, (n, gpu.guard_hits, gpu.fixups)
        _exact(gpu, ora, "inject")
        ctx.set_option(abi.LGS_OPT_INJECT_INDEX, 0)
        ctx.set_option(abi.LGS_OPT_GUARD_EPS, 0.49)
        gpu, n = _match(ctx, cells, mx, my, 0.05, params, r, ang, init)
        assert n == 2 and gpu.guard_hits > 64
        _exact(gpu, ora, "full-host-projection")
    finally:
        ctx.set_option(abi.LGS_OPT_GUARD_EPS, 1e-9)
        ctx.set_option(abi.LGS_OPT_INJECT_INDEX, 0)


def test_small_window_batch_and_counter_reuse(ctx, world, room):
    """A batch of queries with different angle counts (T) and valid-beam
    counts, then lone calls with other T on the same context: the per-item
    wrap-around counters must come back to 0 after every launch."""
    cells, mx, my = room
    g = ctx.grid_from_array(cells, mx, my, 0.05)
    rng = np.random.default_rng(11)
    ang = scene.beam_angles(721)
    scans, inits, raw = [], [], []
    for k in range(5):
        true = (rng.uniform(-1, 1), rng.uniform(-1, 1), rng.uniform(-3, 3))
        r = scene.ray_cast(world, true, ang)
        r[rng.random(721) < 0.1 * k] = 25.0   # fewer valid beams per item
        raw.append(r)
        scans.append(ctx.scan(r, ang))
        inits.append((true[0] + 0.04, true[1] - 0.03, true[2] + 0.1))
    for theta in (0.5, 0.3, 0.7):
        params = (5, 0.2, 0.2, theta, 20.0)
        outs = ctx.optimize_pose_query_batch([g] * len(scans), abi.RtcsmParams(*params), launcher_cost(), scans, inits)
        for k, o in enumerate(outs):
            _exact(o, oracle_match(cells, mx, my, 0.05, params, raw[k], ang, inits[k]), f"batch{theta}/{k}")
        lone, n = _match(ctx, cells, mx, my, 0.05, params, raw[0], ang, inits[0])
        assert n == 1
        _exact(lone, oracle_match(cells, mx, my, 0.05, params, raw[0], ang, inits[0]), f"lone{theta}")
