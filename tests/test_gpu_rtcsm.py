"""GPU parity tests for K1 (correlative matcher) and K2 (coarse-map precompute).

Every compute call goes through the C-ABI (liblgs_hip.so); the oracle
(oracle/lgs_oracle.c, test infrastructure) is the checker.  Bar:
  * cell indices, every coarse/fine score, the argmax window and the found
    flag: bit-exact;
  * normalized cost and covariance: |gpu - oracle| <= 1e-5 (north_star), the
    only differences being device exp/sin/cos vs glibc in the last ulp.
"""
import ctypes as C

import numpy as np
import pytest

import oracle_bind as ob
from conftest import launcher_cost
from lgs_amd import abi, scene

pytestmark = pytest.mark.gpu
DBL_MIN = 2.2250738585072014e-308
TOL = 1e-5


def build_map(world, n_cells, res, patch, poses, n_beams=1081, center=(0.0, 0.0)):
    ang = scene.beam_angles(n_beams)
    m = ob.OMap(res, patch, n_cells, n_cells, center)
    bp = ob.BuilderParams(0.01, 20.0, 0.6, 0.45)
    for p in poses:
        m.integrate(p, ob.OScan(scene.ray_cast(world, p, ang), ang), bp)
    return m.cells(), m.m.min_x, m.m.min_y


def oracle_match(cells, min_x, min_y, res, params, ranges, angles, init, thr=None, rel=(0, 0, 0)):
    g = ob.OGrid(cells, min_x, min_y, res)
    sc = ob.OScan(ranges, angles, rel, 0.0, 30.0)
    prm = ob.RtcsmParams(*params)
    out = ob.Summary()
    cost = launcher_cost(oracle=True)
    if thr is None:
        ob.lib().orc_rtcsm_optimize_pose_query(C.byref(g.g), C.byref(prm), C.byref(cost), C.byref(sc.s),
                                               ob.Pose(*init), C.byref(out))
    else:
        cg = ob.OGrid(ob.precompute(cells, params[0]), min_x, min_y, res)
        ob.lib().orc_rtcsm_optimize_pose(C.byref(g.g), C.byref(cg.g), C.byref(prm), C.byref(cost),
                                         C.byref(sc.s), ob.Pose(*init), thr, C.byref(out))
    return out


def assert_same(gpu, ora, tag=""):
    assert gpu.pose_found == ora.pose_found, tag
    assert list(gpu.win) == list(ora.win), tag
    assert list(gpu.steps) == list(ora.steps), tag
    assert list(gpu.best_win) == list(ora.best_win), (tag, list(gpu.best_win), list(ora.best_win))
    assert gpu.score_max == ora.score_max, (tag, gpu.score_max, ora.score_max)
    assert gpu.score_threshold == ora.score_threshold
    assert gpu.estimated_pose.tuple() == (ora.estimated_pose.x, ora.estimated_pose.y, ora.estimated_pose.theta)
    assert abs(gpu.normalized_cost - ora.normalized_cost) <= TOL, tag
    assert np.allclose(list(gpu.covariance), list(ora.covariance), rtol=0, atol=TOL), tag


# ---------------------------------------------------------------- K2
@pytest.mark.parametrize("shape,win", [((100, 100), 5), ((37, 53), 5), ((8, 3), 5), ((64, 200), 1),
                                       ((90, 70), 2), ((128, 96), 8), ((40, 41), 32), ((50, 60), 40)])
def test_precompute_parity(ctx, shape, win):
    rng = np.random.default_rng(shape[0] * 1000 + win)
    cells = rng.choice([0.0, 0.0, 0.0, 0.45, 0.6, 0.999], size=shape) * rng.uniform(0.5, 1.0, size=shape)
    g = ctx.grid_from_array(cells, -1.0, -2.0, 0.05)
    out = ctx.precompute_max(g, win).download()
    assert np.array_equal(out, ob.precompute(cells, win))


# ---------------------------------------------------------------- K1 dense scores
@pytest.mark.parametrize("seed", range(3))
def test_dense_scores_bit_exact(ctx, world, seed):
    rng = np.random.default_rng(seed)
    cells, mx, my = build_map(world, 400, 0.05, 100, scene.arc_poses(4), n_beams=361)
    ang = scene.beam_angles(361)
    true = (0.5 + 0.1 * seed, 0.2, 0.3 * seed)
    r = scene.ray_cast(world, true, ang)
    init = (true[0] + rng.uniform(-0.1, 0.1), true[1] + rng.uniform(-0.1, 0.1), true[2] + 0.05)
    params = (5, 0.6, 0.6, 0.2, 20.0)
    g = ctx.grid_from_array(cells, mx, my, 0.05)
    cg = ctx.precompute_max(g, 5)
    sc = ctx.scan(r, ang)
    dims, cs, fs = ctx.dense_scores(g, cg, abi.RtcsmParams(*params), sc, init)
    og = ob.OGrid(cells, mx, my, 0.05)
    ocg = ob.OGrid(ob.precompute(cells, 5), mx, my, 0.05)
    osc = ob.OScan(r, ang)
    odims = (C.c_int * 7)()
    ocs = np.zeros_like(cs)
    ofs = np.zeros_like(fs)
    ob.lib().orc_rtcsm_dense_scores(C.byref(og.g), C.byref(ocg.g), C.byref(ob.RtcsmParams(*params)),
                                    C.byref(osc.s), ob.Pose(*init), ob.dp(ocs), ob.dp(ofs), odims)
    assert dims == list(odims)
    assert np.array_equal(cs, ocs)
    assert np.array_equal(fs, ofs)


# ---------------------------------------------------------------- K1 full match
@pytest.mark.parametrize("seed", range(12))
def test_optimize_pose_small_scenes(ctx, world, seed):
    rng = np.random.default_rng(100 + seed)
    cells, mx, my = build_map(world, 400, 0.05, 100, scene.arc_poses(5), n_beams=541)
    ang = scene.beam_angles(541)
    true = (rng.uniform(-1, 1), rng.uniform(-1, 1), rng.uniform(-np.pi, np.pi))
    r = scene.ray_cast(world, true, ang)
    init = (true[0] + rng.uniform(-0.3, 0.3), true[1] + rng.uniform(-0.3, 0.3), true[2] + rng.uniform(-0.2, 0.2))
    params = (5, 1.0, 1.0, 0.6, 20.0)
    g = ctx.grid_from_array(cells, mx, my, 0.05)
    sc = ctx.scan(r, ang)
    gpu = ctx.optimize_pose_query(g, abi.RtcsmParams(*params), launcher_cost(), sc, init)
    ora = oracle_match(cells, mx, my, 0.05, params, r, ang, init)
    assert_same(gpu, ora, f"seed{seed}")
    assert gpu.fine_blocks <= ora.fine_blocks


@pytest.mark.parametrize("low_res", [1, 3, 5, 10])
def test_optimize_pose_low_resolutions(ctx, world, low_res):
    """LowRes 5 (JSON) takes the multi-wave transposed block evaluator, other
    values (10 = factory default) the generic one-wave evaluator."""
    rng = np.random.default_rng(low_res)
    cells, mx, my = build_map(world, 400, 0.05, 100, scene.arc_poses(5), n_beams=541)
    ang = scene.beam_angles(541)
    true = (0.3, -0.4, 0.9)
    r = scene.ray_cast(world, true, ang)
    init = (true[0] + rng.uniform(-0.2, 0.2), true[1] + rng.uniform(-0.2, 0.2), true[2] + 0.1)
    params = (low_res, 0.8, 0.8, 0.4, 20.0)
    g = ctx.grid_from_array(cells, mx, my, 0.05)
    sc = ctx.scan(r, ang)
    gpu = ctx.optimize_pose_query(g, abi.RtcsmParams(*params), launcher_cost(), sc, init)
    ora = oracle_match(cells, mx, my, 0.05, params, r, ang, init)
    assert_same(gpu, ora, f"lowres{low_res}")


def test_config1_launcher_json_window(ctx, world):
    """Config 1: 360 beams, 400x400 @ 10 cm, JSON ScanMatcherRealTimeCorrelative
    (launcher_settings_default.json:42-50: LowRes 5, 0.2/0.2/0.5, 20 m)."""
    cells, mx, my = build_map(world, 400, 0.1, 100, scene.arc_poses(5), n_beams=360)
    ang = scene.beam_angles(360)
    true = (0.4, -0.3, 0.7)
    r = scene.ray_cast(world, true, ang)
    init = (0.43, -0.32, 0.68)
    params = (5, 0.2, 0.2, 0.5, 20.0)
    g = ctx.grid_from_array(cells, mx, my, 0.1)
    sc = ctx.scan(r, ang)
    gpu = ctx.optimize_pose_query(g, abi.RtcsmParams(*params), launcher_cost(), sc, init)
    ora = oracle_match(cells, mx, my, 0.1, params, r, ang, init)
    assert_same(gpu, ora)


def test_empty_map_returns_window_corner(ctx):
    """Nothing beats the threshold -> corner (-winX, -winY, -winTheta), found=0
    (C/mapping/scan_matcher_real_time_correlative.cpp:80-82, :120)."""
    cells = np.zeros((200, 200))
    ang = scene.beam_angles(181)
    r = np.full(181, 3.0)
    init = (0.1, 0.2, 0.3)
    params = (5, 0.4, 0.4, 0.3, 20.0)
    g = ctx.grid_from_array(cells, -5.0, -5.0, 0.05)
    sc = ctx.scan(r, ang)
    gpu = ctx.optimize_pose_query(g, abi.RtcsmParams(*params), launcher_cost(), sc, init)
    ora = oracle_match(cells, -5.0, -5.0, 0.05, params, r, ang, init)
    assert gpu.pose_found == 0
    assert list(gpu.best_win) == [-gpu.win[0], -gpu.win[1], -gpu.win[2]]
    assert_same(gpu, ora)


def test_uniform_map_ties(ctx):
    """Every pose ties: the first occurrence in (t, x, y) order must win."""
    cells = np.full((160, 160), 0.5)
    ang = scene.beam_angles(91)
    r = np.full(91, 1.0)
    init = (0.0, 0.0, 0.0)
    params = (5, 0.5, 0.5, 0.2, 20.0)
    g = ctx.grid_from_array(cells, -4.0, -4.0, 0.05)
    sc = ctx.scan(r, ang)
    gpu = ctx.optimize_pose_query(g, abi.RtcsmParams(*params), launcher_cost(), sc, init)
    ora = oracle_match(cells, -4.0, -4.0, 0.05, params, r, ang, init)
    assert_same(gpu, ora)


def test_beams_beyond_scan_range_max(ctx, world):
    cells, mx, my = build_map(world, 400, 0.05, 100, scene.arc_poses(4), n_beams=361)
    ang = scene.beam_angles(361)
    r = scene.ray_cast(world, (0.2, 0.1, 0.5), ang)
    r[::7] = 25.0  # >= ScanRangeMax: skipped by ComputeScanIndices, still counted in NumOfScans
    params = (5, 0.6, 0.6, 0.4, 20.0)
    init = (0.25, 0.05, 0.45)
    g = ctx.grid_from_array(cells, mx, my, 0.05)
    sc = ctx.scan(r, ang)
    gpu = ctx.optimize_pose_query(g, abi.RtcsmParams(*params), launcher_cost(), sc, init)
    ora = oracle_match(cells, mx, my, 0.05, params, r, ang, init)
    assert_same(gpu, ora)


@pytest.mark.parametrize("seed", range(4))
def test_scan_leaving_map_low_edges(ctx, world, seed):
    """Scan points left of / below the map: coarse reads out of bounds return 0
    while fine reads land inside -> 'unsafe' blocks; result must stay exact."""
    rng = np.random.default_rng(7 + seed)
    # small map anchored so that the room's lower-left walls hug x=0 / y=0
    cells, mx, my = build_map(world, 600, 0.05, 100, scene.arc_poses(5), n_beams=541)
    sub = cells[40:360, 40:360].copy()  # crop: nonzero cells at the low edges
    smx, smy = mx + 40 * 0.05, my + 40 * 0.05
    ang = scene.beam_angles(541)
    true = (rng.uniform(-1, 0), rng.uniform(-1, 0), rng.uniform(-3, 3))
    r = scene.ray_cast(world, true, ang)
    init = (true[0] + 0.1, true[1] - 0.1, true[2] + 0.1)
    params = (5, 1.0, 1.0, 0.4, 20.0)
    for thr in (None, 0.3):
        g = ctx.grid_from_array(sub, smx, smy, 0.05)
        sc = ctx.scan(r, ang)
        if thr is None:
            gpu = ctx.optimize_pose_query(g, abi.RtcsmParams(*params), launcher_cost(), sc, init)
        else:
            cg = ctx.precompute_max(g, 5)
            gpu = ctx.optimize_pose(g, cg, abi.RtcsmParams(*params), launcher_cost(), sc, init, thr)
        ora = oracle_match(sub, smx, smy, 0.05, params, r, ang, init, thr=thr)
        assert_same(gpu, ora, f"seed{seed} thr{thr}")


def test_guard_fixup_paths(ctx, world):
    """Force the host-side exactness machinery: (a) corrupt every guarded
    device index (must be detected and patched), (b) guard everything (full
    host re-projection), (c) dense refinement of every block."""
    cells, mx, my = build_map(world, 400, 0.05, 100, scene.arc_poses(4), n_beams=361)
    ang = scene.beam_angles(361)
    r = scene.ray_cast(world, (0.3, 0.3, 1.0), ang)
    params = (5, 0.5, 0.5, 0.3, 20.0)
    init = (0.35, 0.28, 1.02)
    ora = oracle_match(cells, mx, my, 0.05, params, r, ang, init)
    g = ctx.grid_from_array(cells, mx, my, 0.05)
    sc = ctx.scan(r, ang)
    P = abi.RtcsmParams(*params)
    try:
        ctx.set_option(abi.LGS_OPT_GUARD_EPS, 0.02)
        ctx.set_option(abi.LGS_OPT_INJECT_INDEX, 1)
        gpu = ctx.optimize_pose_query(g, P, launcher_cost(), sc, init)
        assert gpu.guard_hits > 0 and gpu.fixups == 1
        assert_same(gpu, ora, "inject")
        ctx.set_option(abi.LGS_OPT_INJECT_INDEX, 0)
        ctx.set_option(abi.LGS_OPT_GUARD_EPS, 0.49)
        gpu = ctx.optimize_pose_query(g, P, launcher_cost(), sc, init)
        assert gpu.guard_hits > 64
        assert_same(gpu, ora, "full-host-projection")
        ctx.set_option(abi.LGS_OPT_GUARD_EPS, 1e-9)
        ctx.set_option(abi.LGS_OPT_FORCE_DENSE, 1)
        gpu = ctx.optimize_pose_query(g, P, launcher_cost(), sc, init)
        assert_same(gpu, ora, "dense")
    finally:
        ctx.set_option(abi.LGS_OPT_GUARD_EPS, 1e-9)
        ctx.set_option(abi.LGS_OPT_INJECT_INDEX, 0)
        ctx.set_option(abi.LGS_OPT_FORCE_DENSE, 0)


def test_batch_equals_single(ctx, world):
    cells, mx, my = build_map(world, 400, 0.05, 100, scene.arc_poses(4), n_beams=361)
    ang = scene.beam_angles(361)
    g = ctx.grid_from_array(cells, mx, my, 0.05)
    cg = ctx.precompute_max(g, 5)
    P = abi.RtcsmParams(5, 0.6, 0.6, 0.4, 20.0)
    rng = np.random.default_rng(5)
    scans, inits = [], []
    for k in range(6):
        true = (rng.uniform(-1, 1), rng.uniform(-1, 1), rng.uniform(-3, 3))
        scans.append(ctx.scan(scene.ray_cast(world, true, ang), ang))
        inits.append((true[0] + 0.1, true[1] - 0.05, true[2] + 0.05))
    outs = ctx.optimize_pose_batch(g, cg, P, launcher_cost(), scans, inits, 0.6)
    for s, i, o in zip(scans, inits, outs):
        single = ctx.optimize_pose(g, cg, P, launcher_cost(), s, i, 0.6)
        assert list(o.best_win) == list(single.best_win) and o.score_max == single.score_max
        assert o.pose_found == single.pose_found and o.normalized_cost == single.normalized_cost


def test_cost_function_parity(ctx, world):
    cells, mx, my = build_map(world, 400, 0.05, 100, scene.arc_poses(4), n_beams=361)
    ang = scene.beam_angles(361)
    r = scene.ray_cast(world, (0.1, 0.2, 0.3), ang)
    g = ctx.grid_from_array(cells, mx, my, 0.05)
    sc = ctx.scan(r, ang)
    og = ob.OGrid(cells, mx, my, 0.05)
    osc = ob.OScan(r, ang)
    for pose in [(0.1, 0.2, 0.3), (0.12, 0.19, 0.31), (-0.5, 0.4, 2.0)]:
        for c in (launcher_cost(), abi.CostGEParams(0.01, 20.0, 0.075, 0.1, 2, 1.0, 0.05)):
            v = ctx.cost_greedy_endpoint(g, c, sc, pose)
            oc = ob.CostGE(c.usable_range_min, c.usable_range_max, c.hit_and_missed_dist, c.occupancy_threshold,
                           c.kernel_size, c.scaling_factor, c.standard_deviation)
            o = ob.lib().orc_cost_ge_cost(C.byref(og.g), C.byref(oc), C.byref(osc.s), ob.Pose(*pose))
            assert abs(v - o) <= TOL * max(1.0, abs(o))


# ---------------------------------------------------------------- config 2 (full size)
@pytest.fixture(scope="module")
def config2(world):
    cells, mx, my = build_map(world, 1000, 0.05, 100, scene.arc_poses(10), n_beams=1081)
    assert (mx, my) == (-25.0, -25.0) and cells.shape == (1000, 1000)
    return cells


@pytest.mark.parametrize("seed", range(3))
def test_config2_full_size_bit_exact(ctx, world, config2, seed):
    """1081 beams, +-2 m / +-30 deg, 1000x1000 @ 5 cm (PatchSize 100)."""
    rng = np.random.default_rng(seed)
    ang = scene.beam_angles(1081)
    true = (1.0, 0.6, 0.1)
    r = scene.ray_cast(world, true, ang)
    init = (true[0] + rng.uniform(-0.3, 0.3), true[1] + rng.uniform(-0.3, 0.3), true[2] + rng.uniform(-0.2, 0.2))
    params = (5, 4.0, 4.0, 1.0471976, 20.0)
    g = ctx.grid_from_array(config2, -25.0, -25.0, 0.05)
    sc = ctx.scan(r, ang)
    gpu = ctx.optimize_pose_query(g, abi.RtcsmParams(*params), launcher_cost(), sc, init)
    ora = oracle_match(config2, -25.0, -25.0, 0.05, params, r, ang, init)
    assert_same(gpu, ora, f"config2 seed{seed}")
    # superblock pruning scores a small fraction of the 421 x 17 x 17 blocks
    assert gpu.coarse_blocks < 0.25 * 421 * 17 * 17, gpu.coarse_blocks
    e = gpu.estimated_pose
    assert abs(e.x - true[0]) < 0.051 and abs(e.y - true[1]) < 0.051 and abs(e.theta - true[2]) < 0.01


# ---------------------------------------------------------------- superblock pruning
def _query_ab(ctx, g, P, sc, init):
    """Same query with superblock pruning on (default) and off."""
    try:
        ctx.set_option(abi.LGS_OPT_SUPER_PRUNE, 1)
        on = ctx.optimize_pose_query(g, P, launcher_cost(), sc, init)
        ctx.set_option(abi.LGS_OPT_SUPER_PRUNE, 0)
        off = ctx.optimize_pose_query(g, P, launcher_cost(), sc, init)
    finally:
        ctx.set_option(abi.LGS_OPT_SUPER_PRUNE, 1)
    return on, off


def _identical(a, b, tag):
    assert a.pose_found == b.pose_found, tag
    assert list(a.best_win) == list(b.best_win), tag
    assert a.score_max == b.score_max, tag
    assert a.normalized_cost == b.normalized_cost, tag
    assert list(a.covariance) == list(b.covariance), tag


@pytest.mark.parametrize("seed", range(16))
def test_super_prune_identical_to_full_scoring(ctx, world, seed):
    """Pruning only skips blocks k_select could never take: the result is
    bit-identical to scoring every coarse block, and fewer blocks are scored."""
    rng = np.random.default_rng(500 + seed)
    cells, mx, my = build_map(world, 400, 0.05, 100, scene.arc_poses(5), n_beams=541)
    ang = scene.beam_angles(541)
    true = (rng.uniform(-1, 1), rng.uniform(-1, 1), rng.uniform(-np.pi, np.pi))
    r = scene.ray_cast(world, true, ang)
    init = (true[0] + rng.uniform(-0.3, 0.3), true[1] + rng.uniform(-0.3, 0.3), true[2] + rng.uniform(-0.2, 0.2))
    params = (5, 1.0 + 0.5 * (seed % 3), 1.0, 0.6, 20.0)
    g = ctx.grid_from_array(cells, mx, my, 0.05)
    sc = ctx.scan(r, ang)
    on, off = _query_ab(ctx, g, abi.RtcsmParams(*params), sc, init)
    _identical(on, off, f"seed{seed}")
    if seed < 4:
        assert_same(on, oracle_match(cells, mx, my, 0.05, params, r, ang, init), f"seed{seed}")
    # (scans leaving this 20 m map put every angle row in the unpruned
    # 'may hold unsafe blocks' class; config 2 checks the pruning rate)
    assert on.coarse_blocks <= off.coarse_blocks
    assert on.fine_blocks <= off.coarse_blocks


@pytest.mark.parametrize("seed", range(3))
def test_super_prune_noise_map(ctx, seed):
    """Dense random map: superblock bounds are loose and many sums are close."""
    rng = np.random.default_rng(900 + seed)
    cells = rng.choice([0.0, 0.3, 0.5, 0.7, 0.9], size=(240, 260)) * rng.uniform(0.9, 1.0, size=(240, 260))
    ang = scene.beam_angles(361)
    r = rng.uniform(0.5, 4.0, size=361)
    init = (rng.uniform(-1, 1), rng.uniform(-1, 1), rng.uniform(-3, 3))
    params = (5, 0.8, 0.8, 0.3, 20.0)
    g = ctx.grid_from_array(cells, -6.0, -6.5, 0.05)
    sc = ctx.scan(r, ang)
    on, off = _query_ab(ctx, g, abi.RtcsmParams(*params), sc, init)
    _identical(on, off, f"noise{seed}")
    assert_same(on, oracle_match(cells, -6.0, -6.5, 0.05, params, r, ang, init), f"noise{seed}")


def test_super_prune_negative_cells(ctx, world):
    """The bound needs nonnegative cells; a map with negative values must
    disable pruning (every block scored) and stay exact."""
    cells, mx, my = build_map(world, 400, 0.05, 100, scene.arc_poses(4), n_beams=361)
    cells = cells - 0.2 * (cells == 0.0)
    ang = scene.beam_angles(361)
    true = (0.2, -0.1, 0.4)
    r = scene.ray_cast(world, true, ang)
    init = (0.25, -0.05, 0.43)
    params = (5, 0.6, 0.6, 0.3, 20.0)
    g = ctx.grid_from_array(cells, mx, my, 0.05)
    sc = ctx.scan(r, ang)
    on, off = _query_ab(ctx, g, abi.RtcsmParams(*params), sc, init)
    _identical(on, off, "negative")
    assert on.coarse_blocks == off.coarse_blocks
    assert_same(on, oracle_match(cells, mx, my, 0.05, params, r, ang, init), "negative")


def test_super_prune_wide_window(ctx, world):
    """+-4.5 m window: 37x37 coarse blocks per angle, 100 superblocks (two
    64-superblock chunks in k_super)."""
    cells, mx, my = build_map(world, 400, 0.05, 100, scene.arc_poses(5), n_beams=541)
    ang = scene.beam_angles(541)
    true = (0.6, -0.2, 1.3)
    r = scene.ray_cast(world, true, ang)
    init = (0.9, -0.5, 1.35)
    params = (5, 9.0, 9.0, 0.2, 20.0)
    g = ctx.grid_from_array(cells, mx, my, 0.05)
    sc = ctx.scan(r, ang)
    on, off = _query_ab(ctx, g, abi.RtcsmParams(*params), sc, init)
    assert list(on.win)[:2] == [90, 90]
    _identical(on, off, "wide")
    assert_same(on, oracle_match(cells, mx, my, 0.05, params, r, ang, init), "wide")


@pytest.mark.parametrize("rx,ry", [(9.0, 1.0), (1.0, 9.0)])
def test_super_prune_anisotropic_windows(ctx, world, rx, ry):
    """Windows whose superblock grid is 10 x 2 / 2 x 10: too many superblock
    rows or columns for the octet layout, so k_super over the fp16 sub-phase
    planes bounds them -- pruned == unpruned == oracle."""
    cells, mx, my = build_map(world, 400, 0.05, 100, scene.arc_poses(5), n_beams=541)
    ang = scene.beam_angles(541)
    true = (0.4, -0.1, 0.9)
    r = scene.ray_cast(world, true, ang)
    init = (0.5, -0.2, 0.95)
    params = (5, rx, ry, 0.2, 20.0)
    g = ctx.grid_from_array(cells, mx, my, 0.05)
    sc = ctx.scan(r, ang)
    on, off = _query_ab(ctx, g, abi.RtcsmParams(*params), sc, init)
    _identical(on, off, "aniso")
    assert_same(on, oracle_match(cells, mx, my, 0.05, params, r, ang, init), "aniso")
    assert on.coarse_blocks < off.coarse_blocks, (on.coarse_blocks, off.coarse_blocks)


def test_super_prune_batch_and_fixed_threshold(ctx, world):
    """OptimizePose with a caller coarse map (decimated per batch) and a
    fixed threshold: pruned batch == unpruned batch."""
    cells, mx, my = build_map(world, 400, 0.05, 100, scene.arc_poses(4), n_beams=361)
    ang = scene.beam_angles(361)
    g = ctx.grid_from_array(cells, mx, my, 0.05)
    cg = ctx.precompute_max(g, 5)
    P = abi.RtcsmParams(5, 0.6, 0.6, 0.4, 20.0)
    rng = np.random.default_rng(77)
    scans, inits = [], []
    for _ in range(5):
        true = (rng.uniform(-1, 1), rng.uniform(-1, 1), rng.uniform(-3, 3))
        scans.append(ctx.scan(scene.ray_cast(world, true, ang), ang))
        inits.append((true[0] + 0.1, true[1] - 0.05, true[2] + 0.05))
    try:
        ctx.set_option(abi.LGS_OPT_SUPER_PRUNE, 0)
        off = ctx.optimize_pose_batch(g, cg, P, launcher_cost(), scans, inits, 0.5)
        ctx.set_option(abi.LGS_OPT_SUPER_PRUNE, 1)
        on = ctx.optimize_pose_batch(g, cg, P, launcher_cost(), scans, inits, 0.5)
    finally:
        ctx.set_option(abi.LGS_OPT_SUPER_PRUNE, 1)
    for k, (a, b) in enumerate(zip(on, off)):
        _identical(a, b, f"batch{k}")
