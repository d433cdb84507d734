"""K4 parity: device ScanMatcherLinearSolver + CostSquareError vs the oracle.

Reference: C/mapping/scan_matcher_linear_solver.cpp:38-148 and
C/mapping/cost_function_square_error.cpp (restated in oracle/lgs_oracle.c).

Tolerance: none -- bit-exact.  The device restates glibc's sincos() and
pow(x, 3.0) operation for operation (csrc/glibc_math.hpp, pinned against this
image's libm by tests/test_libm_pin.py), folds pow(x, 2.0) to x*x as GCC does,
and adds every sum in beam order like the reference's loops, so every
OptimizeStep, every cost, the stopping decision, the covariance and the whole
50-iteration trajectory equal the oracle's bit for bit:
  * every step: the device's pose k+1 == the oracle's OptimizeStep from the
    device's pose k, and the cost the convergence test saw == the oracle's
    Cost at that pose;
  * the stopping rule (:64-69) on those costs, the summary covariance;
  * the whole loop against the oracle's own loop (same iteration count, same
    trajectory, same estimated pose and normalized cost) -- BASELINE config 3
    (1081 beams, 50 iterations, 1000x1000 @ 5 cm) over 16 seeds, plus
    361-beam and shape-edge cases.
The reference's loop is chaotic at the last-ulp level (ComputeSmoothedValue
truncates coordinates that sit on integers +- rounding; a 1-ulp change of the
initial pose moves its 50-iteration result by up to ~1e-5, tools/diag_ls.py),
so anything short of the oracle's exact arithmetic diverges end to end.
"""
import ctypes as C

import numpy as np
import pytest

import oracle_bind as ob
from lgs_amd import abi, scene

pytestmark = pytest.mark.gpu

CONFIG3 = (50, 0.0, 0.01, 20.0, 1e-3, 1e-3, 0.01, 20.0)     # BASELINE config 3
JSON_DEFAULT = (100, 1e-3, 0.01, 20.0, 1e-3, 1e-3, 0.01, 20.0)  # launcher_settings_default.json:31-40 + :12-15
BP = (0.01, 20.0, 0.6, 0.45)


@pytest.fixture(scope="module")
def small_map(world):
    """600x600 @ 5 cm map built by the oracle's UpdateGridMap restatement."""
    ang = scene.beam_angles(361)
    m = ob.OMap(0.05, 100, 600, 600)
    for p in scene.arc_poses(6):
        m.integrate(p, ob.OScan(scene.ray_cast(world, p, ang), ang), ob.BuilderParams(*BP))
    return m.cells(), m.m.min_x, m.m.min_y


@pytest.fixture(scope="module")
def big_map(world):
    """config 3: 1000x1000 @ 5 cm, 1081-beam arc map (numpy builder)."""
    ang = scene.beam_angles(1081)
    w, h, mx, my = scene.map_geometry(1000, 100, 0.05)
    return scene.approx_occupancy_map(world, scene.arc_poses(10), ang, w, h, mx, my, 0.05), mx, my


def oracle_solve(og, lp, r, ang, init, rel=(0.0, 0.0, 0.0), min_range=0.0, max_range=30.0):
    out = ob.Summary()
    n = max(1, lp[0])
    traj = (ob.Pose * n)()
    ob.lib().orc_linsolve_optimize_pose(C.byref(og.g), C.byref(ob.LinsolveParams(*lp)),
                                        C.byref(ob.OScan(r, ang, rel, min_range, max_range).s),
                                        ob.Pose(*init), C.byref(out), traj)
    return out, [(p.x, p.y, p.theta) for p in traj]


def check_solve(ctx, g, og, lp, r, ang, init, rel=(0.0, 0.0, 0.0), min_range=0.0, max_range=30.0):
    d, dtraj = ctx.linsolve(g, abi.LinsolveParams(*lp), ctx.scan(r, ang, rel, min_range, max_range), init,
                            trajectory=True)
    olp = ob.LinsolveParams(*lp)
    osc = ob.OScan(r, ang, rel, min_range, max_range)
    assert d.pose_found == 1
    assert len(dtraj) == d.iterations >= 1
    # 1. every OptimizeStep from the device's own previous pose, and the cost
    #    the convergence test saw, against the oracle at the same poses
    prev = (d.sensor_pose.x, d.sensor_pose.y, d.sensor_pose.theta)
    for k, t in enumerate(dtraj):
        o = ob.lib().orc_linsolve_step(C.byref(og.g), C.byref(olp), C.byref(osc.s), ob.Pose(*prev))
        assert (o.x, o.y, o.theta) == tuple(t[:3]), (k, (o.x, o.y, o.theta), t)
        oc = ob.lib().orc_sq_cost(C.byref(og.g), lp[6], lp[7], C.byref(osc.s), ob.Pose(*t[:3]))
        assert oc == t[3], (k, oc, t[3])
        prev = t[:3]
    # 2. the stopping rule (:64-69) on the costs the device saw
    stop, pc = None, float("inf")
    for k, t in enumerate(dtraj, 1):
        if k >= lp[0] or abs(pc - t[3]) < lp[1]:
            stop = k
            break
        pc = t[3]
    assert stop == d.iterations
    assert d.cost == dtraj[-1][3] and d.normalized_cost == d.cost / len(r)
    bp = d.best_sensor_pose
    assert (bp.x, bp.y, bp.theta) == dtraj[-1][:3]
    # 3. covariance at the final pose
    cov = (C.c_double * 9)()
    ob.lib().orc_sq_covariance(C.byref(og.g), lp[6], lp[7], C.byref(osc.s), ob.Pose(bp.x, bp.y, bp.theta), cov)
    assert list(d.covariance) == list(cov)
    # 4. whole loop vs the oracle's own loop: identical
    o, otraj = oracle_solve(og, lp, r, ang, init, rel, min_range, max_range)
    assert d.iterations == o.best_win[0]
    assert [tuple(t[:3]) for t in dtraj] == otraj[:d.iterations]
    de, oe = d.estimated_pose, o.estimated_pose
    assert (de.x, de.y, de.theta) == (oe.x, oe.y, oe.theta)
    assert d.normalized_cost == o.normalized_cost
    assert list(d.covariance) == list(o.covariance)
    return d, o


def test_cost_and_covariance_at_pose(ctx, world, small_map):
    cells, mx, my = small_map
    g = ctx.grid_from_array(cells, mx, my, 0.05)
    og = ob.OGrid(cells, mx, my, 0.05)
    ang = scene.beam_angles(361)
    rng = np.random.default_rng(1)
    for _ in range(25):
        true = (rng.uniform(-1.5, 1.5), rng.uniform(-1.5, 1.5), rng.uniform(-3, 3))
        r = scene.ray_cast(world, true, ang)
        # evaluated off the scan's true pose: hit points then do not sit exactly
        # on the room's cell-aligned walls (integer coordinates, where the
        # reference's truncation makes the value discontinuous)
        p = (true[0] + rng.uniform(-0.04, 0.04), true[1] + rng.uniform(-0.04, 0.04), true[2] + 0.01)
        c, cov = ctx.cost_square_error(g, 0.01, 20.0, ctx.scan(r, ang), p, covariance=True)
        osc = ob.OScan(r, ang)
        oc = ob.lib().orc_sq_cost(C.byref(og.g), 0.01, 20.0, C.byref(osc.s), ob.Pose(*p))
        ocov = (C.c_double * 9)()
        ob.lib().orc_sq_covariance(C.byref(og.g), 0.01, 20.0, C.byref(osc.s), ob.Pose(*p), ocov)
        assert c == oc
        assert list(cov) == list(ocov)


def test_cost_outside_and_empty(ctx, world):
    """Poses far outside the map (index clamping) and an all-unknown map."""
    ang = scene.beam_angles(181)
    cells = np.zeros((120, 100))
    cells[40:60, 30:70] = 0.8
    g = ctx.grid_from_array(cells, -2.5, -3.0, 0.05)
    og = ob.OGrid(cells, -2.5, -3.0, 0.05)
    r = scene.ray_cast(world, (0.0, 0.0, 0.3), ang)
    for p in [(0.0, 0.0, 0.0), (50.0, -40.0, 1.0), (-1e4, 1e4, 2.0), (0.1, 0.1, -3.1)]:
        c = ctx.cost_square_error(g, 0.01, 20.0, ctx.scan(r, ang), p)
        oc = ob.lib().orc_sq_cost(C.byref(og.g), 0.01, 20.0, C.byref(ob.OScan(r, ang).s), ob.Pose(*p))
        assert c == oc
    ez = ctx.grid_from_array(np.zeros((50, 50)), 0.0, 0.0, 0.05)
    oz = ob.OGrid(np.zeros((50, 50)), 0.0, 0.0, 0.05)
    d, _ = check_solve(ctx, ez, oz, (5, 0.0, 0.01, 20.0, 1e-3, 1e-3, 0.01, 20.0), r, ang, (1.0, 1.0, 0.0))
    assert d.iterations == 5


@pytest.mark.parametrize("seed", range(6))
def test_linsolve_small(ctx, world, small_map, seed):
    cells, mx, my = small_map
    g = ctx.grid_from_array(cells, mx, my, 0.05)
    og = ob.OGrid(cells, mx, my, 0.05)
    ang = scene.beam_angles(361)
    rng = np.random.default_rng(100 + seed)
    true = (rng.uniform(-1, 1), rng.uniform(-1, 1), rng.uniform(-3, 3))
    r = scene.ray_cast(world, true, ang)
    init = (true[0] + rng.uniform(-0.05, 0.05), true[1] + rng.uniform(-0.05, 0.05), true[2] + rng.uniform(-0.03, 0.03))
    lp = CONFIG3 if seed % 2 == 0 else JSON_DEFAULT
    check_solve(ctx, g, og, lp, r, ang, init)


def test_linsolve_sensor_offset_and_filters(ctx, world, small_map):
    """Relative sensor pose (Compound / MoveBackward) and differing step / cost
    beam filters (matcher usable range vs CostSquareError's vs scan min/max)."""
    cells, mx, my = small_map
    g = ctx.grid_from_array(cells, mx, my, 0.05)
    og = ob.OGrid(cells, mx, my, 0.05)
    ang = scene.beam_angles(361)
    r = scene.ray_cast(world, (0.4, -0.3, 0.7), ang)
    lp = (30, 0.0, 0.5, 6.0, 2e-3, 5e-4, 1.0, 9.0)
    check_solve(ctx, g, og, lp, r, ang, (0.37, -0.27, 0.68), rel=(0.1, -0.05, 0.02), min_range=0.3,
                max_range=12.0)


def test_linsolve_batch_equals_single(ctx, world, small_map):
    cells, mx, my = small_map
    g = ctx.grid_from_array(cells, mx, my, 0.05)
    ang = scene.beam_angles(361)
    rng = np.random.default_rng(7)
    scans, inits = [], []
    for _ in range(9):
        true = (rng.uniform(-1, 1), rng.uniform(-1, 1), rng.uniform(-3, 3))
        scans.append(ctx.scan(scene.ray_cast(world, true, ang), ang))
        inits.append((true[0] + 0.02, true[1] - 0.03, true[2] + 0.01))
    lp = abi.LinsolveParams(*CONFIG3)
    batch = ctx.linsolve_batch(g, lp, scans, inits)
    # a lone refine runs split over one workgroup per 64 beams (the default),
    # on one workgroup (LGS_OPT_LINSOLVE_SPLIT 0), or -- after a hand-off
    # time-out, forced here with LGS_OPT_HANDOFF_SPIN_US 0 -- split first and
    # then rerun on one workgroup: every path computes the batch kernel's bits
    for split, spin in ((1, 200000), (0, 200000), (1, 0)):
        ctx.set_option(abi.LGS_OPT_LINSOLVE_SPLIT, split)
        ctx.set_option(abi.LGS_OPT_HANDOFF_SPIN_US, spin)
        try:
            for s, i, b in zip(scans, inits, batch):
                one = ctx.linsolve(g, lp, s, i)
                assert (one.estimated_pose.x, one.estimated_pose.y, one.estimated_pose.theta) == \
                    (b.estimated_pose.x, b.estimated_pose.y, b.estimated_pose.theta), (split, spin)
                assert one.normalized_cost == b.normalized_cost and list(one.covariance) == list(b.covariance)
                assert one.iterations == b.iterations
        finally:
            ctx.set_option(abi.LGS_OPT_LINSOLVE_SPLIT, 1)
            ctx.set_option(abi.LGS_OPT_HANDOFF_SPIN_US, 200000)


@pytest.mark.parametrize("n_beams", [1, 63, 65, 1280, 1281, 3000, 8300])
def test_linsolve_shapes(ctx, world, small_map, n_beams):
    """Beam counts at the kernels' edges: 1 beam (one workgroup), 63/65 (one
    and two split groups), 1280/1281 (the split refine's 20-group limit and one
    k_linsolve chunk; beyond, the one-workgroup kernel runs several chunks whose
    sums continue in beam order)."""
    cells, mx, my = small_map
    g = ctx.grid_from_array(cells, mx, my, 0.05)
    og = ob.OGrid(cells, mx, my, 0.05)
    ang = scene.beam_angles(n_beams) if n_beams > 1 else np.array([0.3])
    r = scene.ray_cast(world, (0.2, -0.1, 0.4), ang)
    check_solve(ctx, g, og, (20, 0.0, 0.01, 20.0, 1e-3, 1e-3, 0.01, 20.0), r, ang, (0.23, -0.12, 0.41))


def test_linsolve_config3(ctx, world, big_map):
    """BASELINE config 3: 1081 beams, 50 iterations, 1000x1000 @ 5 cm, 16
    seeds: every step, cost, stopping decision and end point bit-exact."""
    cells, mx, my = big_map
    g = ctx.grid_from_array(cells, mx, my, 0.05)
    og = ob.OGrid(cells, mx, my, 0.05)
    ang = scene.beam_angles(1081)
    for seed in range(16):
        rng = np.random.default_rng(300 + seed)
        true = (rng.uniform(-1.2, 1.2), rng.uniform(-1.2, 1.2), rng.uniform(-3, 3))
        r = scene.ray_cast(world, true, ang)
        init = (true[0] + rng.uniform(-0.05, 0.05), true[1] + rng.uniform(-0.05, 0.05),
                true[2] + rng.uniform(-0.03, 0.03))
        d, o = check_solve(ctx, g, og, CONFIG3, r, ang, init)
        assert d.iterations == 50


def test_linsolve_batch_fills_device(ctx, world, small_map):
    """A device-filling batch (more refines than CUs: 300 workgroups on 256
    CUs, as bench.py's batched_refines_per_s_per_gpu_256 and more) gives
    every refine the bits of the lone refine."""
    cells, mx, my = small_map
    g = ctx.grid_from_array(cells, mx, my, 0.05)
    ang = scene.beam_angles(361)
    rng = np.random.default_rng(17)
    base = []
    for _ in range(12):
        true = (rng.uniform(-1, 1), rng.uniform(-1, 1), rng.uniform(-3, 3))
        base.append((ctx.scan(scene.ray_cast(world, true, ang), ang), true))
    scans, inits = [], []
    for k in range(300):
        s, true = base[k % len(base)]
        scans.append(s)
        inits.append((true[0] + 0.001 * (k % 7), true[1] - 0.002 * (k % 5), true[2] + 0.001 * (k % 3)))
    lp = abi.LinsolveParams(*CONFIG3)
    batch = ctx.linsolve_batch(g, lp, scans, inits)
    for k in list(range(0, 300, 23)) + [299]:
        one = ctx.linsolve(g, lp, scans[k], inits[k])
        b = batch[k]
        assert (one.estimated_pose.x, one.estimated_pose.y, one.estimated_pose.theta) == \
            (b.estimated_pose.x, b.estimated_pose.y, b.estimated_pose.theta), k
        assert one.normalized_cost == b.normalized_cost and one.iterations == b.iterations, k
