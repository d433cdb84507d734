"""CPU tests of the oracle (oracle/lgs_oracle.c) against the known-answer
vectors in tests/golden/kat.json, plus property tests of the restatement.

No GPU needed.  See tests/golden/make_kat.py for where the vectors come from
("parity unpinned": the reference has no tests and is not buildable here).
"""
import ctypes as C
import json
import math
import os

import numpy as np
import pytest

import oracle_bind as ob

KAT = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "kat.json")))
DBL_MIN = 2.2250738585072014e-308


@pytest.mark.parametrize("case", KAT["bresenham_hand"] + KAT["bresenham_py"])
def test_bresenham_kat(case):
    assert [list(p) for p in ob.bresenham(*case["args"])] == case["pts"]


@pytest.mark.parametrize("case", KAT["swm_hand"] + KAT["swm_py"])
def test_sliding_window_max_kat(case):
    v = np.array(case["in"], dtype=np.float64)
    out = np.zeros_like(v)
    ob.lib().orc_sliding_window_max(ob.dp(v), 1, ob.dp(out), 1, len(v), case["win"])
    assert out.tolist() == case["out"]


@pytest.mark.parametrize("case", KAT["precompute_py"])
def test_precompute_kat(case):
    out = ob.precompute(np.array(case["grid"]), case["win"])
    assert out.tolist() == case["out"]


def test_bayes_kat():
    L = ob.lib()
    for s in KAT["bayes_py"]:
        v = 0.0
        for o, want in zip(s["obs"], s["values"]):
            v = L.orc_bayes_update(v, s["p_hit"] if o == "h" else s["p_miss"])
            assert v == want
    for h in KAT["bayes_hand"]:
        assert L.orc_bayes_update(h["v"], h["p"]) == h["out"]


def test_pose_algebra_kat():
    L = ob.lib()
    for c in KAT["pose_py"]:
        r = L.orc_compound(ob.Pose(*c["s"]), ob.Pose(*c["d"]))
        assert (r.x, r.y, r.theta) == tuple(c["compound"])
        r = L.orc_move_backward(ob.Pose(*c["s"]), ob.Pose(*c["d"]))
        assert (r.x, r.y, r.theta) == tuple(c["move_backward"])


@pytest.mark.parametrize("i", range(len(KAT["rtcsm_py"])))
def test_rtcsm_search_kat(i):
    c = KAT["rtcsm_py"][i]
    grid = np.array(c["grid"])
    g = ob.OGrid(grid, 0.0, 0.0, c["res"])
    cg = ob.OGrid(ob.precompute(grid, c["low_res"]), 0.0, 0.0, c["res"])
    sc = ob.OScan(c["ranges"], c["angles"])
    prm = ob.RtcsmParams(c["low_res"], *c["range"], c["scan_range_max"])
    out = ob.Summary()
    cost = ob.CostGE(0.01, 20.0, 0.075, 0.1, 1, 0.05, 1.0)
    ob.lib().orc_rtcsm_optimize_pose(C.byref(g.g), C.byref(cg.g), C.byref(prm), C.byref(cost), C.byref(sc.s),
                                     ob.Pose(*c["sensor"]), c["nthr"], C.byref(out))
    assert bool(out.pose_found) == c["found"]
    assert out.score_max == c["score"]
    assert list(out.best_win) == c["best"]
    assert list(out.win) == c["win"]
    assert out.steps[2] == c["step_t"]


@pytest.mark.parametrize("i", range(len(KAT["bb_py"])))
def test_bb_search_kat(i):
    """ScanMatcherBranchBound: best node, score and the number of nodes the
    LIFO search visits, against the pure-Python restatement."""
    c = KAT["bb_py"][i]
    grid = np.array(c["grid"])
    H = c["node_height_max"]
    pyr = ob.precompute_pyramid(grid, H)
    keep = [ob.OGrid(m, 0.0, 0.0, c["res"]) for m in pyr]
    maps = (ob.Grid * (H + 1))(*[k.g for k in keep])
    g = ob.OGrid(grid, 0.0, 0.0, c["res"])
    sc = ob.OScan(c["ranges"], c["angles"])
    prm = ob.BBParams(H, *c["range"], c["scan_range_max"], *c["usable"])
    out = ob.Summary()
    cost = ob.CostGE(0.01, 20.0, 0.075, 0.1, 1, 0.05, 1.0)
    ob.lib().orc_bb_optimize_pose(C.byref(g.g), maps, C.byref(prm), C.byref(cost), C.byref(sc.s),
                                  ob.Pose(*c["sensor"]), c["nthr"], C.byref(out))
    assert bool(out.pose_found) == c["found"]
    assert out.score_max == c["score"]
    assert list(out.best_win) == c["best"]
    assert list(out.win) == c["win"]
    assert out.steps[2] == c["step_t"]
    assert out.coarse_evals == c["visited"]


@pytest.mark.parametrize("i", range(len(KAT["interp_py"])))
def test_scan_interpolate_kat(i):
    """ScanInterpolator::Interpolate against the pure-Python restatement (bit-exact)."""
    c = KAT["interp_py"][i]
    r, a = ob.scan_interpolate(c["ranges"], c["angles"], c["dist_scans"], c["dist_empty"])
    assert r.tolist() == c["out_ranges"]
    assert a.tolist() == c["out_angles"]


def test_pyramid_is_precompute_per_height():
    rng = np.random.default_rng(3)
    grid = rng.choice([0.0, 0.0, 0.3, 0.8], size=(37, 50)) * rng.uniform(0.5, 1.0, size=(37, 50))
    pyr = ob.precompute_pyramid(grid, 5)
    for h, m in enumerate(pyr):
        assert np.array_equal(m, ob.precompute(grid, 1 << h))


def _small_scene(seed, n=64, w=80):
    rng = np.random.default_rng(seed)
    grid = np.zeros((w, w))
    k = rng.integers(0, w * w, size=w * w // 6)
    grid.reshape(-1)[k] = rng.choice([0.45, 0.3, 0.6, 0.8, 0.999, 0.02], size=len(k))
    ranges = rng.uniform(0.3, 1.5, size=n)
    angles = -np.pi + np.arange(n) * (2 * np.pi / n)
    return grid, ranges, angles


@pytest.mark.parametrize("seed", range(6))
def test_pruned_search_equals_dense_first_argmax(seed):
    """SURVEY §0 finding 3, checked on the restatement: when no coarse read
    falls left/below the map, the reference's pruned loop returns the first
    maximum of the dense fine scores in (t, x, y) order."""
    grid, ranges, angles = _small_scene(seed)
    res = 0.05
    g = ob.OGrid(grid, -2.0, -2.0, res)
    cg = ob.OGrid(ob.precompute(grid, 5), -2.0, -2.0, res)
    sc = ob.OScan(ranges, angles)
    prm = ob.RtcsmParams(5, 0.6, 0.6, 0.3, 20.0)
    init = ob.Pose(0.1, -0.05, 0.2)
    dims = (C.c_int * 7)()
    ob.lib().orc_rtcsm_dense_scores(C.byref(g.g), C.byref(cg.g), C.byref(prm), C.byref(sc.s), init, None, None,
                                    dims)
    wx, wy, wt, ncx, ncy, nfx, nfy = list(dims)
    T = 2 * wt + 1
    fine = np.zeros((T, nfx, nfy))
    coarse = np.zeros((T, ncx, ncy))
    ob.lib().orc_rtcsm_dense_scores(C.byref(g.g), C.byref(cg.g), C.byref(prm), C.byref(sc.s), init,
                                    ob.dp(coarse), ob.dp(fine), dims)
    out = ob.Summary()
    cost = ob.CostGE(0.01, 20.0, 0.075, 0.1, 1, 0.05, 1.0)
    ob.lib().orc_rtcsm_optimize_pose(C.byref(g.g), C.byref(cg.g), C.byref(prm), C.byref(cost), C.byref(sc.s),
                                     init, DBL_MIN, C.byref(out))
    # dense order (t, xc, yc, xf, yf): reorder fine scores block-wise
    best = None
    for t in range(T):
        for jx in range(ncx):
            for jy in range(ncy):
                blk = fine[t, jx * 5:(jx + 1) * 5, jy * 5:(jy + 1) * 5]
                m = blk.max()
                if best is None or m > best[0]:
                    xo, yo = np.argwhere(blk == m)[0]  # row-major = x outer, y inner
                    best = (m, t - wt, -wx + jx * 5 + xo, -wy + jy * 5 + yo)
    assert out.score_max == best[0]
    assert list(out.best_win) == [best[2], best[3], best[1]]
    # coarse bound property
    for t in range(T):
        for jx in range(ncx):
            for jy in range(ncy):
                assert coarse[t, jx, jy] >= fine[t, jx * 5:(jx + 1) * 5, jy * 5:(jy + 1) * 5].max()


def test_patch_index_negative_quirk():
    """GridCellIndexToPatchIndex (H/grid_map/grid_map.hpp:905-915): exact negative
    multiples map one patch too low, so Resize allocates one extra patch."""
    m = ob.OMap(0.05, 64, 0, 0)
    assert m.geometry()["w"] == 0
    # cell -192 = -3 * 64 -> patch -4 (not -3)
    ob.lib().orc_map_resize(C.byref(m.m), -192 * 0.05, 0.0, 0.01, 0.01)
    g = m.geometry()
    assert g["npx"] == 5 and abs(g["min_x"] - (-256 * 0.05)) < 1e-12


def test_map_init_geometry():
    m = ob.OMap(0.05, 100, 1000, 1000)
    assert m.geometry() == dict(w=1000, h=1000, min_x=-25.0, min_y=-25.0, npx=10, npy=10)
    m = ob.OMap(0.05, 64, 1000, 1000)
    g = m.geometry()
    assert g["w"] == 1024 and abs(g["min_x"] + 25.6) < 1e-12


def test_integrate_scan_counts(world):
    from lgs_amd import scene
    ang = scene.beam_angles(181)
    pose = (0.3, -0.2, 0.4)
    r = scene.ray_cast(world, pose, ang)
    m = ob.OMap(0.05, 100, 600, 600)
    bp = ob.BuilderParams(0.01, 20.0, 0.6, 0.45)
    m.integrate(pose, ob.OScan(r, ang), bp)
    hits = m.hits()
    valid = ((r > 0.01) & (r < 20.0)).sum()
    assert hits.sum() == valid
    cells = m.cells()
    assert ((cells > 0) == ((hits + m.misses()) > 0)).all()
    assert cells.max() <= 0.999 and cells[cells > 0].min() >= 1e-3


def test_construct_map_from_scans_topright_quirk():
    """topRight starts at numeric_limits<double>::min() (C/mapping/grid_map_builder.cpp:236-237):
    with every point at negative x/y the map still reaches x = y = 0."""
    ang = np.linspace(np.pi, 1.5 * np.pi, 9)
    r = np.full(9, 1.0)
    m = ob.OMap(0.05, 16, 0, 0)
    bp = ob.BuilderParams(0.01, 20.0, 0.6, 0.45)
    m.construct([(-3.0, -3.0, 0.0)], [ob.OScan(r, ang)], bp)
    g = m.geometry()
    assert g["min_x"] + g["w"] * 0.05 > 0.0 and g["min_y"] + g["h"] * 0.05 > 0.0


def test_linsolve_converges(world):
    from lgs_amd import scene
    ang = scene.beam_angles(361)
    m = ob.OMap(0.05, 100, 600, 600)
    bp = ob.BuilderParams(0.01, 20.0, 0.6, 0.45)
    for p in scene.arc_poses(6):
        m.integrate(p, ob.OScan(scene.ray_cast(world, p, ang), ang), bp)
    g = ob.OGrid(m.cells(), m.m.min_x, m.m.min_y, 0.05)
    true = (1.0, 0.2, 1.7)
    sc = ob.OScan(scene.ray_cast(world, true, ang), ang)
    lp = ob.LinsolveParams(20, 0.0, 0.01, 20.0, 1e-3, 1e-3, 0.01, 20.0)
    out = ob.Summary()
    traj = (ob.Pose * 20)()
    ob.lib().orc_linsolve_optimize_pose(C.byref(g.g), C.byref(lp), C.byref(sc.s), ob.Pose(1.03, 0.18, 1.71),
                                        C.byref(out), traj)
    e = out.estimated_pose
    assert abs(e.x - true[0]) < 0.03 and abs(e.y - true[1]) < 0.03 and abs(e.theta - true[2]) < 0.02
    assert out.best_win[0] == 20


def test_colpiv_qr_solves():
    rng = np.random.default_rng(3)
    for _ in range(50):
        A = rng.normal(size=(3, 3))
        H = A @ A.T + 1e-3 * np.eye(3)
        b = rng.normal(size=3)
        x = np.zeros(3)
        ob.lib().orc_solve3_colpiv_qr(ob.dp(np.ascontiguousarray(H)), ob.dp(b), ob.dp(x))
        assert np.allclose(H @ x, b, rtol=1e-9, atol=1e-9)


# ---- round-2 known answers (tests/golden/kat_ext.py) ----

def _ogrid(c):
    return ob.OGrid(np.array(c["grid"], dtype=np.float64), c["min"][0], c["min"][1], c["res"])


def _oscan(c, rel=(0.0, 0.0, 0.0)):
    return ob.OScan(c["ranges"], c["angles"], rel, c["scan_range"][0], c["scan_range"][1])


@pytest.mark.parametrize("i", range(len(KAT["cost_ge_py"])))
def test_cost_greedy_endpoint_kat(i):
    """CostGreedyEndpoint Cost / ComputeCovariance (cost_function_greedy_endpoint.cpp:32-171)
    in both constructor argument orders (the launcher's swap, slam_launcher.cpp:68-71):
    bit-exact (same glibc exp, same summation order)."""
    c = KAT["cost_ge_py"][i]
    g, s = _ogrid(c), _oscan(c)
    cp = ob.CostGE(*c["params"])
    assert ob.lib().orc_cost_ge_cost(C.byref(g.g), C.byref(cp), C.byref(s.s), ob.Pose(*c["pose"])) == c["cost"]
    cov = np.zeros(9)
    ob.lib().orc_cost_ge_covariance(C.byref(g.g), C.byref(cp), C.byref(s.s), ob.Pose(*c["pose"]), ob.dp(cov))
    assert cov.tolist() == c["cov"]


def test_cost_greedy_endpoint_orders_differ():
    """the swapped order really is a different cost (scale 0.05, sigma 1.0)"""
    pairs = [KAT["cost_ge_py"][k:k + 2] for k in range(0, len(KAT["cost_ge_py"]), 2)]
    assert all(a["order"] == "json" and b["order"] == "launcher" for a, b in pairs)
    assert any(a["cost"] != b["cost"] for a, b in pairs)


@pytest.mark.parametrize("i", range(len(KAT["sq_py"])))
def test_square_error_and_step_kat(i):
    """CostSquareError bicubic value / cost / covariance and one LinearSolver
    OptimizeStep with the column-pivoting QR (cost_function_square_error.cpp:20-346,
    scan_matcher_linear_solver.cpp:88-148).  Eigen's inner summation order is not
    restated, so the bar is a relative 1e-12."""
    c = KAT["sq_py"][i]
    g, s = _ogrid(c), _oscan(c)
    L = ob.lib()
    for (x, y), want in zip(c["points"], c["smoothed"]):
        assert L.orc_sq_smoothed_value(C.byref(g.g), x, y) == pytest.approx(want, rel=1e-12, abs=1e-15)
    um, uM = c["usable"]
    pose = ob.Pose(*c["pose"])
    assert L.orc_sq_cost(C.byref(g.g), um, uM, C.byref(s.s), pose) == pytest.approx(c["cost"], rel=1e-12)
    cov = np.zeros(9)
    L.orc_sq_covariance(C.byref(g.g), um, uM, C.byref(s.s), pose, ob.dp(cov))
    assert np.allclose(cov, c["cov"], rtol=1e-12, atol=1e-14)
    lp = ob.LinsolveParams(1, 0.0, um, uM, c["reg"][0], c["reg"][1], um, uM)
    st = L.orc_linsolve_step(C.byref(g.g), C.byref(lp), C.byref(s.s), pose)
    assert np.allclose([st.x, st.y, st.theta], c["step"], rtol=1e-12, atol=1e-14)


def test_colpiv_qr_kat():
    for c in KAT["colpiv_qr_py"]:
        x = np.zeros(3)
        ob.lib().orc_solve3_colpiv_qr(ob.dp(np.array(c["H"])), ob.dp(np.array(c["b"])), ob.dp(x))
        assert np.allclose(x, c["x"], rtol=1e-12, atol=1e-14)


def _geo(m):
    g = m.geometry()
    return dict(w=g["w"], h=g["h"], min_x=g["min_x"], min_y=g["min_y"], npx=g["npx"], npy=g["npy"])


@pytest.mark.parametrize("i", range(len(KAT["geometry_py"])))
def test_grid_geometry_kat(i):
    """GridMap constructor / Resize / Expand / patch index (grid_map.hpp:337-391,
    652-736, 905-915): every state bit-exact."""
    c = KAT["geometry_py"][i]
    res, ps, ncx, ncy, cx, cy = c["init"]
    m = ob.OMap(res, ps, ncx, ncy, (cx, cy))
    assert _geo(m) == c["init_state"]
    for op, want in zip(c["ops"], c["states"]):
        if op[0] == "resize":
            ob.lib().orc_map_resize(C.byref(m.m), *op[1:5])
        else:
            ob.lib().orc_map_expand(C.byref(m.m), *op[1:6])
        assert _geo(m) == want, op


@pytest.mark.parametrize("i", range(len(KAT["construct_geometry_py"])))
def test_construct_map_geometry_kat(i):
    """ConstructMapFromScans' bounding box and Resize (grid_map_builder.cpp:227-290),
    incl. the DBL_MIN topRight start: the resulting geometry bit-exact."""
    c = KAT["construct_geometry_py"][i]
    res, ps, nc = c["init"]
    m = ob.OMap(res, ps, nc, nc)
    scans = [ob.OScan(n["ranges"], n["angles"], tuple(n["rel"]), *n["scan_range"]) for n in c["nodes"]]
    m.construct([tuple(n["pose"]) for n in c["nodes"]], scans, ob.BuilderParams(*c["usable"], 0.6, 0.45))
    assert _geo(m) == c["state"]


def _draw_image_py(cells, patches, ps, min_x, min_y, res, nodes, traj, lo, hi, scan, scan_pose):
    """Second restatement of MapSaver::SaveMapCore's image (C/io/map_saver.cpp:
    278-463) and GridMap::ComputeActualMapSize (H/grid_map/grid_map.hpp:969-1015)
    in plain Python, from the oracle map's cells and patch flags."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
    from make_kat import bresenham, sincos
    ys, xs = np.nonzero(patches)
    pminx, pminy, pmaxx, pmaxy = xs.min(), ys.min(), xs.max() + 1, ys.max() + 1
    gx0, gy0, gx1, gy1 = pminx * ps, pminy * ps, pmaxx * ps, pmaxy * ps
    W, H = gx1 - gx0, gy1 - gy0
    img = np.full((H, W, 3), 192, dtype=np.uint8)
    for py in range(pminy, pmaxy):
        for px in range(pminx, pmaxx):
            if not patches[py, px]:
                continue
            for yy in range(ps):
                for xx in range(ps):
                    v = cells[py * ps + yy, px * ps + xx]
                    if 0.0 < v <= 1.0:
                        img[(py - pminy) * ps + yy, (px - pminx) * ps + xx] = int((1.0 - v) * 255.0)

    def cell(x, y):
        return math.floor((x - min_x) / res), math.floor((y - min_y) / res)

    def dot(x, y, s, rgb):
        img[max(0, y):max(0, y + s), max(0, x):max(0, x + s)] = rgb

    if traj:
        prev = cell(nodes[lo][0], nodes[lo][1])
        for i in range(lo + 1, hi + 1):
            cur = cell(nodes[i][0], nodes[i][1])
            for x, y in bresenham(prev[0], prev[1], cur[0], cur[1]):
                if gx0 <= x < gx1 - 1 and gy0 <= y < gy1 - 1:
                    dot(x - gx0, y - gy0, 2, (255, 0, 0))
            prev = cur
    if scan is not None:
        r, a, rel = scan
        sx, sy = cell(scan_pose[0], scan_pose[1])
        if gx0 <= sx < gx1 - 2 and gy0 <= sy < gx1 - 2:        # :380 compares y with the x bound
            dot(sx - gx0, sy - gy0, 3, (0, 255, 0))
        s, c = sincos(scan_pose[2])
        sp = (scan_pose[0] + c * rel[0] - s * rel[1], scan_pose[1] + s * rel[0] + c * rel[1], scan_pose[2] + rel[2])
        for ri, ai in zip(r, a):
            s, c = sincos(sp[2] + ai)
            x, y = cell(sp[0] + ri * c, sp[1] + ri * s)
            if gx0 <= x < gx1 - 1 and gy0 <= y < gy1 - 1:
                dot(x - gx0, y - gy0, 2, (0, 0, 255))
    return img[::-1], [pminx, pminy, pmaxx, pmaxy, gx0, gy0, gx1, gy1, pmaxx - pminx, pmaxy - pminy, W, H]


@pytest.mark.parametrize("overlay", [0, 1, 2])
def test_map_saver_image_restatement(world, overlay):
    """orc_map_draw_image / orc_map_actual_size vs the Python restatement;
    the oracle's patch flags (set by Update, moved by Resize) equal the
    patches holding an updated cell for a map that was never reset."""
    from lgs_amd import scene
    ang = scene.beam_angles(91)
    poses = [(0.2 * k - 0.8, 0.15 * k, 0.3 * k) for k in range(8)]
    m = ob.OMap(0.05, 16, 0, 0, center=poses[0][:2])
    bp = ob.BuilderParams(0.01, 20.0, 0.6, 0.45)
    for p in poses:
        m.integrate(p, ob.OScan(scene.ray_cast(world, p, ang), ang), bp)
    g = m.geometry()
    touched = (m.hits() + m.misses()) > 0
    per_patch = touched.reshape(g["npy"], 16, g["npx"], 16).any(axis=(1, 3))
    assert np.array_equal(m.patches().astype(bool), per_patch)
    assert not per_patch.all()
    scan, oscan, sp = None, None, poses[3]
    if overlay == 2:
        r = scene.ray_cast(world, sp, ang)
        scan = (r, ang, (0.05, 0.0, 0.1))
        oscan = ob.OScan(r, ang, rel=(0.05, 0.0, 0.1))
    got = m.draw_image(poses, draw_trajectory=overlay >= 1, node_min=1, node_max=6, scan=oscan, scan_pose=sp)
    want, size = _draw_image_py(m.cells(), m.patches(), 16, g["min_x"], g["min_y"], 0.05, poses, overlay >= 1, 1,
                                6, scan, sp)
    assert m.actual_size() == (int(per_patch.sum()), size)
    assert np.array_equal(got, want)
