"""The oracle pinned against the REFERENCE ITSELF (CPU, no GPU).

oracle/_ref/libref_pin.so is built by oracle/ref/Makefile from the parts of
/root/reference that compile in this image without any stand-in header (the
reference's own headers and .cpp files, compiled in place with its -O3 and no
-march; see oracle/ref/ref_pin.cpp for the list).  Every comparison below is
bit-exact on seeded inputs, including the inputs where a fused glibc sincos()
differs from separate sin()/cos() -- which pins the oracle's (and the HIP host
code's) "GCC fuses the pair" rule to the reference binary itself.

Skips when the library is absent (the GPU box has no /root/reference)."""
import ctypes as C
import math
import os

import numpy as np
import pytest

import oracle_bind as ob

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_SO = os.path.join(ROOT, "oracle", "_ref", "libref_pin.so")
_D = C.POINTER(C.c_double)

pytestmark = pytest.mark.skipif(not os.path.exists(REF_SO), reason="oracle/_ref not built (no /root/reference)")


@pytest.fixture(scope="module")
def ref():
    L = C.CDLL(REF_SO)
    for f in ("ref_compound", "ref_inverse_compound", "ref_move_backward"):
        getattr(L, f).argtypes = [_D, _D, _D]
    L.ref_hit_points.argtypes = [_D, _D, C.c_int, _D, _D]
    L.ref_hit_and_missed_points.argtypes = [_D, _D, C.c_int, _D, C.c_double, _D]
    L.ref_bayes_sequence.argtypes = [_D, C.c_int, _D]
    L.ref_score_pixel_accurate.argtypes = [_D, C.c_int, C.c_int, C.c_double, C.c_double, C.c_double, _D, _D,
                                           C.c_int, C.c_double, C.c_double, C.c_double, C.c_double, _D, _D]
    L.ref_loss.restype = C.c_int
    L.ref_loss.argtypes = [C.c_int, C.c_double, _D, C.c_int, _D]
    L.ref_carmen_load.restype = C.c_longlong
    L.ref_carmen_load.argtypes = [C.c_char_p, _D, C.c_longlong, C.c_char_p, C.c_longlong, C.POINTER(C.c_int)]
    return L


def dp(a):
    return np.ascontiguousarray(a, dtype=np.float64).ctypes.data_as(_D)


def arr3(p):
    return np.array(p, dtype=np.float64)


def _sincos_disagree(n, rng):
    """angles where glibc sincos(x) != (sin(x), cos(x)) -- the rows where the
    fused-pair rule decides the bits"""
    lib = C.CDLL("libm.so.6")
    lib.sincos.argtypes = [C.c_double, _D, _D]
    lib.sin.restype = lib.cos.restype = C.c_double
    lib.sin.argtypes = lib.cos.argtypes = [C.c_double]
    out = []
    s, c = C.c_double(), C.c_double()
    while len(out) < n:
        x = rng.uniform(-8.0, 8.0)
        lib.sincos(x, C.byref(s), C.byref(c))
        if s.value != lib.sin(x) or c.value != lib.cos(x):
            out.append(x)
    return np.array(out)


def test_pose_algebra_bit_exact(ref):
    """H/pose.hpp Compound / InverseCompound / MoveBackward vs orc_*."""
    rng = np.random.default_rng(1)
    L = ob.lib()
    thetas = np.concatenate([rng.uniform(-7, 7, 3000), _sincos_disagree(200, rng)])
    out = np.zeros(3)
    for th in thetas:
        s = (rng.uniform(-50, 50), rng.uniform(-50, 50), th)
        d = (rng.uniform(-2, 2), rng.uniform(-2, 2), rng.uniform(-1, 1))
        for name in ("compound", "inverse_compound", "move_backward"):
            getattr(ref, "ref_" + name)(dp(arr3(s)), dp(arr3(d)), dp(out))
            o = getattr(L, "orc_" + name)(ob.Pose(*s), ob.Pose(*d))
            assert (o.x, o.y, o.theta) == tuple(out), (name, s, d)


def test_hit_points_and_cells_bit_exact(ref):
    """ScanData::HitPoint (H/sensor/sensor_data.hpp:162-173) -> the cells
    orc_rtcsm_scan_indices computes (ComputeScanIndices :178-203), including
    sensor angles where sincos and sin/cos disagree."""
    rng = np.random.default_rng(2)
    n = 1081
    ang = -2.356194490192345 + np.arange(n) * (4.71238898038469 / (n - 1))
    bad = _sincos_disagree(64, rng)
    cells = np.zeros((50, 60))
    g = ob.OGrid(cells, -12.5, -11.0, 0.05)
    xy = np.zeros(2 * n)
    idx = (C.c_int * (2 * n))()
    for k in range(64):
        r = rng.uniform(0.05, 19.0, n)
        th = bad[k] - ang[rng.integers(n)]       # some beam lands on a disagreeing sum
        pose = (rng.uniform(-3, 3), rng.uniform(-3, 3), th)
        ref.ref_hit_points(dp(r), dp(ang), n, dp(arr3(pose)), dp(xy))
        m = ob.lib().orc_rtcsm_scan_indices(C.byref(g.g), ob.Pose(*pose), C.byref(ob.OScan(r, ang).s), 20.0, idx)
        assert m == n
        want = np.floor((xy.reshape(-1, 2) - [-12.5, -11.0]) / 0.05).astype(np.int64)
        got = np.array(idx[:2 * n]).reshape(-1, 2)
        assert np.array_equal(got, want), k


def test_bayes_update_sequences_bit_exact(ref):
    """BinaryBayesGridCell::Update (H/grid_map/binary_bayes_grid_cell.hpp:75-119)
    vs orc_bayes_update over random hit/miss sequences and extreme probabilities."""
    rng = np.random.default_rng(3)
    for case in range(300):
        n = int(rng.integers(1, 200))
        ph, pm = [(0.6, 0.45), (0.9, 0.1), (0.51, 0.49), (1.0, 0.0), (0.7, 0.3)][case % 5]
        probs = np.where(rng.random(n) < rng.random(), ph, pm)
        if case % 7 == 0:
            probs = rng.uniform(-0.5, 1.5, n)   # out-of-range inputs exercise the clamps
        want = np.zeros(n)
        ref.ref_bayes_sequence(dp(probs), n, dp(want))
        v, got = 0.0, []
        for p in probs:
            v = ob.lib().orc_bayes_update(v, float(p))
            got.append(v)
        assert np.array_equal(np.array(got), want), case


def test_score_pixel_accurate_bit_exact(ref):
    """ScorePixelAccurate::Score (C/mapping/score_function_pixel_accurate.cpp:20-77,
    the branch-and-bound matcher's node score) vs orc_pixel_accurate_score."""
    rng = np.random.default_rng(4)
    out = np.zeros(3)
    for k in range(200):
        h, w = int(rng.integers(20, 90)), int(rng.integers(20, 90))
        cells = np.where(rng.random((h, w)) < 0.3, rng.choice([0.3, 0.6, 0.999, 0.001], (h, w)), 0.0)
        mx, my, res = rng.uniform(-3, 0), rng.uniform(-3, 0), [0.05, 0.1, 0.025][k % 3]
        n = int(rng.integers(1, 400))
        r = rng.uniform(0.0, 6.0, n)
        r[rng.integers(0, n, max(1, n // 10))] = rng.choice([0.0, 0.01, 20.0, 30.0])
        a = np.sort(rng.uniform(-np.pi, np.pi, n))
        pose = (rng.uniform(-1, 1), rng.uniform(-1, 1), rng.uniform(-4, 4))
        smin, smax, umin, umax = [(0.0, 30.0, 0.01, 20.0), (0.05, 5.0, 0.01, 20.0), (0.0, 30.0, 0.5, 4.0)][k % 3]
        ref.ref_score_pixel_accurate(dp(cells), w, h, mx, my, res, dp(r), dp(a), n, smin, smax, umin, umax,
                                     dp(arr3(pose)), dp(out))
        g = ob.OGrid(cells, mx, my, res)
        bp = ob.BBParams(1, 0.1, 0.1, 0.1, 20.0, umin, umax)
        got = ob.lib().orc_pixel_accurate_score(C.byref(g.g), C.byref(bp),
                                                C.byref(ob.OScan(r, a, min_range=smin, max_range=smax).s),
                                                ob.Pose(*pose))
        assert got == out[0], k


def _loss_py(kind, s, t):
    """restatement of C/mapping/robust_loss_function.cpp (the LM optimizer's weights)"""
    if kind == 0:
        return (t if t <= s else 2.0 * math.sqrt(s * t) - s), (1.0 if t <= s else math.sqrt(s / t))
    if kind == 1:
        return s * math.log1p(t / s), s / (s + t)
    if kind == 2:
        e = math.sqrt(t / s)
        return 2.0 * s * (e - math.log1p(e)), 1.0 / (1.0 + e)
    if kind == 3:
        return s * t / (s + t), (s * s) / ((s + t) * (s + t))
    if kind == 4:
        return s * (-math.expm1(-t / s)), math.exp(-t / s)
    if kind == 5:
        return s * t / (s + t), (1.0 if t <= s else math.pow(2.0 * s / (t + s), 2.0))
    return t, 1.0


def test_robust_loss_functions(ref):
    """the six robust losses + LossSquared: the host pose-graph optimizer's
    restatement (lgs_amd/posegraph.py uses these formulas) vs the reference"""
    rng = np.random.default_rng(5)
    t = np.concatenate([[0.0, 1e-12, 0.5, 1.0, 2.0], rng.exponential(3.0, 500)])
    out = np.zeros(2 * len(t))
    for kind in range(7):
        for s in (0.1, 1.0, 5.0):
            assert ref.ref_loss(kind, s, dp(t), len(t), dp(out)) == 0
            for i, x in enumerate(t):
                lo, we = _loss_py(kind, s, float(x))
                assert out[2 * i] == pytest.approx(lo, rel=1e-15, abs=0.0), (kind, s, x)
                assert out[2 * i + 1] == pytest.approx(we, rel=1e-15, abs=0.0), (kind, s, x)
