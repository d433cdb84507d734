"""f4 host components on the CPU: the Carmen log reader
pinned to the REFERENCE's own CarmenLogReader (committed vectors from
oracle/_ref, tests/golden/make_carmen_golden.py; live comparison when the
reference library is built here), the robust losses pinned to the reference
(tests/test_ref_pin.py builds the same library), PoseGraphOptimizerLM vs a
numpy restatement of C/mapping/pose_graph_optimizer_lm.cpp (tests/lm_oracle.py,
both linear solvers, every loss), the pose-graph JSON layout and the PNG
encoder."""
import ctypes as C
import json
import os

import numpy as np
import pytest

import lm_oracle as lo
from lgs_amd import io

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden", "carmen_ref.json")
REF_SO = os.path.join(ROOT, "oracle", "_ref", "libref_pin.so")


def bits(a):
    return np.ascontiguousarray(a, dtype=np.float64).view(np.uint64)


def test_carmen_reader_matches_reference_vectors():
    """every record, id and field bit-exact with the reference reader's
    output on the committed texts (malformed, truncated and empty lines)"""
    g = json.load(open(GOLDEN))
    assert len(g["cases"]) >= 3
    for c in g["cases"]:
        stream, ids, n = io.carmen_load(c["text"])
        want = np.array([float.fromhex(x) for x in c["stream"]])
        assert n == c["records"]
        assert ids == c["ids"]
        assert np.array_equal(bits(stream), bits(want))


@pytest.mark.skipif(not os.path.exists(REF_SO), reason="oracle/_ref not built (no /root/reference)")
def test_carmen_reader_matches_reference_live():
    """fresh random logs through both readers"""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    import make_carmen_golden as mk
    L = mk.load_ref_lib()
    for seed in range(5):
        for text in mk.carmen_texts(seed):
            s1, i1, n1 = mk.ref_load(L, text)
            s2, i2, n2 = io.carmen_load(text)
            assert (n1, i1) == (n2, i2)
            assert np.array_equal(bits(s1), bits(s2))


def test_carmen_ids_byte_count():
    """lgs_carmen_load reports the bytes the sensor ids need (terminators
    included), so a caller sizes the ids buffer exactly; a short buffer gets
    a prefix and the same count."""
    import ctypes as C
    text = "ODOM 1 2 3 4 5 6 7.5 host 8\n" * 40 + "ROBOTLASER1 0 -1 2 0.25 30 0.1 0 2 4 5 0 0 0.1 2 1 0.2 0 0 0 0 0 11.5 h 12\n"
    L = io.load()
    n, nid = C.c_int(), C.c_longlong()
    need = L.lgs_carmen_load(text.encode(), None, 0, None, 0, C.byref(nid), C.byref(n))
    assert need > 0 and n.value == 41 and nid.value == 40 * len("ODOM\0") + len("ROBOTLASER1\0")
    small = C.create_string_buffer(7)
    nid2 = C.c_longlong()
    L.lgs_carmen_load(text.encode(), None, 0, small, 7, C.byref(nid2), None)
    assert nid2.value == nid.value and small.raw == b"ODOM\0OD"
    _, ids, _ = io.carmen_load(text)
    assert ids == ["ODOM"] * 40 + ["ROBOTLASER1"]


def test_carmen_record_layout():
    """a hand-written log: what each record type carries"""
    text = ("PARAM Laser.AngleIncrement 0.5\n"
            "ODOM 1 2 3 4 5 6 7.5 host 8\n"
            "FLASER 3 1 2 3 0.5 0 0 1 0 0 9.5 host 10\n"
            "ROBOTLASER1 0 -1 2 0.25 30 0.1 0 2 4 5 0 0 0.1 2 1 0.2 0 0 0 0 0 11.5 h 12\n")
    s, ids, n = io.carmen_load(text)
    assert n == 3 and ids == ["ODOM", "FLASER", "ROBOTLASER1"]
    assert list(s[:8]) == [0, 7.5, 1, 2, 3, 4, 0, 5]   # odometry: timestamp, pose, velocity (tv, 0, rv)
    f = s[8:8 + 16 + 6]
    assert f[0] == 1 and f[1] == 9.5 and f[2] == 3
    assert list(f[3:6]) == [1, 0, 0]                      # odometry pose = robot pose
    assert f[12] == 0.0 and f[13] == 80.0                 # default min/max range
    assert f[14] == -np.pi / 2 and f[15] == -np.pi / 2 + 0.5 * 3   # MinAngle default, + increment * n
    assert list(f[16:19]) == [-np.pi / 2, -np.pi / 2 + 0.5, -np.pi / 2 + 1.0]
    assert list(f[19:22]) == [1, 2, 3]
    r = s[8 + 22:]
    assert r[2] == 2 and r[13] == 30.0 and r[14] == -1 and r[15] == -1 + 0.25
    assert list(r[16 + 2:16 + 4]) == [4, 5]


def _loss_py(kind, s, t):
    lo_, we = lo.loss_fn(kind, s)
    return lo_(t), we(t)


def test_robust_losses():
    t = np.concatenate([[0.0, 1e-12, 0.5, 1.0, 2.0], np.random.default_rng(5).exponential(3.0, 400)])
    for kind in range(7):
        for s in (0.1, 1.0, 5.0):
            loss, weight = io.robust_loss(kind, s, t)
            for i, x in enumerate(t):
                a, b = _loss_py(kind, s, float(x))
                assert loss[i] == pytest.approx(a, rel=1e-15, abs=0.0)
                assert weight[i] == pytest.approx(b, rel=1e-15, abs=0.0)


@pytest.mark.skipif(not os.path.exists(REF_SO), reason="oracle/_ref not built (no /root/reference)")
def test_robust_losses_bit_exact_vs_reference():
    L = C.CDLL(REF_SO)
    L.ref_loss.restype = C.c_int
    L.ref_loss.argtypes = [C.c_int, C.c_double, C.POINTER(C.c_double), C.c_int, C.POINTER(C.c_double)]
    t = np.concatenate([[0.0, 1e-12, 0.5, 1.0, 2.0], np.random.default_rng(6).exponential(3.0, 1000)])
    out = np.zeros(2 * len(t))
    for kind in range(7):
        for s in (0.1, 1.0, 5.0):
            assert L.ref_loss(kind, s, t.ctypes.data_as(C.POINTER(C.c_double)), len(t),
                              out.ctypes.data_as(C.POINTER(C.c_double))) == 0
            loss, weight = io.robust_loss(kind, s, t)
            assert np.array_equal(bits(loss), bits(out[0::2])), kind
            assert np.array_equal(bits(weight), bits(out[1::2])), kind


@pytest.mark.parametrize("solver", [io.LM_SPARSE_CHOLESKY, io.LM_CONJUGATE_GRADIENT])
@pytest.mark.parametrize("kind,scale", [(0, 1.0), (1, 0.5), (2, 2.0), (3, 1.0), (4, 3.0), (5, 2.0), (6, 1.0)])
def test_lm_matches_restatement(solver, kind, scale):
    """poses, iteration count, final total error and the damping factor after
    the call, against the dense numpy restatement (tolerance 1e-9: the
    restatement solves densely, the product a block sparse Cholesky or the
    same CG recurrence, so roundings differ)"""
    rng = np.random.default_rng(100 + kind + 10 * solver)
    init, edges = lo.random_graph(80, 12, rng, outliers=2)
    P, it, tot, lam = io.optimize_lm(init, edges, solver=solver, iters=10, tol=1e-6, lam=1e-3, loss=kind,
                                     scale=scale)
    Q, it2, tot2, lam2 = lo.optimize(init, edges, solver, 10, 1e-6, 1e-3, kind, scale)
    assert it == it2 and lam == lam2
    assert tot == pytest.approx(tot2, rel=1e-9)
    assert np.abs(P - Q).max() <= 1e-9


def test_lm_anchors_node_zero_and_closes_loops():
    """the 1e9 diagonal keeps node 0 in place; loop edges pull the drifted
    dead-reckoning chain back (total error drops by orders of magnitude)"""
    rng = np.random.default_rng(7)
    init, edges = lo.random_graph(300, 40, rng, noise=0.05)
    before = lo.total_error(init, edges, lambda t: t)
    P, it, tot, _ = io.optimize_lm(init, edges, iters=20, tol=1e-9, lam=1e-4, loss="squared")
    assert np.abs(P[0] - init[0]).max() < 1e-6
    assert tot < before * 1e-2


def test_lm_large_sparse_graph():
    """a 5000-node graph: the block sparse factorisation stays sparse (the
    dense restatement would need a 15000^2 matrix); cross-checked against the
    CG solver's fixed point"""
    rng = np.random.default_rng(8)
    init, edges = lo.random_graph(5000, 200, rng, noise=0.01)
    P, it, tot, _ = io.optimize_lm(init, edges, iters=6, tol=1e-12, lam=1e-4, loss="huber", scale=1.0)
    assert it == 6 and np.isfinite(P).all()
    P2, _, tot2, _ = io.optimize_lm(P, edges, iters=1, tol=0.0, lam=1e-12, loss="huber", scale=1.0)
    assert tot2 <= tot * (1 + 1e-6)


def test_lm_rejects_bad_input():
    with pytest.raises(RuntimeError):
        io.optimize_lm([(0, 0, 0), (1, 0, 0)], [(0, 5, (1, 0, 0), np.eye(3))])
    with pytest.raises(RuntimeError):
        io.optimize_lm([(0, 0, 0)], [], loss=42)


def test_pose_graph_json(tmp_path):
    """SavePoseGraph (C/io/map_saver.cpp:56-120) in boost write_json form:
    string values, 17 significant digits, upper-triangle information"""
    rng = np.random.default_rng(9)
    poses = rng.uniform(-5, 5, (4, 3))
    ts = [1000.125, 0.1, 2.0 / 3.0, 1e-7]
    info = np.array([[1.0, 0.5, 0.25], [0.5, 2.0, 0.125], [0.25, 0.125, 3.0]])
    edges = [(0, 1, (0.1, 0.2, 1.0 / 3.0), info), (3, 0, (-1.5, 2.0, 0.0), info * 7)]
    f = str(tmp_path / "g")
    io.save_pose_graph([0, 1, 2, 3], poses, ts, edges, f)
    text = open(f + ".posegraph.json").read()
    d = json.loads(text)
    nodes, es = d["PoseGraph"]["Nodes"], d["PoseGraph"]["Edges"]
    assert [n["Index"] for n in nodes] == ["0", "1", "2", "3"]
    for k, n in enumerate(nodes):
        assert [float(n["Pose"][c]) for c in ("X", "Y", "Theta")] == list(poses[k])
        assert float(n["TimeStamp"]) == ts[k]
    assert es[1]["StartNodeIdx"] == "3" and es[1]["EndNodeIdx"] == "0"
    assert [float(v) for v in es[0]["InformationMatrix"]] == [1.0, 0.5, 0.25, 2.0, 0.125, 3.0]
    assert float(es[0]["RelativePose"]["Theta"]) == 1.0 / 3.0
    assert '"Theta": "0.33333333333333331"' in text          # max_digits10
    assert text.startswith('{\n    "PoseGraph": {\n        "Nodes": [\n            {\n                "Index": "0",')
    assert text.endswith("}\n")


def test_png_writer_round_trip(tmp_path):
    rng = np.random.default_rng(10)
    for h, w in ((1, 1), (3, 7), (64, 100), (257, 33)):
        img = rng.integers(0, 256, (h, w, 3), dtype=np.uint8)
        f = str(tmp_path / f"i{h}x{w}.png")
        io.write_png(f, img)
        assert np.array_equal(io.read_png_rgb8(f), img)
