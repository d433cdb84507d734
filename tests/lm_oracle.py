"""CPU restatement of PoseGraphOptimizerLM (test infrastructure only).

Follows C/mapping/pose_graph_optimizer_lm.cpp line by line with dense numpy
linear algebra: Optimize (:13-65), OptimizeStep (:68-220; the SparseCholesky
solve becomes numpy.linalg.solve, the ConjugateGradient solve Eigen's
Jacobi-preconditioned CG recurrence, Eigen/src/IterativeLinearSolvers/
ConjugateGradient.h, default tolerance = machine epsilon, 2 * cols
iterations), ComputeErrorJacobians (:224-280), ComputeErrorFunction
(:283-299), ComputeTotalError (:302-338), and the robust losses of
C/mapping/robust_loss_function.cpp (pinned against the reference itself in
tests/test_ref_pin.py).  Pose algebra uses glibc's fused sincos like the
reference binary (tests/oracle_bind.py pins that rule).
"""
import ctypes as C
import math

import numpy as np

_libm = C.CDLL("libm.so.6")
_libm.sincos.argtypes = [C.c_double, C.POINTER(C.c_double), C.POINTER(C.c_double)]


def sincos(x):
    s, c = C.c_double(), C.c_double()
    _libm.sincos(x, C.byref(s), C.byref(c))
    return s.value, c.value


def normalize_angle(t):
    """H/util.hpp:125-135"""
    r = math.fmod(t, 2.0 * math.pi)
    if r > math.pi:
        r -= 2.0 * math.pi
    elif r < -math.pi:
        r += 2.0 * math.pi
    return r


def loss_fn(kind, s):
    """(Loss, Weight) of C/mapping/robust_loss_function.cpp"""
    if kind == 0:
        return (lambda t: t if t <= s else 2.0 * math.sqrt(s * t) - s), \
               (lambda t: 1.0 if t <= s else math.sqrt(s / t))
    if kind == 1:
        return (lambda t: s * math.log1p(t / s)), (lambda t: s / (s + t))
    if kind == 2:
        return (lambda t: 2.0 * s * (math.sqrt(t / s) - math.log1p(math.sqrt(t / s)))), \
               (lambda t: 1.0 / (1.0 + math.sqrt(t / s)))
    if kind == 3:
        return (lambda t: s * t / (s + t)), (lambda t: (s * s) / ((s + t) * (s + t)))
    if kind == 4:
        return (lambda t: s * (-math.expm1(-t / s))), (lambda t: math.exp(-t / s))
    if kind == 5:
        return (lambda t: s * t / (s + t)), (lambda t: 1.0 if t <= s else math.pow(2.0 * s / (t + s), 2.0))
    return (lambda t: t), (lambda t: 1.0)


def error(sp, ep, z):
    """ComputeErrorFunction: InverseCompound(start, end) - z, angle normalised"""
    st, ct = sincos(sp[2])
    dx, dy = ep[0] - sp[0], ep[1] - sp[1]
    rel = (ct * dx + st * dy, -st * dx + ct * dy, ep[2] - sp[2])
    return np.array([rel[0] - z[0], rel[1] - z[1], normalize_angle(rel[2] - z[2])])


def total_error(poses, edges, loss):
    tot = 0.0
    for s, e, z, info in edges:
        ev = error(poses[s], poses[e], z)
        tot += loss(float(ev @ np.asarray(info) @ ev))
    return tot


def cg(A, b):
    n = len(b)
    x = np.zeros(n)
    d = np.diag(A)
    inv = np.where(d != 0.0, 1.0 / np.where(d != 0.0, d, 1.0), 1.0)
    tol = np.finfo(float).eps
    rhs2 = b @ b
    if rhs2 == 0.0:
        return x
    thr = max(tol * tol * rhs2, np.finfo(float).tiny)
    r = b.copy()
    if r @ r < thr:
        return x
    p = inv * r
    abs_new = r @ p
    for _ in range(2 * n):
        t = A @ p
        alpha = abs_new / (p @ t)
        x += alpha * p
        r -= alpha * t
        if r @ r < thr:
            break
        z = inv * r
        abs_old, abs_new = abs_new, r @ z
        p = z + (abs_new / abs_old) * p
    return x


def optimize(poses, edges, solver=0, iters=10, tol=1e-3, lam=1e-4, loss_kind=0, scale=1.0):
    """PoseGraphOptimizerLM::Optimize -> (poses [n, 3], iterations, total error, lambda after)"""
    loss, weight = loss_fn(loss_kind, scale)
    P = np.array(poses, dtype=np.float64).copy()
    n = len(P)
    prev = total = np.finfo(float).max
    it = 0
    while True:
        H = np.zeros((3 * n, 3 * n))
        b = np.zeros(3 * n)
        for s, e, z, info in edges:
            info = np.asarray(info, dtype=np.float64)
            sp, ep = P[s], P[e]
            dx, dy = ep[0] - sp[0], ep[1] - sp[1]
            st, ct = sincos(sp[2])
            Js = np.array([[-ct, -st, -st * dx + ct * dy], [st, -ct, -ct * dx - st * dy], [0.0, 0.0, -1.0]])
            Je = np.array([[ct, st, 0.0], [-st, ct, 0.0], [0.0, 0.0, 1.0]])
            ev = error(sp, ep, z)
            W = weight(float(ev @ info @ ev)) * info
            JsW, JeW = Js.T @ W, Je.T @ W
            H[3 * s:3 * s + 3, 3 * s:3 * s + 3] += JsW @ Js
            H[3 * e:3 * e + 3, 3 * e:3 * e + 3] += JeW @ Je
            H[3 * s:3 * s + 3, 3 * e:3 * e + 3] += JsW @ Je
            H[3 * e:3 * e + 3, 3 * s:3 * s + 3] += (JsW @ Je).T
            b[3 * s:3 * s + 3] += JsW @ ev
            b[3 * e:3 * e + 3] += JeW @ ev
        for i in range(3):
            H[i, i] += 1e9
        H[np.diag_indices(3 * n)] += lam
        delta = np.linalg.solve(H, -b) if solver == 0 else cg(H, -b)
        P += delta.reshape(n, 3)
        total = total_error(P, edges, loss)
        it += 1
        if it >= iters or abs(prev - total) < tol:
            break
        lam = lam * 0.5 if total < prev else lam * 2.0
        prev = total
    return P, it, total, lam


def random_graph(n, loops, rng, noise=0.05, outliers=0):
    """A noisy odometry chain of n nodes plus `loops` loop edges (and some
    outlier loop edges) over a ground-truth closed trajectory."""
    t = np.linspace(0.0, 2.0 * np.pi, n, endpoint=False)
    truth = np.stack([5.0 * np.cos(t), 3.0 * np.sin(t), t + np.pi / 2.0], axis=1)

    def rel(a, b):
        st, ct = sincos(a[2])
        dx, dy = b[0] - a[0], b[1] - a[1]
        return (ct * dx + st * dy, -st * dx + ct * dy, normalize_angle(b[2] - a[2]))

    info = np.diag([100.0, 100.0, 400.0])
    edges = []
    for i in range(n - 1):
        z = np.array(rel(truth[i], truth[i + 1])) + rng.normal(0.0, [0.01, 0.01, 0.005])
        edges.append((i, i + 1, tuple(z), info))
    for _ in range(loops):
        i, j = sorted(rng.choice(n, 2, replace=False))
        edges.append((int(j), int(i), rel(truth[j], truth[i]), info * 2.0))
    for _ in range(outliers):
        i, j = sorted(rng.choice(n, 2, replace=False))
        edges.append((int(j), int(i), tuple(rng.uniform(-2, 2, 3)), info))
    # initial guess: dead reckoning with drift
    init = [truth[0].copy()]
    for i in range(n - 1):
        z = np.array(edges[i][2]) + rng.normal(0.0, [noise, noise, noise / 5])
        st, ct = sincos(init[-1][2])
        p = init[-1]
        init.append(np.array([p[0] + ct * z[0] - st * z[1], p[1] + st * z[0] + ct * z[1], p[2] + z[2]]))
    return np.array(init), edges
