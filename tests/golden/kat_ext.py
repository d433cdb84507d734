"""Second, pure-Python restatements of the reference functions that
tests/golden/make_kat.py did not cover in round 1 (test infrastructure only):
CostGreedyEndpoint cost / covariance under both constructor argument orders,
CostSquareError's bicubic value / map gradient / cost / covariance, one
ScanMatcherLinearSolver::OptimizeStep with Eigen's column-pivoting Householder
QR, and the GridMap geometry (constructor, Resize, Expand, patch index,
ConstructMapFromScans bounding box).

Written from the reference source text, independently of oracle/lgs_oracle.c.
make_kat.py imports these and stores their outputs in kat.json.  Floating-point
conventions as make_kat.py (IEEE binary64, glibc sincos for paired sin/cos,
glibc pow/exp through math.pow/math.exp)."""
from __future__ import annotations

import math

from make_kat import compound, gval, sincos


# ---- CostGreedyEndpoint (C/mapping/cost_function_greedy_endpoint.cpp:32-171) ----

def ge_cost(grid, min_x, min_y, res, ranges, angles, smin, smax, pose, umin, umax, hmd, occ, ks, scaling, stddev):
    """Cost (:32-111).  pose = sensor pose; (smin, smax) = scan MinRange/MaxRange.
    (scaling, stddev) are the constructor's scalingFactor / standardDeviation
    slots (cost_function_greedy_endpoint.cpp:9-26)."""
    var = stddev * stddev
    lo, hi = max(umin, smin), min(umax, smax)
    cost = 0.0
    for r, a in zip(ranges, angles):
        if r >= hi or r <= lo:
            continue
        sn, cs = sincos(pose[2] + a)                    # HitAndMissedPoint (sensor_data.hpp:177-197)
        hx, hy = pose[0] + r * cs, pose[1] + r * sn
        mx, my = pose[0] + (r - hmd) * cs, pose[1] + (r - hmd) * sn
        hix, hiy = math.floor((hx - min_x) / res), math.floor((hy - min_y) / res)
        mix, miy = math.floor((mx - min_x) / res), math.floor((my - min_y) / res)
        d = (ks + 1) * res                              # SquaredDistance(0, 0, k+1, k+1)
        best = d * d + d * d
        for ky in range(-ks, ks + 1):
            for kx in range(-ks, ks + 1):
                hv = gval(grid, hix + kx, hiy + ky)
                mv = gval(grid, mix + kx, miy + ky)
                if hv == 0.0 or mv == 0.0:
                    continue
                if hv < occ or mv > occ:
                    continue
                dx, dy = kx * res, ky * res
                sq = dx * dx + dy * dy
                best = min(sq, best)
        cost -= math.exp(-0.5 * best / var)
    return cost * scaling


def ge_covariance(grid, min_x, min_y, res, ranges, angles, smin, smax, pose, *cp):
    """ComputeGradient + ComputeCovariance (:114-171): central differences with
    step = resolution (x, y) and 1e-2 rad, cov = g g^T + 0.01 I."""
    dl, da = res, 1e-2

    def c(p):
        return ge_cost(grid, min_x, min_y, res, ranges, angles, smin, smax, p, *cp)
    x, y, t = pose
    g = [0.5 * (c((x + dl, y, t)) - c((x - dl, y, t))) / dl,
         0.5 * (c((x, y + dl, t)) - c((x, y - dl, t))) / dl,
         0.5 * (c((x, y, t + da)) - c((x, y, t - da))) / da]
    cov = [g[i] * g[j] for i in range(3) for j in range(3)]
    cov[0] += 0.01
    cov[4] += 0.01
    cov[8] += 0.01
    return cov


# ---- CostSquareError / ScanMatcherLinearSolver (C/mapping/cost_function_square_error.cpp:20-346,
#      C/mapping/scan_matcher_linear_solver.cpp:88-148).  Eigen's summation order inside its
#      small products is not restated bit for bit: these vectors pin to a relative 1e-12. ----

def _bicubic_h(t):
    at = abs(t)
    if at <= 1.0:
        return math.pow(at, 3.0) - 2.0 * math.pow(at, 2.0) + 1.0
    if at <= 2.0:
        return -math.pow(at, 3.0) + 5.0 * math.pow(at, 2.0) - 8.0 * at + 4.0
    return 0.0


def sq_smoothed(grid, x, y):
    """ComputeSmoothedValue (:276-346): bicubic kernel over the 4x4 cells around
    the floating index, edge-clamped cell reads, result clamped to [0, 1]."""
    h, w = len(grid), len(grid[0])

    def f(a, b):
        xc = min(max(int(a), 0), w - 1)               # static_cast<int> truncates toward zero
        yc = min(max(int(b), 0), h - 1)
        return grid[yc][xc]
    fx, fy = math.floor(x), math.floor(y)
    xs = (1.0 + x - fx, x - fx, fx + 1.0 - x, fx + 2.0 - x)
    ys = (1.0 + y - fy, y - fy, fy + 1.0 - y, fy + 2.0 - y)
    px = (x - xs[0], x - xs[1], x + xs[2], x + xs[3])
    py = (y - ys[0], y - ys[1], y + ys[2], y + ys[3])
    vx = [_bicubic_h(t) for t in xs]
    vy = [_bicubic_h(t) for t in ys]
    row = [sum(vx[i] * f(px[i], py[j]) for i in range(4)) for j in range(4)]
    v = sum(row[j] * vy[j] for j in range(4))
    return min(max(v, 0.0), 1.0)


def sq_map_gradient(grid, min_x, min_y, res, pose, r, a):
    """ComputeMapGradient(pose, range, angle) (:200-226) over ComputeMapGradient(mapPos) (:172-197)."""
    sn, cs = sincos(pose[2] + a)
    hx, hy = pose[0] + r * cs, pose[1] + r * sn
    fx, fy = (hx - min_x) / res, (hy - min_y) / res
    dd = res * 0.1
    gx = (sq_smoothed(grid, fx + 0.05, fy) - sq_smoothed(grid, fx - 0.05, fy)) / dd
    gy = (sq_smoothed(grid, fx, fy + 0.05) - sq_smoothed(grid, fx, fy - 0.05)) / dd
    return (gx, gy, -r * sn * gx + r * cs * gy)


def sq_cost(grid, min_x, min_y, res, ranges, angles, smin, smax, pose, umin, umax):
    """Cost (:20-58)"""
    lo, hi = max(umin, smin), min(umax, smax)
    c = 0.0
    for r, a in zip(ranges, angles):
        if r >= hi or r <= lo:
            continue
        sn, cs = sincos(pose[2] + a)
        v = sq_smoothed(grid, (pose[0] + r * cs - min_x) / res, (pose[1] + r * sn - min_y) / res)
        c += math.pow(1.0 - v, 2.0)
    return c


def sq_covariance(grid, min_x, min_y, res, ranges, angles, smin, smax, pose, umin, umax):
    """ComputeGradient + ComputeCovariance (:61-135)"""
    lo, hi = max(umin, smin), min(umax, smax)
    g = [0.0, 0.0, 0.0]
    for r, a in zip(ranges, angles):
        if r >= hi or r <= lo:
            continue
        sn, cs = sincos(pose[2] + a)
        e = 1.0 - sq_smoothed(grid, (pose[0] + r * cs - min_x) / res, (pose[1] + r * sn - min_y) / res)
        mg = sq_map_gradient(grid, min_x, min_y, res, pose, r, a)
        for k in range(3):
            g[k] += 2.0 * e * (-mg[k])
    cov = [g[i] * g[j] for i in range(3) for j in range(3)]
    cov[0] += 0.01
    cov[4] += 0.01
    cov[8] += 0.01
    return cov


def colpiv_qr_solve(H, b):
    """Eigen::ColPivHouseholderQR<Matrix3d>::solve (Eigen 3.3 algorithm; Eigen is
    not vendored by the reference): pivot on the largest remaining column norm
    (first maximum), Householder reflector beta = -sign(c0) |x|,
    tau = (beta - c0) / beta, essential part x_tail / (c0 - beta); solve applies
    Q^T, back-substitutes R and undoes the column permutation."""
    n = 3
    A = [list(H[3 * i:3 * i + 3]) for i in range(3)]
    perm = list(range(n))
    taus, ess = [], []
    norms = [math.sqrt(sum(A[i][j] ** 2 for i in range(n))) for j in range(n)]
    for k in range(n):
        j = k
        for c in range(k + 1, n):
            if norms[c] > norms[j]:
                j = c
        if j != k:
            for i in range(n):
                A[i][k], A[i][j] = A[i][j], A[i][k]
            norms[k], norms[j] = norms[j], norms[k]
            perm[k], perm[j] = perm[j], perm[k]
        c0 = A[k][k]
        tail = [A[i][k] for i in range(k + 1, n)]
        tsq = sum(t * t for t in tail)
        if tsq <= 2.2250738585072014e-308:
            tau, beta, v = 0.0, c0, [0.0] * len(tail)
        else:
            beta = math.sqrt(c0 * c0 + tsq)
            if c0 >= 0.0:
                beta = -beta
            v = [t / (c0 - beta) for t in tail]
            tau = (beta - c0) / beta
        A[k][k] = beta
        for i in range(k + 1, n):
            A[i][k] = v[i - k - 1]
        for c in range(k + 1, n):            # I - tau [1 v][1 v]^T on the left
            tmp = A[k][c] + sum(v[i - k - 1] * A[i][c] for i in range(k + 1, n))
            A[k][c] -= tau * tmp
            for i in range(k + 1, n):
                A[i][c] -= tau * v[i - k - 1] * tmp
        for c in range(k + 1, n):
            norms[c] = math.sqrt(sum(A[i][c] ** 2 for i in range(k + 1, n)))
        taus.append(tau)
        ess.append(v)
    y = list(b)
    for k in range(n):                       # Q^T b
        v = ess[k]
        tmp = y[k] + sum(v[i - k - 1] * y[i] for i in range(k + 1, n))
        y[k] -= taus[k] * tmp
        for i in range(k + 1, n):
            y[i] -= taus[k] * v[i - k - 1] * tmp
    z = [0.0] * n
    for k in range(n - 1, -1, -1):
        z[k] = (y[k] - sum(A[k][c] * z[c] for c in range(k + 1, n))) / A[k][k]
    x = [0.0] * n
    for k in range(n):
        x[perm[k]] = z[k]
    return x


def linsolve_step(grid, min_x, min_y, res, ranges, angles, smin, smax, pose, umin, umax, treg, rreg):
    """OptimizeStep (:88-148)"""
    lo, hi = max(umin, smin), min(umax, smax)
    B = [0.0] * 3
    H = [0.0] * 9
    for r, a in zip(ranges, angles):
        if r >= hi or r <= lo:
            continue
        sn, cs = sincos(pose[2] + a)
        e = 1.0 - sq_smoothed(grid, (pose[0] + r * cs - min_x) / res, (pose[1] + r * sn - min_y) / res)
        g = sq_map_gradient(grid, min_x, min_y, res, pose, r, a)
        for i in range(3):
            B[i] += e * g[i]
            for j in range(3):
                H[3 * i + j] += g[i] * g[j]
    H[0] += treg
    H[4] += treg
    H[8] += rreg
    d = colpiv_qr_solve(H, B)
    return (pose[0] + d[0], pose[1] + d[1], pose[2] + d[2])


# ---- GridMap geometry (H/grid_map/grid_map.hpp:337-391, 652-736, 905-915) and the
#      ConstructMapFromScans bounding box (C/mapping/grid_map_builder.cpp:227-290) ----

def _ctrunc_div(a, b):
    q = abs(a) // abs(b)
    return q if (a >= 0) == (b > 0) else -q


def patch_index(idx, ps):
    """GridCellIndexToPatchIndex (:905-915): exact negative multiples land one patch low."""
    return _ctrunc_div(idx, ps) - 1 if idx < 0 else idx // ps


class Geo:
    def __init__(self, res, ps, ncx, ncy, cx=0.0, cy=0.0):
        """GridMap(res, ps, numCellsX, numCellsY, center) (:337-391)"""
        self.res, self.ps = res, ps
        self.npx = int(math.ceil(float(max(0, ncx)) / float(ps)))
        self.npy = int(math.ceil(float(max(0, ncy)) / float(ps)))
        self.ncx, self.ncy = self.npx * ps, self.npy * ps
        ox = float(self.ncx // 2) if self.ncx % 2 == 0 else self.ncx // 2 + 0.5
        oy = float(self.ncy // 2) if self.ncy % 2 == 0 else self.ncy // 2 + 0.5
        self.min_x, self.min_y = cx - ox * res, cy - oy * res

    def idx(self, x, y):
        return math.floor((x - self.min_x) / self.res), math.floor((y - self.min_y) / self.res)

    def inside(self, x, y):
        i, j = self.idx(x, y)
        return 0 <= i < self.ncx and 0 <= j < self.ncy

    def resize(self, x0, y0, x1, y1):
        """Resize (:652-711)"""
        i0, j0 = self.idx(x0, y0)
        i1, j1 = self.idx(x1, y1)
        p0x, p0y = patch_index(i0, self.ps), patch_index(j0, self.ps)
        p1x, p1y = patch_index(i1, self.ps), patch_index(j1, self.ps)
        self.npx, self.npy = max(0, p1x - p0x + 1), max(0, p1y - p0y + 1)
        self.ncx, self.ncy = self.npx * self.ps, self.npy * self.ps
        self.min_x += float(p0x * self.ps) * self.res
        self.min_y += float(p0y * self.ps) * self.res

    def expand(self, x0, y0, x1, y1, step):
        """Expand (:714-736)"""
        if self.inside(x0, y0) and self.inside(x1, y1):
            return
        mnx, mny = self.min_x + self.res * 0, self.min_y + self.res * 0
        mxx, mxy = self.min_x + self.res * self.ncx, self.min_y + self.res * self.ncy
        mnx = x0 - step if x0 < mnx else mnx
        mny = y0 - step if y0 < mny else mny
        mxx = x1 + step if x1 > mxx else mxx
        mxy = y1 + step if y1 > mxy else mxy
        self.resize(mnx, mny, mxx, mxy)

    def state(self):
        return dict(w=self.ncx, h=self.ncy, min_x=self.min_x, min_y=self.min_y, npx=self.npx, npy=self.npy)


def construct_bbox(nodes, umin, umax):
    """ConstructMapFromScans (:227-282): bounding box of the sensor poses and the
    hit points, topRight starting at numeric_limits<double>::min()."""
    bl = [1.7976931348623157e308, 1.7976931348623157e308]
    tr = [2.2250738585072014e-308, 2.2250738585072014e-308]
    for pose, rel, ranges, angles, smin, smax in nodes:
        sp = compound(pose, rel)
        bl = [min(bl[0], sp[0]), min(bl[1], sp[1])]
        tr = [max(tr[0], sp[0]), max(tr[1], sp[1])]
        lo, hi = max(umin, smin), min(umax, smax)
        for r, a in zip(ranges, angles):
            if r >= hi or r <= lo:
                continue
            sn, cs = sincos(sp[2] + a)
            hx, hy = sp[0] + r * cs, sp[1] + r * sn
            bl = [min(bl[0], hx), min(bl[1], hy)]
            tr = [max(tr[0], hx), max(tr[1], hy)]
    return bl, tr


def extend(kat, rnd):
    """Add the vectors of this module to kat (called by make_kat.main)."""
    # CostGreedyEndpoint cost / covariance in the JSON order and in the
    # launcher's swapped order (slam_launcher.cpp:68-71 passes the
    # standardDeviation setting into the scalingFactor slot and vice versa)
    ge = []
    for case in range(6):
        w = h = 28
        grid = [[0.0] * w for _ in range(h)]
        for _ in range(260):
            grid[rnd.randrange(h)][rnd.randrange(w)] = rnd.choice([0.05, 0.08, 0.2, 0.6, 0.9, 0.999, 0.001])
        n = 40
        ranges = [rnd.uniform(0.05, 0.6) for _ in range(n)]
        ranges[5] = 0.0                                  # <= minRange: skipped
        ranges[7] = 30.0                                 # >= maxRange: skipped
        angles = [-math.pi + i * (2 * math.pi / n) for i in range(n)]
        pose = (0.7 + 0.01 * case, 0.68 - 0.013 * case, 0.3 * case)
        ks = [1, 1, 2, 0, 3, 1][case]
        for order, (scaling, stddev) in (("json", (1.0, 0.05)), ("launcher", (0.05, 1.0))):
            cp = (0.01, 20.0, 0.075, 0.1, ks, scaling, stddev)
            ge.append({"grid": grid, "min": [0.0, 0.0], "res": 0.05, "ranges": ranges, "angles": angles,
                       "scan_range": [0.0, 30.0], "pose": pose, "params": cp, "order": order,
                       "cost": ge_cost(grid, 0.0, 0.0, 0.05, ranges, angles, 0.0, 30.0, pose, *cp),
                       "cov": ge_covariance(grid, 0.0, 0.0, 0.05, ranges, angles, 0.0, 30.0, pose, *cp)})
    kat["cost_ge_py"] = ge

    # bicubic value, square-error cost / covariance, one OptimizeStep
    sq = []
    for case in range(4):
        w = h = 26
        grid = [[0.0] * w for _ in range(h)]
        for _ in range(220):
            grid[rnd.randrange(h)][rnd.randrange(w)] = rnd.choice([0.3, 0.6, 0.9, 0.999, rnd.random()])
        n = 36
        ranges = [rnd.uniform(0.1, 0.55) for _ in range(n)]
        ranges[3] = 25.0
        angles = [-math.pi + i * (2 * math.pi / n) for i in range(n)]
        pose = (0.64 + 0.02 * case, 0.61, 0.4 * case - 0.3)
        pts = [(rnd.uniform(-2.5, w + 1.5), rnd.uniform(-2.5, h + 1.5)) for _ in range(30)]
        pts += [(3.0, 4.0), (0.0, 0.0), (w - 1.0, h - 1.0), (-0.5, 7.25)]
        sq.append({"grid": grid, "min": [0.0, 0.0], "res": 0.05, "ranges": ranges, "angles": angles,
                   "scan_range": [0.0, 30.0], "pose": pose, "usable": [0.01, 20.0], "reg": [0.01, 0.01],
                   "points": pts, "smoothed": [sq_smoothed(grid, x, y) for x, y in pts],
                   "cost": sq_cost(grid, 0.0, 0.0, 0.05, ranges, angles, 0.0, 30.0, pose, 0.01, 20.0),
                   "cov": sq_covariance(grid, 0.0, 0.0, 0.05, ranges, angles, 0.0, 30.0, pose, 0.01, 20.0),
                   "step": linsolve_step(grid, 0.0, 0.0, 0.05, ranges, angles, 0.0, 30.0, pose, 0.01, 20.0,
                                         0.01, 0.01)})
    kat["sq_py"] = sq

    qr = []
    for case in range(40):
        A = [[rnd.gauss(0, 1) for _ in range(3)] for _ in range(3)]
        H = [sum(A[i][k] * A[j][k] for k in range(3)) + (0.01 if i == j else 0.0)
             for i in range(3) for j in range(3)]
        if case == 0:
            H = [4.0, 0.0, 0.0, 0.0, 1.0, 0.0, 0.0, 0.0, 9.0]   # the pivots reorder every column
        b = [rnd.gauss(0, 1) for _ in range(3)]
        qr.append({"H": H, "b": b, "x": colpiv_qr_solve(H, b)})
    kat["colpiv_qr_py"] = qr

    # GridMap geometry: constructor, Resize / Expand sequences (negative patch
    # indices included) and the extra-patch quirk of exact negative multiples
    geo = []
    for case in range(12):
        res = [0.05, 0.1, 0.025][case % 3]
        ps = [64, 100, 16, 7][case % 4]
        ncx, ncy = rnd.choice([0, 1, 5, 99, 100, 640]), rnd.choice([0, 3, 64, 101])
        cx, cy = rnd.uniform(-2, 2), rnd.uniform(-2, 2)
        g = Geo(res, ps, ncx, ncy, cx, cy)
        init = g.state()
        ops, states = [], []
        for _ in range(6):
            x0, y0 = rnd.uniform(-40, 10), rnd.uniform(-40, 10)
            x1, y1 = x0 + rnd.uniform(0, 30), y0 + rnd.uniform(0, 30)
            if rnd.random() < 0.5:
                op = ["resize", x0, y0, x1, y1]
                g.resize(x0, y0, x1, y1)
            else:
                op = ["expand", x0, y0, x1, y1, rnd.choice([0.0, 1.0, 5.0])]
                g.expand(x0, y0, x1, y1, op[5])
            ops.append(op)
            states.append(g.state())
        xq = g.min_x - 3 * ps * res + 0.25 * res        # lands on cell -3 ps: patch -4
        ops.append(["resize", xq, g.min_y, xq + 1.0, g.min_y + 1.0])
        g.resize(xq, g.min_y, xq + 1.0, g.min_y + 1.0)
        states.append(g.state())
        geo.append({"init": [res, ps, ncx, ncy, cx, cy], "init_state": init, "ops": ops, "states": states})
    kat["geometry_py"] = geo

    # ConstructMapFromScans: the bounding-box Resize of a map in a given state
    cm = []
    for case in range(5):
        ps, nc = [16, 100, 64, 32, 50][case], [0, 50, 200, 0, 10][case]
        g = Geo(0.05, ps, nc, nc)
        nodes = []
        for _ in range(1 + case):
            n = 20
            ang = [-math.pi / 2 + i * math.pi / (n - 1) for i in range(n)]
            rr = [rnd.uniform(0.2, 4.0) for _ in range(n)]
            rr[2] = 0.001                                # <= UsableRangeMin: skipped
            pose = (rnd.uniform(-3, 3), rnd.uniform(-3, 3), rnd.uniform(-3, 3))
            rel = (0.1 * (case % 2), -0.05 * (case % 2), 0.02 * case)
            nodes.append((pose, rel, rr, ang, 0.0, 30.0))
        if case == 3:        # every point at negative x / y: topRight stays DBL_MIN
            nodes = [((-5.0, -5.0, 0.0), (0.0, 0.0, 0.0), [1.0] * 9,
                      [math.pi + k * (0.5 * math.pi / 8) for k in range(9)], 0.0, 30.0)]
        bl, tr = construct_bbox(nodes, 0.01, 20.0)
        g.resize(bl[0], bl[1], tr[0], tr[1])
        cm.append({"init": [0.05, ps, nc],
                   "nodes": [{"pose": p, "rel": r, "ranges": rr, "angles": aa, "scan_range": [a, b]}
                             for p, r, rr, aa, a, b in nodes],
                   "usable": [0.01, 20.0], "bbox": [bl, tr], "state": g.state()})
    kat["construct_geometry_py"] = cm
