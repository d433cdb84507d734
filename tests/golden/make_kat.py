"""Generate tests/golden/kat.json: known-answer vectors for the oracle.

The reference (Forrest-Z/my-lidar-graph-slam) ships no tests, fixtures or
golden data, and it cannot be built here without a stand-in for Eigen (see
DESIGN.md §Oracle), so these vectors are NOT reference outputs.  They come from
two sources independent of oracle/lgs_oracle.c:

  * "hand" cases: traced by hand through the reference source text (the trace
    is recorded next to each case);
  * "py" cases: a second, pure-Python restatement of the same reference
    functions below (Python floats are IEEE binary64 without FMA contraction and
    math.exp/acos and the ctypes-bound glibc sincos() below are glibc's, like
    the reference's build: GCC -O3 fuses each sin(x)/cos(x) pair of the
    reference into one sincos() call, which differs from separate sin/cos in
    ~0.1% of inputs, so paired sites here call sincos()).

Agreement of the C oracle with both pins the oracle against restatement bugs;
it does not pin it to the reference binary ("parity unpinned").

Run:  python tests/golden/make_kat.py   (rewrites kat.json deterministically)
"""
from __future__ import annotations

import ctypes
import ctypes.util
import json
import math
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
if HERE not in sys.path:
    sys.path.insert(0, HERE)

_libm = ctypes.CDLL(ctypes.util.find_library("m"))
_libm.sincos.restype = None
_libm.sincos.argtypes = [ctypes.c_double, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double)]


def sincos(x):
    """glibc sincos(x) -> (sin, cos)."""
    sn, cs = ctypes.c_double(), ctypes.c_double()
    _libm.sincos(x, ctypes.byref(sn), ctypes.byref(cs))
    return sn.value, cs.value


# ---------------- pure-Python restatement (small cases only) ----------------

def bresenham(x0, y0, x1, y1):
    """H/util.hpp:256-303 (C++ int semantics: deltaX / 2 truncates toward 0;
    deltaX is non-negative here so // is identical)."""
    pts = []
    dx, dy = x1 - x0, y1 - y0
    sx = -1 if dx < 0 else 1
    sy = -1 if dy < 0 else 1
    nx, ny = x0, y0
    dx, dy = abs(dx * 2), abs(dy * 2)
    pts.append((nx, ny))
    if dx > dy:
        err = dy - dx // 2
        while nx != x1:
            if err >= 0:
                ny += sy
                err -= dx
            nx += sx
            err += dy
            pts.append((nx, ny))
    else:
        err = dx - dy // 2
        while ny != y1:
            if err >= 0:
                nx += sx
                err -= dy
            ny += sy
            err += dx
            pts.append((nx, ny))
    return pts


def sliding_window_max(vals, win):
    """H/util.hpp:198-253 with inFunc returning 0.0 past the end."""
    n = len(vals)
    inf = lambda i: vals[i] if i < n else 0.0
    out = [None] * n
    q = []
    idx_in = 0
    idx_out = 0
    while idx_in < win:
        while q and inf(idx_in) >= inf(q[-1]):
            q.pop()
        q.append(idx_in)
        idx_in += 1
    while idx_in < n:
        out[idx_out] = inf(q[0])
        idx_out += 1
        while q and q[0] <= idx_in - win:
            q.pop(0)
        while q and inf(idx_in) >= inf(q[-1]):
            q.pop()
        q.append(idx_in)
        idx_in += 1
    while idx_out < n:
        out[idx_out] = inf(q[0])
        idx_out += 1
    return out


def precompute(grid, win):
    """C/mapping/grid_map_builder.cpp:518-536 (row pass along y, then x)."""
    h, w = len(grid), len(grid[0])
    tmp = [[0.0] * w for _ in range(h)]
    for x in range(w):
        col = sliding_window_max([grid[y][x] for y in range(h)], win)
        for y in range(h):
            tmp[y][x] = col[y]
    out = [[0.0] * w for _ in range(h)]
    for y in range(h):
        out[y] = sliding_window_max(tmp[y], win)
    return out


PMIN = 1e-3
PMAX = 1.0 - PMIN


def clamp(v, lo, hi):
    return lo if v < lo else (hi if hi < v else v)


def bayes(v, p):
    """H/grid_map/binary_bayes_grid_cell.hpp:75-119"""
    if v == 0.0:
        return clamp(p, PMIN, PMAX)
    co = clamp(v, PMIN, PMAX)
    cp = clamp(p, PMIN, PMAX)
    o = (co / (1.0 - co)) * (cp / (1.0 - cp))
    return clamp(clamp(o / (1.0 + o), PMIN, PMAX), PMIN, PMAX)


def compound(s, d):
    st, ct = sincos(s[2])
    return (ct * d[0] - st * d[1] + s[0], st * d[0] + ct * d[1] + s[1], s[2] + d[2])


def move_backward(e, d):
    th = e[2] - d[2]
    st, ct = sincos(th)
    return (e[0] - ct * d[0] + st * d[1], e[1] - st * d[0] - ct * d[1], th)


def gval(grid, x, y):
    h, w = len(grid), len(grid[0])
    return grid[y][x] if (0 <= x < w and 0 <= y < h) else 0.0


def rtcsm_search(grid, coarse, min_x, min_y, res, ranges, angles, sensor, low_res, rx, ry, rt,
                 rmax, nthr):
    """C/mapping/scan_matcher_real_time_correlative.cpp:50-125 (search part)."""
    mr = ranges[0]
    for r in ranges[1:]:
        if mr < r:
            mr = r
    max_range = rmax if rmax < mr else mr
    theta = res / max_range
    step_t = math.acos(1.0 - 0.5 * theta * theta)
    wx = int(math.ceil(0.5 * rx / res))
    wy = int(math.ceil(0.5 * ry / res))
    wt = int(math.ceil(0.5 * rt / step_t))
    thr = nthr * len(ranges)
    smax = thr
    best = [-wx, -wy, -wt]
    for t in range(-wt, wt + 1):
        th = sensor[2] + step_t * t
        idx = []
        for r, a in zip(ranges, angles):
            if r >= rmax:
                continue
            sn, cs = sincos(th + a)
            hx = sensor[0] + r * cs
            hy = sensor[1] + r * sn
            idx.append((int(math.floor((hx - min_x) / res)), int(math.floor((hy - min_y) / res))))
        for x in range(-wx, wx + 1, low_res):
            for y in range(-wy, wy + 1, low_res):
                s = 0.0
                for ix, iy in idx:
                    s += gval(coarse, ix + x, iy + y)
                if s <= smax:
                    continue
                for xf in range(x, x + low_res):
                    for yf in range(y, y + low_res):
                        s = 0.0
                        for ix, iy in idx:
                            s += gval(grid, ix + xf, iy + yf)
                        if smax < s:
                            smax = s
                            best = [xf, yf, t]
    return dict(found=smax > thr, score=smax, best=best, win=[wx, wy, wt], step_t=step_t)


def pixel_accurate_score(grid, min_x, min_y, res, ranges, angles, pose, umin, umax, smin, smax):
    """C/mapping/score_function_pixel_accurate.cpp:19-77"""
    min_range = umin if smin < umin else smin      # std::max
    max_range = smax if smax < umax else umax      # std::min
    s = 0.0
    for r, a in zip(ranges, angles):
        if r >= max_range or r <= min_range:
            continue
        sn, cs = sincos(pose[2] + a)
        hx = pose[0] + r * cs
        hy = pose[1] + r * sn
        v = gval(grid, int(math.floor((hx - min_x) / res)), int(math.floor((hy - min_y) / res)))
        if v == 0.0:
            continue
        s += v
    return s


def bb_search(grid, min_x, min_y, res, ranges, angles, sensor, H, rx, ry, rt, rmax, nthr, umin, umax):
    """C/mapping/scan_matcher_branch_bound.cpp:47-140 (search part) with the
    PrecomputeGridMaps pyramid (C/mapping/grid_map_builder.cpp:471-495)."""
    pyr = [precompute(grid, 1 << h) for h in range(H + 1)]
    mr = ranges[0]
    for r in ranges[1:]:
        if mr < r:
            mr = r
    max_range = rmax if rmax < mr else mr
    theta = res / max_range
    step_t = math.acos(1.0 - 0.5 * theta * theta)
    wx = int(math.ceil(0.5 * rx / res))
    wy = int(math.ceil(0.5 * ry / res))
    wt = int(math.ceil(0.5 * rt / step_t))
    thr = nthr * len(ranges)
    smax = thr
    best = [0, 0, 0]
    stack = []
    ws_max = 1 << H
    for x in range(-wx, wx + 1, ws_max):
        for y in range(-wy, wy + 1, ws_max):
            for t in range(-wt, wt + 1):
                stack.append((x, y, t, H))
    visited = 0
    while stack:
        x, y, t, h = stack.pop()
        pose = (sensor[0] + x * res, sensor[1] + y * res, sensor[2] + t * step_t)
        sc = pixel_accurate_score(pyr[h], min_x, min_y, res, ranges, angles, pose, umin, umax, 0.0, 30.0)
        visited += 1
        if sc <= smax:
            continue
        if h == 0:
            smax = sc
            best = [x, y, t]
            continue
        w = 1 << (h - 1)
        stack += [(x, y, t, h - 1), (x + w, y, t, h - 1), (x, y + w, t, h - 1), (x + w, y + w, t, h - 1)]
    return dict(found=smax > thr, score=smax, best=best, win=[wx, wy, wt], step_t=step_t, visited=visited)


def scan_interpolate(ranges, angles, dist_scans, dist_empty):
    """ScanInterpolator::Interpolate (C/mapping/scan_interpolator.cpp:9-98):
    ToCartesianCoordinate (H/util.hpp:148-152, a sin/cos pair -> sincos),
    Distance (H/point.hpp:113-117), ToPolarCoordinate (H/util.hpp:156-161)."""
    pts = []
    for r, a in zip(ranges, angles):
        sn, cs = sincos(a)
        pts.append((r * cs, r * sn))
    out = [pts[0]]
    prev = pts[0]
    acc = 0.0
    i = 1
    while i < len(ranges):
        p = pts[i]
        d = math.sqrt((prev[0] - p[0]) * (prev[0] - p[0]) + (prev[1] - p[1]) * (prev[1] - p[1]))
        if acc + d < dist_scans:
            acc += d
            prev = p
        elif acc + d >= dist_empty:
            out.append(p)
            prev = p
            acc = 0.0
        else:
            ratio = (dist_scans - acc) / d
            q = ((p[0] - prev[0]) * ratio + prev[0], (p[1] - prev[1]) * ratio + prev[1])
            out.append(q)
            prev = q
            acc = 0.0
            continue            # process point i again
        i += 1
    return ([math.sqrt(x * x + y * y) for x, y in out], [math.atan2(y, x) for x, y in out])


def main():
    rnd = random.Random(1234)
    kat = {"_note": __doc__.strip().splitlines()[0]}

    # Bresenham: hand-traced cases + Python restatement over all octants
    kat["bresenham_hand"] = [
        {"args": [0, 0, 5, 2], "pts": [[0, 0], [1, 0], [2, 1], [3, 1], [4, 2], [5, 2]],
         "trace": "dX=10 dY=4 err=4-5=-1; x-major; y steps when err>=0 at x=2 and x=4"},
        {"args": [0, 0, 0, 0], "pts": [[0, 0]], "trace": "zero-length ray: start cell only"},
        {"args": [0, 0, -3, 3], "pts": [[0, 0], [-1, 1], [-2, 2], [-3, 3]],
         "trace": "|2dx|==|2dy| -> y-major branch, err=6-3=3 >=0 every step"},
        {"args": [2, 3, 2, -1], "pts": [[2, 3], [2, 2], [2, 1], [2, 0], [2, -1]],
         "trace": "vertical, stepY=-1, dX=0 -> err=0-4=-4 never >=0 after err+=0"},
    ]
    cases = []
    for _ in range(200):
        a = [rnd.randint(-30, 30) for _ in range(4)]
        cases.append({"args": a, "pts": [list(p) for p in bresenham(*a)]})
    kat["bresenham_py"] = cases

    # SlidingWindowMax
    kat["swm_hand"] = [
        {"in": [1.0, 3.0, 2.0, 0.0, 5.0], "win": 2, "out": [3.0, 3.0, 2.0, 5.0, 5.0],
         "trace": "out[i]=max(in[i],in[i+1]) for i<=3; tail repeats max(in[3..4])"},
        {"in": [1.0, 2.0], "win": 3, "out": [2.0, 2.0], "trace": "n<win: one window incl. 0.0 past end"},
        {"in": [-1.0, -2.0], "win": 3, "out": [0.0, 0.0], "trace": "past-end reads are Unknown=0.0"},
        {"in": [4.0, 1.0, 1.0, 1.0], "win": 1, "out": [4.0, 1.0, 1.0, 1.0], "trace": "win=1 identity"},
    ]
    sw = []
    for _ in range(100):
        n = rnd.randint(1, 40)
        win = rnd.randint(1, 12)
        vals = [rnd.choice([0.0, 0.0, 0.45, 0.6, rnd.random()]) for _ in range(n)]
        sw.append({"in": vals, "win": win, "out": sliding_window_max(vals, win)})
    kat["swm_py"] = sw

    # PrecomputeGridMap on small grids (odd/even sizes, w < win)
    pc = []
    for (h, w, win) in [(7, 9, 3), (8, 8, 5), (3, 4, 5), (1, 1, 2), (10, 6, 1), (12, 13, 4)]:
        grid = [[rnd.choice([0.0, 0.0, 0.0, 0.3, 0.7, rnd.random()]) for _ in range(w)] for _ in range(h)]
        pc.append({"grid": grid, "win": win, "out": precompute(grid, win)})
    kat["precompute_py"] = pc

    # Bayes update sequences (first-hit assignment, clamps, saturation)
    seqs = []
    for seq in (["h"], ["m"], ["h", "h", "h"], ["m"] * 40, ["h"] * 20 + ["m"] * 3,
                ["m", "h", "m", "h", "m"], [rnd.choice("hm") for _ in range(60)]):
        v = 0.0
        vals = []
        for o in seq:
            v = bayes(v, 0.6 if o == "h" else 0.45)
            vals.append(v)
        seqs.append({"obs": "".join(seq), "p_hit": 0.6, "p_miss": 0.45, "values": vals})
    kat["bayes_py"] = seqs
    kat["bayes_hand"] = [
        {"v": 0.0, "p": 0.6, "out": 0.6, "trace": "unknown cell: ClampValue(0.6)"},
        {"v": 0.0, "p": 1.0, "out": 0.999, "trace": "clamped to 1-1e-3"},
        {"v": 0.001, "p": 0.45, "out": 0.001, "trace": "odds product below pmin -> clamp to 1e-3 (fixed point)"},
    ]

    # pose algebra
    pa = []
    for _ in range(50):
        s = (rnd.uniform(-10, 10), rnd.uniform(-10, 10), rnd.uniform(-4, 4))
        d = (rnd.uniform(-1, 1), rnd.uniform(-1, 1), rnd.uniform(-1, 1))
        pa.append({"s": s, "d": d, "compound": compound(s, d), "move_backward": move_backward(s, d)})
    kat["pose_py"] = pa

    # tiny correlative searches (pure-Python pruned loop)
    rs = []
    for case in range(6):
        w = h = 24
        grid = [[0.0] * w for _ in range(h)]
        for _ in range(80):
            grid[rnd.randrange(h)][rnd.randrange(w)] = rnd.choice([0.6, 0.8, 0.999, 0.45, 0.01])
        if case == 3:
            grid = [[0.5] * w for _ in range(h)]        # forced ties
        if case == 4:
            grid = [[0.0] * w for _ in range(h)]        # empty map -> corner pose
        lr = 3
        coarse = precompute(grid, lr)
        n = 24
        ranges = [rnd.uniform(0.1, 0.5) for _ in range(n)]
        if case == 5:
            ranges[3] = 30.0                             # beam >= ScanRangeMax is skipped
        angles = [-math.pi + i * (2 * math.pi / n) for i in range(n)]
        sensor = (0.61, 0.59, 0.1 * case)
        res = 0.05
        out = rtcsm_search(grid, coarse, 0.0, 0.0, res, ranges, angles, sensor, lr, 0.3, 0.2, 0.4,
                           20.0, 2.2250738585072014e-308 if case != 2 else 0.3)
        rs.append({"grid": grid, "low_res": lr, "ranges": ranges, "angles": angles, "sensor": sensor,
                   "res": res, "range": [0.3, 0.2, 0.4], "scan_range_max": 20.0,
                   "nthr": 2.2250738585072014e-308 if case != 2 else 0.3, **out})
    kat["rtcsm_py"] = rs

    # tiny branch-and-bound searches (pure-Python LIFO search)
    bb = []
    for case in range(5):
        w = h = 20
        grid = [[0.0] * w for _ in range(h)]
        for _ in range(60):
            grid[rnd.randrange(h)][rnd.randrange(w)] = rnd.choice([0.6, 0.8, 0.999, 0.45, 0.01])
        if case == 3:
            grid = [[0.5] * w for _ in range(h)]        # ties everywhere
        n = 16
        ranges = [rnd.uniform(0.1, 0.45) for _ in range(n)]
        if case == 4:
            ranges[2] = 0.005                            # below the usable range: skipped
        angles = [-math.pi + i * (2 * math.pi / n) for i in range(n)]
        sensor = (0.52, 0.49, 0.2 * case)
        H = 2 if case != 1 else 3
        nthr = 2.2250738585072014e-308 if case != 2 else 0.4
        out = bb_search(grid, 0.0, 0.0, 0.05, ranges, angles, sensor, H, 0.3, 0.2, 0.3, 20.0, nthr, 0.01, 20.0)
        bb.append({"grid": grid, "node_height_max": H, "ranges": ranges, "angles": angles, "sensor": sensor,
                   "res": 0.05, "range": [0.3, 0.2, 0.3], "scan_range_max": 20.0, "nthr": nthr,
                   "usable": [0.01, 20.0], **out})
    kat["bb_py"] = bb

    # ScanInterpolator (DistScans / DistThresholdEmpty of the launcher JSON and others)
    si = []
    for case in range(8):
        n = [1, 2, 37, 181, 361, 90, 50, 120][case]
        a0, a1 = -math.pi / 2 * (1 + 0.5 * (case % 2)), math.pi / 2 * (1 + 0.5 * (case % 2))
        angles = [a0 + (a1 - a0) * k / max(1, n - 1) for k in range(n)]
        ranges = []
        for k in range(n):
            base = 1.0 + 0.8 * math.sin(0.05 * k * (case + 1))
            ranges.append(base if rnd.random() > 0.1 else base * rnd.uniform(1.5, 4.0))   # gaps
        if case == 6:
            ranges = [0.5] * n                           # equal-range arc: spacing below DistScans
        ds, de = [(0.05, 0.25), (0.05, 0.25), (0.05, 0.25), (0.05, 0.25), (0.1, 0.3), (0.02, 0.5),
                  (0.05, 0.25), (0.03, 0.06)][case]
        rr, aa = scan_interpolate(ranges, angles, ds, de)
        si.append({"ranges": ranges, "angles": angles, "dist_scans": ds, "dist_empty": de,
                   "out_ranges": rr, "out_angles": aa})
    kat["interp_py"] = si

    import kat_ext                  # round-2 restatements (cost, refine, geometry)
    kat_ext.extend(kat, rnd)

    with open(os.path.join(HERE, "kat.json"), "w") as f:
        json.dump(kat, f, indent=None, separators=(",", ":"))
    print("wrote", os.path.join(HERE, "kat.json"))


if __name__ == "__main__":
    main()
