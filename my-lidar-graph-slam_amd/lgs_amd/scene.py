"""Synthetic 2-D LiDAR scenes for tests and bench.py.

World: a 24 m x 24 m walled room centred at the origin with 40 random
axis-aligned boxes (seed 42, sides 0.2-2.2 m) kept clear of the central
4 m x 4 m area where sensor poses live, so every beam of a pose within 1.5 m
of the centre is < 20 m (nothing is dropped by ScanRangeMax).

Scans: N beams, angles -135 deg + i * 270/(N-1) deg, ranges from an exact
analytic ray cast (capped at 30 m).
"""
from __future__ import annotations

import numpy as np

ROOM_HALF = 12.0


def make_world(seed: int = 42, n_boxes: int = 40, room_half: float = ROOM_HALF, clear: float = 2.0):
    """Return segments (S, 4) = [x0, y0, x1, y1] of the room walls and box edges."""
    rng = np.random.default_rng(seed)
    segs = [
        (-room_half, -room_half, room_half, -room_half),
        (room_half, -room_half, room_half, room_half),
        (room_half, room_half, -room_half, room_half),
        (-room_half, room_half, -room_half, -room_half),
    ]
    boxes = []
    while len(boxes) < n_boxes:
        w, h = rng.uniform(0.2, 2.2, size=2)
        cx, cy = rng.uniform(-room_half + 1.2, room_half - 1.2, size=2)
        x0, x1, y0, y1 = cx - w / 2, cx + w / 2, cy - h / 2, cy + h / 2
        if x1 > -clear and x0 < clear and y1 > -clear and y0 < clear:
            continue
        boxes.append((x0, y0, x1, y1))
        segs += [(x0, y0, x1, y0), (x1, y0, x1, y1), (x1, y1, x0, y1), (x0, y1, x0, y0)]
    return np.array(segs, dtype=np.float64)


def beam_angles(n: int = 1081, fov_deg: float = 270.0) -> np.ndarray:
    start = -np.deg2rad(fov_deg / 2.0)
    return start + np.arange(n, dtype=np.float64) * (np.deg2rad(fov_deg) / (n - 1))


def ray_cast(segs: np.ndarray, pose, angles: np.ndarray, max_range: float = 30.0) -> np.ndarray:
    """Exact distance along each beam from the sensor pose to the nearest segment."""
    x, y, th = pose
    d = np.stack([np.cos(th + angles), np.sin(th + angles)], axis=1)  # (N, 2)
    p = segs[:, :2]
    q = segs[:, 2:] - segs[:, :2]  # (S, 2)
    # o + t d = p + u q  ->  t = cross(p - o, q) / cross(d, q), u = cross(p - o, d) / cross(d, q)
    po = p - np.array([x, y])
    den = d[:, None, 0] * q[None, :, 1] - d[:, None, 1] * q[None, :, 0]  # (N, S)
    tnum = po[None, :, 0] * q[None, :, 1] - po[None, :, 1] * q[None, :, 0]
    unum = po[None, :, 0] * d[:, None, 1] - po[None, :, 1] * d[:, None, 0]
    with np.errstate(divide="ignore", invalid="ignore"):
        t = tnum / den
        u = unum / den
    ok = (np.abs(den) > 1e-12) & (t > 1e-9) & (u >= 0.0) & (u <= 1.0)
    t = np.where(ok, t, np.inf)
    r = t.min(axis=1)
    return np.minimum(r, max_range)


def arc_poses(n: int = 10, spacing: float = 0.4, radius: float = 1.0, center=(0.0, 0.0)):
    """Poses on a circular arc, `spacing` metres apart, heading along the arc."""
    cx, cy = center
    dphi = spacing / radius
    phis = -0.5 * dphi * (n - 1) + dphi * np.arange(n)
    return [(cx + radius * np.cos(p), cy + radius * np.sin(p), p + np.pi / 2) for p in phis]


def map_geometry(n_cells: int = 1000, patch_size: int = 100, res: float = 0.05, center=(0.0, 0.0)):
    """GridMap(res, ps, n, n, center) geometry (H/grid_map/grid_map.hpp:337-391)."""
    npatch = int(np.ceil(n_cells / patch_size))
    w = npatch * patch_size
    off = (w // 2) if w % 2 == 0 else (w // 2 + 0.5)
    return w, w, center[0] - off * res, center[1] - off * res


def approx_occupancy_map(segs, poses, angles, w, h, min_x, min_y, res, p_hit=0.6, p_miss=0.45,
                         usable_max=20.0):
    """Fast numpy occupancy map for benchmark inputs (not a parity artefact):
    free cells along each ray sampled at res/2, hit cells at the end point,
    values combined with the binary Bayes rule in odds space."""
    lo = np.zeros((h, w))
    seen = np.zeros((h, w), dtype=bool)
    l_hit = np.log(p_hit / (1 - p_hit))
    l_miss = np.log(p_miss / (1 - p_miss))
    for pose in poses:
        r = ray_cast(segs, pose, angles)
        keep = r < usable_max
        x, y, th = pose
        for rr, aa in zip(r[keep], angles[keep]):
            ts = np.arange(0.0, rr, res * 0.5)
            px = x + ts * np.cos(th + aa)
            py = y + ts * np.sin(th + aa)
            ix = np.floor((px - min_x) / res).astype(np.int64)
            iy = np.floor((py - min_y) / res).astype(np.int64)
            cells = np.unique(iy * w + ix)
            hx = int(np.floor((x + rr * np.cos(th + aa) - min_x) / res))
            hy = int(np.floor((y + rr * np.sin(th + aa) - min_y) / res))
            cells = cells[cells != hy * w + hx]
            flat = lo.reshape(-1)
            sflat = seen.reshape(-1)
            flat[cells] += l_miss
            sflat[cells] = True
            flat[hy * w + hx] += l_hit
            sflat[hy * w + hx] = True
    p = 1.0 / (1.0 + np.exp(-lo))
    p = np.clip(p, 1e-3, 1 - 1e-3)
    return np.where(seen, p, 0.0)


def loop_problem(segs, build_map, n_maps: int = 32, nodes_per_map: int = 16, n_beams: int = 1081,
                 seed: int = 5, perturb=(2.0, 0.4), arc_scans: int = 10, map_beams: int = 1081):
    """Config-5 style loop-closure batch: `n_maps` local maps, each built by
    `build_map(poses, angles) -> (cells, min_x, min_y, res)` from `arc_scans`
    scans on an arc around its own centre, and `nodes_per_map` candidate
    nodes per map whose scans are taken near that centre and whose initial
    poses are the true poses perturbed by U(+-perturb[0] m, +-perturb[1] rad).
    Returns (maps, candidates) as lgs_amd.loopbatch.LocalMap / Candidate lists
    (candidates query-major)."""
    from .loopbatch import Candidate, LocalMap
    rng = np.random.default_rng(seed)
    ang = beam_angles(n_beams)
    mang = beam_angles(map_beams)
    maps, cands = [], []
    node = 0
    for q in range(n_maps):
        c = (rng.uniform(-1.5, 1.5), rng.uniform(-1.5, 1.5))
        poses = arc_poses(arc_scans, center=c)
        cells, mx, my, res = build_map(poses, mang)
        maps.append(LocalMap(cells, mx, my, res, poses[0], node))
        node += arc_scans
        for _ in range(nodes_per_map):
            true = (c[0] + rng.uniform(-1.0, 1.0), c[1] + rng.uniform(-1.0, 1.0), rng.uniform(-np.pi, np.pi))
            r = ray_cast(segs, true, ang)
            init = (true[0] + rng.uniform(-perturb[0], perturb[0]), true[1] + rng.uniform(-perturb[0], perturb[0]),
                    true[2] + rng.uniform(-perturb[1], perturb[1]))
            cands.append(Candidate(q, r, ang, init, node))
            node += 1
    return maps, cands
