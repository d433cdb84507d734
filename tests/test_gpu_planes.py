"""The coarse map as the matcher holds it on the device: the
padded phase planes written straight by the batched precompute
(k_precompute_planes) or by the phase-plane copy of a supplied coarse map
(k_decimate), and the fp16 superblock planes (k_super_planes), checked
element by element against the oracle's PrecomputeGridMap
(C/mapping/grid_map_builder.cpp:518-536, H/util.hpp:198-253)."""
import math

import numpy as np
import pytest

import oracle_bind as ob
from conftest import launcher_cost
from lgs_amd import abi, scene

pytestmark = pytest.mark.gpu


def layout(W, H, res, lr, rx, ry):
    wx, wy = math.ceil(0.5 * rx / res), math.ceil(0.5 * ry / res)
    ncx, ncy = 2 * wx // lr + 1, 2 * wy // lr + 1
    nsbx, nsby = (ncx + 3) // 4, (ncy + 3) // 4
    M = 4 * max(nsbx, nsby)
    Wq, Hq = -(-W // lr), -(-H // lr)
    Wqp = (Wq + 2 * M + 3) & ~3
    Hqp = Hq + 2 * M
    Wq4, Hq4 = ((-(-Wqp // 4)) + 7) & ~7, -(-Hqp // 4)
    # octet layout (k_rtcsm.hip set_plane_layout) for windows of <= 9 x 9
    # superblocks: 8-bit units (r06) of 8 rows (4q .. 4q + 7, 8 bytes) or,
    # for windows of more than 5 superblock rows, 12 rows (12 bytes)
    oct = nsbx <= 9 and nsby <= 9 and nsbx * nsby <= 64
    u8 = 3 if oct and nsby > 5 else 2
    Qo = (Hq4 + 3) // 4 + 1
    return dict(M=M, Wq=Wq, Hq=Hq, Wqp=Wqp, Hqp=Hqp, Wq4=Wq4, Hq4=Hq4, sub4=Wq4 * Hq4, oct=oct, Qo=Qo,
                subO=Qo * Wq4, u8=u8)


def half_round_up(x):
    """fp16 rounded toward +inf (k_rtcsm.hip half_round_up_bits), +0 for zeros"""
    h = x.astype(np.float16)
    lo = h.astype(np.float64) < x
    h[lo] = np.nextafter(h[lo], np.float16(np.inf))
    h[x == 0] = 0
    return h


def expected_planes(cells, lr, L):
    C = ob.precompute(cells, lr)
    H, W = C.shape
    P = np.zeros((lr * lr, L["Hqp"], L["Wqp"]))
    for ry in range(lr):
        for rx in range(lr):
            sub = C[ry::lr, rx::lr]
            P[ry * lr + rx, L["M"]:L["M"] + sub.shape[0], L["M"]:L["M"] + sub.shape[1]] = sub
    return P


def clamp_strip(P, lr, M):
    """The superblock planes' input: the phase planes with the strip left of /
    below the map (padded column / row M - 1 of the planes rx > 0 / ry > 0)
    holding the map's first coarse column / row"""
    Q = P.copy()
    for ry in range(lr):
        for rx in range(lr):
            p = ry * lr + rx
            if rx > 0:
                Q[p, :, M - 1] = P[ry * lr, :, M]
            if ry > 0:
                Q[p, M - 1, :] = P[rx, M, :]
            if rx > 0 and ry > 0:
                Q[p, M - 1, M - 1] = P[0, M, M]
    return Q


def unit_u8(h):
    """the 8-bit unit value of an fp16 round-up h (k_rtcsm.hip quad_u8):
    ceil(255 h), exact in fp32 (h has 11 significant bits)"""
    return np.clip(np.ceil(h.astype(np.float32) * np.float32(255.0)), 0, 255).astype(np.uint8)


def check_super(P, S, lr, L):
    """S (sub-phase layout) == the forward 4x4 max of every (strip-clamped)
    plane rounded up to fp16 (bit-exact: round-up is monotone, so the max of the
    round-ups is the round-up of the max); octet layouts hold the 8-bit
    round-up ceil(255 h) of that fp16 value"""
    Hqp, Wqp = L["Hqp"], L["Wqp"]
    pad = np.zeros((lr * lr, Hqp + 3, Wqp + 3))
    pad[:, :Hqp, :Wqp] = clamp_strip(P, lr, L["M"])
    m = np.max([pad[:, j:j + Hqp, i:i + Wqp] for j in range(4) for i in range(4)], axis=0)
    pstride4 = 16 * L["sub4"]
    B = S.view(np.uint8)
    for p in range(lr * lr):
        got = np.zeros((Hqp, Wqp))
        for sy in range(4):
            for sx in range(4):
                if L["oct"]:
                    # units (q, X) of 4 u8 bytes = rows 4q .. 4q + 4 u8 - 1: rows
                    # from the first dword, and dword d equals unit q + d's first
                    h = 4 * L["u8"]   # bytes per unit
                    o = (p * 16 + sy * 4 + sx) * L["subO"] * h
                    u = B[o:o + L["subO"] * h].reshape(L["Qo"], L["Wq4"], h)
                    blk = u[:, :, :4].transpose(0, 2, 1).reshape(4 * L["Qo"], L["Wq4"])[:L["Hq4"]]
                    assert np.array_equal(u[:-2, :, 4:8], u[1:-1, :, :4]), (p, sy, sx)
                    if L["u8"] == 3:
                        assert np.array_equal(u[:-3, :, 8:12], u[2:-1, :, :4]), (p, sy, sx)
                else:
                    blk = S[p * pstride4 + (sy * 4 + sx) * L["sub4"]:][:L["sub4"]].reshape(L["Hq4"], L["Wq4"])
                ys, xs = np.arange(sy, Hqp, 4), np.arange(sx, Wqp, 4)
                got[np.ix_(ys, xs)] = blk[:len(ys), :len(xs)].astype(np.float64)
        want = half_round_up(m[p])
        want = (unit_u8(want) if L["oct"] else want).astype(np.float64)
        assert np.array_equal(got, want), (p, np.argwhere(got != want)[:4])


@pytest.mark.parametrize("lr,n,batch,rxy,fused", [
    (5, 400, 1, (1.0, 1.2), 1), (5, 400, 3, (1.0, 1.2), 1), (4, 200, 2, (1.0, 1.2), 1), (2, 150, 2, (1.0, 1.2), 1),
    (8, 240, 1, (1.0, 1.2), 1), (3, 100, 2, (1.0, 1.2), 1),
    # config-2 window (5 x 5 superblocks) and a 6 x 7 window (24-byte units),
    # planes + units in one pass (k_planes_super) and in two (precompute +
    # k_super_planes); maps not a multiple of 16 coarse rows, 80-row quads
    (5, 400, 2, (4.0, 4.0), 1), (5, 400, 2, (4.0, 4.0), 0), (5, 455, 2, (5.0, 5.4), 1), (5, 455, 2, (5.0, 5.4), 0),
    (5, 1000, 2, (4.0, 4.0), 1), (5, 35, 2, (1.0, 1.2), 1),
    # last 8-row tile starting inside the final window (1008 > 1010 - 5): its
    # footprint does not continue the previous tile's (the streaming batched
    # precompute reloads instead of carrying the halo rows)
    (5, 1010, 2, (1.0, 1.2), 1)])
def test_device_coarse_planes(ctx, world, lr, n, batch, rxy, fused):
    rng = np.random.default_rng(lr * 100 + n)
    cells = np.where(rng.random((n, n)) < 0.3, rng.choice([0.001, 0.3, 0.45, 0.6, 0.999], (n, n)), 0.0)
    mx = my = -0.05 * n / 2
    g = ctx.grid_from_array(cells, mx, my, 0.05)
    ang = scene.beam_angles(361)
    scans = [ctx.scan(rng.uniform(0.5, 4.0, 361), ang) for _ in range(batch)]
    P = abi.RtcsmParams(lr, rxy[0], rxy[1], 0.3, 20.0)
    inits = [(rng.uniform(-0.5, 0.5), rng.uniform(-0.5, 0.5), rng.uniform(-3, 3)) for _ in range(batch)]
    try:
        ctx.set_option(abi.LGS_OPT_FUSED_PLANES, fused)
        if batch == 1:
            ctx.optimize_pose_query(g, P, launcher_cost(), scans[0], inits[0])
        else:
            ctx.optimize_pose_query_batch(g, P, launcher_cost(), scans, inits)
    finally:
        ctx.set_option(abi.LGS_OPT_FUSED_PLANES, 1)
    L = layout(n, n, 0.05, lr, rxy[0], rxy[1])
    want = expected_planes(cells, lr, L)
    for j in range(batch):
        got = ctx.debug_buffer("planes", j)[:want.size].reshape(want.shape)
        assert np.array_equal(got, want), j
        check_super(want, ctx.debug_buffer("super", j), lr, L)


def test_device_coarse_planes_supplied_map(ctx):
    """OptimizePose with a caller's coarse map: the phase-plane copy, incl. a map
    whose size is not a multiple of LowRes (the plain-scratch route)"""
    rng = np.random.default_rng(3)
    for n, lr in [(203, 5), (160, 4)]:
        cells = np.where(rng.random((n, n)) < 0.3, rng.random((n, n)), 0.0)
        g = ctx.grid_from_array(cells, -5.0, -5.0, 0.05)
        cg = ctx.precompute_max(g, lr)
        ang = scene.beam_angles(181)
        sc = ctx.scan(rng.uniform(0.5, 4.0, 181), ang)
        P = abi.RtcsmParams(lr, 1.0, 1.2, 0.3, 20.0)
        ctx.optimize_pose(g, cg, P, launcher_cost(), sc, (0.1, 0.2, 0.3), 0.1)
        L = layout(n, n, 0.05, lr, 1.0, 1.2)
        want = expected_planes(cells, lr, L)
        got = ctx.debug_buffer("planes", 0)[:want.size].reshape(want.shape)
        assert np.array_equal(got, want), (n, lr)
        out = ctx.optimize_pose_query(g, P, launcher_cost(), sc, (0.1, 0.2, 0.3))
        got = ctx.debug_buffer("planes", 0)[:want.size].reshape(want.shape)
        assert np.array_equal(got, want), (n, lr, "query")
        assert out.pose_found in (0, 1)
