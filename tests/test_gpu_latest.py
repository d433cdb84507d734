"""The latest map's incremental rebuild against the oracle.

UpdateLatestMap (C/mapping/grid_map_builder.cpp:196-207) rebuilds the latest
map from the last n scans after every scan (ConstructMapFromScans :227-332:
Resize to the window's box, Reset, every scan's rays in order).  The device
keeps the window's sorted key lists and recomputes only the cells the entering
or the leaving scan touches when the geometry holds; every step here compares
the whole latest map (cells, hit/miss counts, patch flags, geometry) and the
local map with the oracle bit for bit, and checks which steps ran
incrementally -- including the transitions that must fall back to a full
rebuild (geometry change, a moved node, other parameters, a different window,
a direct update of the map)."""
import numpy as np
import pytest

import oracle_bind as ob
from lgs_amd import abi, scene
from test_gpu_raycast import same_map

pytestmark = pytest.mark.gpu
BP = (0.01, 20.0, 0.6, 0.45)


def _traj(n, r=5.0, dth=0.02):
    return [(r * np.cos(dth * k), r * np.sin(dth * k), dth * k + np.pi / 2) for k in range(n)]


def _setup(ctx, world, poses, n_beams=1081):
    ang = scene.beam_angles(n_beams)
    ranges = [scene.ray_cast(world, p, ang) for p in poses]
    dscans = [ctx.scan(r, ang) for r in ranges]
    oscans = [ob.OScan(r, ang) for r in ranges]
    return ang, ranges, dscans, oscans


def test_append_scan_sliding_window_every_step(ctx, world):
    """40 AppendScan steps of a 10-scan window: after the first full build,
    the window grows (no scan leaves) then slides (the oldest leaves); each
    step must be incremental and bit-exact, the local map too."""
    poses = _traj(41)
    _, _, dscans, oscans = _setup(ctx, world, poses)
    bp, obp = abi.BuilderParams(*BP), ob.BuilderParams(*BP)
    local = ctx.map(0.05, 100, 200, 200, center=poses[0][:2])
    latest = ctx.map(0.05, 100, 200, 200, center=poses[0][:2])
    olocal = ob.OMap(0.05, 100, 200, 200, center=poses[0][:2])
    olatest = ob.OMap(0.05, 100, 200, 200, center=poses[0][:2])
    full_before = 0
    for k in range(len(poses)):
        lo = max(0, k - 9)
        local.append_scan(latest, dscans[lo:k + 1], poses[lo:k + 1], bp)
        olocal.integrate(poses[k], oscans[k], obp)
        olatest.construct(poses[lo:k + 1], oscans[lo:k + 1], obp)
        same_map(latest, olatest, f"latest k{k}")
        if k % 8 == 0:
            same_map(local, olocal, f"local k{k}")
        rb = latest.rebuilds()
        if k > 0:
            # a full rebuild happens only when the window's box moves the geometry
            if rb["full"] > full_before:
                assert latest.geometry() != prev_geom, k
        full_before = rb["full"]
        prev_geom = latest.geometry()
    rb = latest.rebuilds()
    assert rb["incremental"] >= 30, rb
    same_map(local, olocal, "local map")


def test_construct_window_transitions(ctx, world):
    """ConstructMapFromScans on one map object through every transition: grow,
    slide, a node moved by loop closure (full), other pHit/pMiss (full), the
    same window again (full: it gained no scan), a jump that changes the
    geometry (full), a direct insert into the map (invalidates), scans
    recreated at the same poses (new ids: full), windows of 1 and 15 scans."""
    poses = _traj(30, r=3.0, dth=0.03)
    _, ranges, dscans, oscans = _setup(ctx, world, poses, 541)
    ang = scene.beam_angles(541)
    gm = ctx.map(0.05, 64, 0, 0)
    om = ob.OMap(0.05, 64, 0, 0)

    def step(lo, hi, bpv=BP, ps=None, tag=""):
        ps = poses if ps is None else ps
        gm.construct(dscans[lo:hi], ps[lo:hi], abi.BuilderParams(*bpv))
        om.construct(ps[lo:hi], oscans[lo:hi], ob.BuilderParams(*bpv))
        same_map(gm, om, tag)
        return gm.rebuilds()

    r0 = step(0, 1, tag="first")
    assert r0 == {"incremental": 0, "full": 1}
    for k in range(2, 12):
        step(max(0, k - 10), k, tag=f"grow/slide {k}")
    r1 = gm.rebuilds()
    assert r1["incremental"] >= 5, r1
    # loop closure moved an old node: full
    moved = list(poses)
    moved[5] = (moved[5][0] + 0.01, moved[5][1], moved[5][2])
    r2 = step(2, 12, ps=moved, tag="moved node")
    assert r2["full"] == r1["full"] + 1, (r1, r2)
    # other builder parameters: full
    r3 = step(3, 13, bpv=(0.01, 20.0, 0.7, 0.4), ps=moved, tag="params")
    assert r3["full"] == r2["full"] + 1
    # the very same window again: full
    r4 = step(3, 13, bpv=(0.01, 20.0, 0.7, 0.4), ps=moved, tag="same window")
    assert r4["full"] == r3["full"] + 1
    for k in range(14, 20):
        step(k - 10, k, ps=moved, tag=f"slide {k}")
    # a direct insert into the latest map: its lists are invalid
    gm.update_scan(dscans[0], poses[0], abi.BuilderParams(*BP))
    om.integrate(poses[0], oscans[0], ob.BuilderParams(*BP))
    same_map(gm, om, "insert")
    r5 = gm.rebuilds()
    r6 = step(10, 20, ps=moved, tag="after insert")
    assert r6["full"] == r5["full"] + 1
    # scans recreated at the same poses (new ids): full
    for i in range(11, 21):
        dscans[i] = ctx.scan(ranges[i], ang)
    r7 = step(11, 21, ps=moved, tag="recreated")
    assert r7["full"] == r6["full"] + 1
    # window of 15 scans (the most the lists hold), then 16 (untagged full rebuilds)
    for k in range(22, 27):
        step(max(0, k - 15), k, ps=moved, tag=f"w15 {k}")
    step(10, 26, ps=moved, tag="w16")
    step(10, 27, ps=moved, tag="w17")
    # a jump far away: the geometry changes
    far = list(moved)
    far[27] = (far[26][0] - 4.0, far[26][1] - 4.0, far[26][2])
    step(18, 28, ps=far, tag="jump")
    for k in range(29, 31):
        step(k - 10, k, ps=far, tag=f"after jump {k}")


def test_append_scan_empty_and_degenerate_scans(ctx, world):
    """Scans without usable beams (every range filtered) inside the window:
    the window's lists hold empty slots; a scan entering or leaving with no
    keys leaves the map as the full rebuild does."""
    poses = _traj(16)
    ang, ranges, dscans, oscans = _setup(ctx, world, poses, 361)
    for k in (3, 4, 9):
        ranges[k] = np.full(361, 25.0)   # >= usable max: every beam skipped
        dscans[k] = ctx.scan(ranges[k], ang)
        oscans[k] = ob.OScan(ranges[k], ang)
    bp, obp = abi.BuilderParams(*BP), ob.BuilderParams(*BP)
    local = ctx.map(0.05, 64, 100, 100, center=poses[0][:2])
    latest = ctx.map(0.05, 64, 100, 100, center=poses[0][:2])
    olocal = ob.OMap(0.05, 64, 100, 100, center=poses[0][:2])
    olatest = ob.OMap(0.05, 64, 100, 100, center=poses[0][:2])
    for k in range(len(poses)):
        lo = max(0, k - 5)
        local.append_scan(latest, dscans[lo:k + 1], poses[lo:k + 1], bp)
        olocal.integrate(poses[k], oscans[k], obp)
        olatest.construct(poses[lo:k + 1], oscans[lo:k + 1], obp)
        same_map(latest, olatest, f"latest k{k}")
    same_map(local, olocal, "local")
    assert latest.rebuilds()["incremental"] > 0
