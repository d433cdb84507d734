"""GPU parity tests for the map rebuilds around loop closure:

  lgs_maps_construct_from_scans  GridMapBuilder::AfterLoopClosure's rebuild of
                                 every local map (C/mapping/grid_map_builder.cpp:62-80)
  lgs_map_construct_global       GridMapBuilder::ConstructGlobalMap (:83-95)

Each rebuilt map must equal the oracle's ConstructMapFromScans on a map in the
same prior state (Resize is anchored to the previous geometry): geometry,
hit/miss counts and cell values bit-exact.  The fused pass over many maps and
the chunked ray-cast (LGS_OPT_RAY_CHUNK_KEYS) must not change a single cell."""
import numpy as np
import pytest

import oracle_bind as ob
from lgs_amd import abi, scene
from test_gpu_raycast import BP, same_map

pytestmark = pytest.mark.gpu


def _trajectory(n, seed=0):
    rng = np.random.default_rng(seed)
    t = np.linspace(0.0, 2.0 * np.pi, n, endpoint=False)
    return [(1.2 * np.cos(a) + rng.uniform(-0.05, 0.05), 0.9 * np.sin(a) + rng.uniform(-0.05, 0.05),
             a + np.pi / 2 + rng.uniform(-0.05, 0.05)) for a in t]


def _nodes(ctx, world, poses, n_beams):
    ang = scene.beam_angles(n_beams)
    rs = [scene.ray_cast(world, p, ang) for p in poses]
    return [ctx.scan(r, ang) for r in rs], [ob.OScan(r, ang) for r in rs]


def _local_maps(ctx, ranges, poses, dscans, oscans, ps=64):
    """Local maps grown scan by scan as UpdateGridMap does (0x0 at the first pose)."""
    bp, obp = abi.BuilderParams(*BP), ob.BuilderParams(*BP)
    gms, oms = [], []
    for lo, hi in ranges:
        gm = ctx.map(0.05, ps, 0, 0, center=poses[lo][:2])
        om = ob.OMap(0.05, ps, 0, 0, center=poses[lo][:2])
        for k in range(lo, hi + 1):
            gm.update_scan(dscans[k], poses[k], bp)
            om.integrate(poses[k], oscans[k], obp)
        gms.append(gm)
        oms.append(om)
    return gms, oms


def _perturb(poses, seed=1):
    rng = np.random.default_rng(seed)
    return [(x + rng.uniform(-0.04, 0.04), y + rng.uniform(-0.04, 0.04), t + rng.uniform(-0.02, 0.02))
            for x, y, t in poses]


@pytest.mark.parametrize("dev", [1, 0])
@pytest.mark.parametrize("chunk", [0, 20000, 1])
def test_after_loop_closure_rebuild(ctx, world, chunk, dev):
    """Four local maps (overlapping node ranges, one single-node map) rebuilt
    after the poses moved; chunk > 0 forces ray-cast passes of that many keys
    (1 = one ray per pass), so passes split maps and scans (the device hit
    points, dev = 1, then hand over to the host path after resizing the maps)."""
    n = 48 if chunk != 1 else 12
    poses = _trajectory(n)
    dscans, oscans = _nodes(ctx, world, poses, 361 if chunk != 1 else 91)
    q = n // 4
    ranges = [(0, q + 2), (q, 2 * q), (2 * q + 1, 2 * q + 1), (2 * q + 2, n - 1)]
    gms, oms = _local_maps(ctx, ranges, poses, dscans, oscans)
    new = _perturb(poses)
    try:
        ctx.set_option(abi.LGS_OPT_DEVICE_HITS, dev)
        if chunk:
            ctx.set_option(abi.LGS_OPT_RAY_CHUNK_KEYS, chunk)
        ctx.construct_maps(gms, ranges, dscans, new, abi.BuilderParams(*BP))
    finally:
        ctx.set_option(abi.LGS_OPT_RAY_CHUNK_KEYS, 1 << 28)
        ctx.set_option(abi.LGS_OPT_DEVICE_HITS, 1)
    obp = ob.BuilderParams(*BP)
    for i, ((lo, hi), gm, om) in enumerate(zip(ranges, gms, oms)):
        om.construct(new[lo:hi + 1], oscans[lo:hi + 1], obp)
        same_map(gm, om, f"map{i}")


def test_after_loop_closure_equals_one_by_one(ctx, world):
    """The fused pass over all maps gives what ConstructMapFromScans per map gives."""
    poses = _trajectory(30, seed=4)
    dscans, oscans = _nodes(ctx, world, poses, 241)
    ranges = [(0, 9), (10, 19), (20, 29)]
    fused, _ = _local_maps(ctx, ranges, poses, dscans, oscans)
    single, _ = _local_maps(ctx, ranges, poses, dscans, oscans)
    new = _perturb(poses, seed=5)
    bp = abi.BuilderParams(*BP)
    ctx.construct_maps(fused, ranges, dscans, new, bp)
    for (lo, hi), gm in zip(ranges, single):
        gm.construct(dscans[lo:hi + 1], new[lo:hi + 1], bp)
    for i, (a, b) in enumerate(zip(fused, single)):
        assert a.geometry() == b.geometry(), i
        for x, y in zip(a.download(), b.download()):
            assert np.array_equal(x, y), i


@pytest.mark.parametrize("dev", [1, 0])
@pytest.mark.parametrize("chunk", [0, 50000])
def test_global_map(ctx, world, chunk, dev):
    """ConstructGlobalMap: a fresh 0x0 map at (0, 0), every node, PatchSize 64."""
    poses = _trajectory(40, seed=2)
    dscans, oscans = _nodes(ctx, world, poses, 541)
    try:
        ctx.set_option(abi.LGS_OPT_DEVICE_HITS, dev)
        if chunk:
            ctx.set_option(abi.LGS_OPT_RAY_CHUNK_KEYS, chunk)
        gm = ctx.construct_global_map(0.05, 64, dscans, poses, abi.BuilderParams(*BP))
    finally:
        ctx.set_option(abi.LGS_OPT_RAY_CHUNK_KEYS, 1 << 28)
        ctx.set_option(abi.LGS_OPT_DEVICE_HITS, 1)
    om = ob.OMap(0.05, 64, 0, 0)
    om.construct(poses, oscans, ob.BuilderParams(*BP))
    same_map(gm, om, "global")


def test_rebuild_reuses_allocation(ctx, world):
    """A rebuild into a smaller box reuses the map's cells; a second rebuild
    into a larger box reallocates -- both still match the oracle."""
    poses = _trajectory(16, seed=6)
    dscans, oscans = _nodes(ctx, world, poses, 181)
    gm = ctx.map(0.05, 32, 0, 0)
    om = ob.OMap(0.05, 32, 0, 0)
    bp, obp = abi.BuilderParams(*BP), ob.BuilderParams(*BP)
    for lo, hi in [(0, 15), (3, 5), (0, 15), (7, 7)]:
        ctx.construct_maps([gm], [(lo, hi)], dscans, poses, bp)
        om.construct(poses[lo:hi + 1], oscans[lo:hi + 1], obp)
        same_map(gm, om, f"{lo}-{hi}")


def test_rebuild_argument_checks(ctx, world):
    poses = _trajectory(4)
    dscans, _ = _nodes(ctx, world, poses, 31)
    a, b = ctx.map(0.05, 16, 0, 0), ctx.map(0.05, 16, 0, 0)
    bp = abi.BuilderParams(*BP)
    for maps, ranges in [([a, a], [(0, 1), (2, 3)]),       # same map twice
                         ([a], [(2, 1)]),                   # empty range
                         ([a, b], [(0, 1), (2, 4)]),        # past the last node
                         ([a], [(-1, 0)])]:
        with pytest.raises(abi.LgsError):
            ctx.construct_maps(maps, ranges, dscans, poses, bp)
    with pytest.raises(abi.LgsError):
        ctx.set_option(abi.LGS_OPT_RAY_CHUNK_KEYS, 0)


@pytest.mark.parametrize("p_hit,p_miss", [(0.6, 0.45), (0.9, 0.1), (0.4, 0.7), (0.55, 0.5)])
def test_long_runs(ctx, world, p_hit, p_miss):
    """Cells updated thousands of times (120 scans from 3 poses: long runs of
    misses next to the sensors and of hits on the walls) go through the
    wavefront-per-run apply; pHit < 0.5 or pMiss >= 0.5 change which updates
    are exact fixed points."""
    ang = scene.beam_angles(721)
    base = [(0.0, 0.0, 0.0), (0.02, -0.01, 0.3), (-0.3, 0.2, 1.0)]
    poses = [base[k % 3] for k in range(120)]
    dscans, oscans = _nodes(ctx, world, poses, 721)
    bp = abi.BuilderParams(0.01, 20.0, p_hit, p_miss)
    gm = ctx.construct_global_map(0.05, 64, dscans, poses, bp)
    om = ob.OMap(0.05, 64, 0, 0)
    om.construct(poses, oscans, ob.BuilderParams(0.01, 20.0, p_hit, p_miss))
    same_map(gm, om, f"{p_hit}/{p_miss}")
    assert om.hits().max() >= 100 and om.misses().max() >= 1000


def test_render_gray_matches_drawmap(ctx, world):
    """f4: MapSaver::DrawMap's gray levels (C/io/map_saver.cpp:276-313) for every
    cell, rows flipped up-down (:455-456); restated with numpy on the same
    downloaded cells (truncating uint8 cast of (1 - p) * 255, 192 for p <= 0)."""
    poses = _trajectory(20, seed=8)
    dscans, _ = _nodes(ctx, world, poses, 361)
    gm = ctx.construct_global_map(0.05, 64, dscans, poses, abi.BuilderParams(*BP))
    cells, _, _ = gm.download()
    img = gm.render_gray()
    want = np.where((cells <= 0.0) | (cells > 1.0), 192, ((1.0 - cells) * 255.0).astype(np.uint8)).astype(np.uint8)
    assert np.array_equal(img, want[::-1])
    assert (img == 192).any() and (img < 192).any()


def test_device_hits_scan_filters_and_empty_scans(ctx, world):
    """Device hit points: beams at exactly the usable range limits, zero and
    NaN-free short ranges, a scan with no usable beam (its sensor still in
    the box, no rays), and maps of one node -- every map as the oracle's."""
    poses = _trajectory(10, seed=9)
    ang = scene.beam_angles(181)
    rs = [scene.ray_cast(world, p, ang) for p in poses]
    rs[2] = np.full(181, 25.0)                 # every beam beyond 20 m: no hit
    rs[4][::7] = 20.0                          # at the usable maximum (excluded)
    rs[4][3::11] = 0.01                        # at the usable minimum (excluded)
    rs[5][::5] = 0.0
    dscans = [ctx.scan(r, ang) for r in rs]
    oscans = [ob.OScan(r, ang) for r in rs]
    ranges = [(0, 3), (2, 2), (4, 9)]
    gms = [ctx.map(0.05, 32, 0, 0, center=poses[lo][:2]) for lo, _ in ranges]
    oms = [ob.OMap(0.05, 32, 0, 0, center=poses[lo][:2]) for lo, _ in ranges]
    ctx.construct_maps(gms, ranges, dscans, poses, abi.BuilderParams(*BP))
    obp = ob.BuilderParams(*BP)
    for i, ((lo, hi), gm, om) in enumerate(zip(ranges, gms, oms)):
        om.construct(poses[lo:hi + 1], oscans[lo:hi + 1], obp)
        same_map(gm, om, f"map{i}")
