"""Patch-native ingest of a reference GridMapType (lgs_grid_upload_patches)
against the dense upload it replaces.

The reference's map is patch-major (H/grid_map/grid_map.hpp:295-317
mPatches; H/grid_map/grid_map_patch.hpp:15-193: cells[y * ps + x], nullptr =
unallocated) with 16-byte BinaryBayesGridCell<double> cells (vptr + mValue,
value at byte 8).  Patches here carry garbage in the vptr half, unallocated
patches and maps in the negative quadrant; the ingested grid must equal
GridMap::Value(x, y, 0.0) of every cell bit for bit, and a correlative match
on it must equal the match on the dense upload."""
import numpy as np
import pytest

from lgs_amd import abi, scene

pytestmark = pytest.mark.gpu


def to_patches(cells, ps, rng, drop=0.3, cell_bytes=16, value_offset=8):
    """Split a dense (h, w) map into reference-layout patches; a fraction of
    the all-unknown patches stays unallocated (None), the rest keep zeros."""
    h, w = cells.shape
    npy, npx = h // ps, w // ps
    out = []
    for py in range(npy):
        for px in range(npx):
            blk = cells[py * ps:(py + 1) * ps, px * ps:(px + 1) * ps]
            if not blk.any() and rng.random() < 1.0 - drop:
                out.append(None)
                continue
            raw = rng.integers(0, 2 ** 63, size=(ps, ps, cell_bytes // 8)).astype(np.uint64)
            raw[:, :, value_offset // 8] = blk.view(np.uint64)
            out.append(raw)
    return out, npx, npy


def reference_value_grid(patches, npx, npy, ps, value_offset=8):
    """GridMap::Value(x, y, 0.0) of every cell (H/grid_map/grid_map.hpp:858-873)."""
    g = np.zeros((npy * ps, npx * ps))
    for p, raw in enumerate(patches):
        if raw is None:
            continue
        py, px = divmod(p, npx)
        g[py * ps:(py + 1) * ps, px * ps:(px + 1) * ps] = raw[:, :, value_offset // 8].view(np.float64)
    return g


@pytest.mark.parametrize("ps,w,h,mx,my", [(100, 1000, 1000, -25.0, -25.0), (64, 384, 256, -9.6, -3.2),
                                          (7, 70, 49, -1.75, 2.0), (1, 5, 3, -0.1, -0.2)])
def test_patch_ingest_equals_value_grid(ctx, world, ps, w, h, mx, my):
    rng = np.random.default_rng(ps)
    cells = np.where(rng.random((h, w)) < 0.3, rng.random((h, w)), 0.0)
    cells[: h // 2, : w // 3] = 0.0     # whole unknown patches
    patches, npx, npy = to_patches(cells, ps, rng)
    assert any(p is None for p in patches) or npx * npy == 1
    g = ctx.grid_from_patches(patches, npx, npy, ps, mx, my, 0.05)
    dev = g.download()
    assert np.array_equal(dev.view(np.uint64), reference_value_grid(patches, npx, npy, ps).view(np.uint64))
    # re-ingest into the same grid after every patch changed allocation state
    patches2 = [None if p is not None else np.zeros((ps, ps, 2), np.uint64) for p in patches]
    ctx.grid_from_patches(patches2, npx, npy, ps, mx, my, 0.05, into=g)
    assert np.array_equal(g.download(), reference_value_grid(patches2, npx, npy, ps))


def test_patch_ingest_other_cell_layouts(ctx):
    rng = np.random.default_rng(3)
    cells = rng.random((40, 60))
    for cb, off in ((8, 0), (24, 16), (32, 8)):
        patches, npx, npy = to_patches(cells, 20, rng, cell_bytes=cb, value_offset=off)
        g = ctx.grid_from_patches(patches, npx, npy, 20, 0.0, 0.0, 0.05, cell_bytes=cb, value_offset=off)
        assert np.array_equal(g.download(), reference_value_grid(patches, npx, npy, 20, off))
    with pytest.raises(abi.LgsError):
        ctx.grid_from_patches([None] * 6, 3, 2, 20, 0.0, 0.0, 0.05, cell_bytes=16, value_offset=4)
    with pytest.raises(abi.LgsError):
        ctx.grid_from_patches([None] * 6, 3, 2, 20, 0.0, 0.0, 0.05,
                              into=ctx.grid(59, 40, 0.0, 0.0, 0.05))


def test_match_on_patch_ingest_equals_dense(ctx, world):
    """Config-2 shape: 1000x1000 @ 5 cm, PatchSize 100, minPos (-25, -25), the
    bench map; OptimizePose(query) on the patch-ingested grid == on the dense
    upload, every field."""
    ang = scene.beam_angles(1081)
    w, h, mx, my = scene.map_geometry(1000, 100, 0.05)
    cells = scene.approx_occupancy_map(world, scene.arc_poses(10), ang, w, h, mx, my, 0.05)
    rng = np.random.default_rng(9)
    patches, npx, npy = to_patches(cells, 100, rng, drop=0.0)
    assert sum(p is None for p in patches) > 0
    pg = ctx.grid_from_patches(patches, npx, npy, 100, mx, my, 0.05)
    dg = ctx.grid_from_array(cells, mx, my, 0.05)
    prm = abi.RtcsmParams(5, 4.0, 4.0, 1.0471976, 20.0)
    cost = abi.CostGEParams(0.01, 20.0, 0.075, 0.1, 1, 0.05, 1.0)
    for k in range(4):
        true = (rng.uniform(-1.5, 1.5), rng.uniform(-1.5, 1.5), rng.uniform(-3, 3))
        sc = ctx.scan(scene.ray_cast(world, true, ang), ang)
        init = (true[0] + 0.2, true[1] - 0.1, true[2] + 0.1)
        a = ctx.optimize_pose_query(pg, prm, cost, sc, init)
        b = ctx.optimize_pose_query(dg, prm, cost, sc, init)
        assert list(a.best_win) == list(b.best_win) and a.score_max == b.score_max
        assert (a.estimated_pose.x, a.estimated_pose.y, a.estimated_pose.theta) == \
            (b.estimated_pose.x, b.estimated_pose.y, b.estimated_pose.theta)
        assert a.normalized_cost == b.normalized_cost and list(a.covariance) == list(b.covariance)


def test_patch_ingest_taller_than_grid_y_limit(ctx):
    """65,600 rows (> the 65,535 grid-y limit): rows are grid-strided."""
    rng = np.random.default_rng(12)
    ps, npx, npy = 8, 1, 8200
    cells = np.where(rng.random((npy * ps, npx * ps)) < 0.5, rng.random((npy * ps, npx * ps)), 0.0)
    patches, npx, npy = to_patches(cells, ps, rng)
    g = ctx.grid_from_patches(patches, npx, npy, ps, 0.0, 0.0, 0.05)
    assert np.array_equal(g.download().view(np.uint64), reference_value_grid(patches, npx, npy, ps).view(np.uint64))


def test_upload_into_map_view_rejected(ctx):
    """A map's grid view changes only through the map (its counters and patch
    flags): dense and patch uploads into it are refused."""
    m = ctx.map(0.05, 10, 20, 20)
    view = m.grid()
    with pytest.raises(abi.LgsError, match="map's grid view"):
        view.upload(np.zeros((view.hgt, view.w)))
    with pytest.raises(abi.LgsError, match="map's grid view"):
        ctx.grid_from_patches([None] * ((view.w // 10) * (view.hgt // 10)), view.w // 10, view.hgt // 10, 10,
                              view.min_x, view.min_y, 0.05, into=view)
