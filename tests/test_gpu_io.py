"""GPU parity tests for MapSaver (SURVEY §8(f) f4, C/io/map_saver.cpp):
the map image the reference writes -- DrawMap over the actual map size
(GridMap::ComputeActualMapSize of the allocated patches), the trajectory and
scan overlays, the up-down flip -- drawn from the device map, against the
oracle's restatement (orc_map_draw_image) on the same scans: every pixel
bit-exact; the PNG decodes to the same pixels; the metadata JSON holds the
reference's fields."""
import json

import numpy as np
import pytest

import oracle_bind as ob
from lgs_amd import abi, io, scene
from test_gpu_mapbuild import _local_maps, _nodes, _perturb, _trajectory
from test_gpu_raycast import BP, same_map

pytestmark = pytest.mark.gpu


def _pair(ctx, world, n=12, beams=361, ps=64, seed=3):
    poses = _trajectory(n, seed=seed)
    dscans, oscans = _nodes(ctx, world, poses, beams)
    gms, oms = _local_maps(ctx, [(0, n - 1)], poses, dscans, oscans, ps=ps)
    return poses, dscans, oscans, gms[0], oms[0]


def test_actual_size_and_patches(ctx, world):
    """ComputeActualMapSize (H/grid_map/grid_map.hpp:969-1015) from the
    device's patch-allocation flags; a local map grown by Expand has
    unallocated patches around the scans."""
    poses, _, _, gm, om = _pair(ctx, world)
    same_map(gm, om)
    n, a = gm.actual_size()
    assert 0 < n < gm.patches().size
    assert a[10] == a[8] * 64 and a[11] == a[9] * 64
    assert (gm.patches() == 0).any()


@pytest.mark.parametrize("overlay", ["none", "trajectory", "scan", "both"])
def test_draw_image_matches_oracle(ctx, world, overlay):
    poses, dscans, oscans, gm, om = _pair(ctx, world, n=16, seed=4)
    traj = overlay in ("trajectory", "both")
    scan = None
    oscan = None
    sp = poses[7]
    if overlay in ("scan", "both"):
        ang = scene.beam_angles(361)
        r = scene.ray_cast(world, sp, ang)
        rel = (0.1, -0.05, 0.02)
        scan = (r, ang, rel)
        oscan = ob.OScan(r, ang, rel=rel)
    img = io.draw_image(gm, poses, draw_trajectory=traj, node_min=2, node_max=13, scan=scan, scan_pose=sp)
    want = om.draw_image(poses, draw_trajectory=traj, node_min=2, node_max=13, scan=oscan, scan_pose=sp)
    assert img.shape == want.shape
    assert np.array_equal(img, want)
    if traj:
        assert ((img[..., 0] == 255) & (img[..., 1] == 0)).any()
    if scan is not None:
        assert ((img[..., 2] == 255) & (img[..., 0] == 0)).any()


def test_saved_png_and_metadata(ctx, world, tmp_path):
    """SaveMapCore: <name>.png decodes to the drawn image; <name>.json is
    SaveMapMetadata's tree (C/io/map_saver.cpp:499-532)"""
    poses, _, _, gm, om = _pair(ctx, world, n=10, seed=5)
    f = str(tmp_path / "map")
    io.save_map(gm, poses, f, draw_trajectory=True, save_metadata=True)
    png = io.read_png_rgb8(f + ".png")
    assert np.array_equal(png, om.draw_image(poses, draw_trajectory=True))
    meta = json.load(open(f + ".json"))["Map"]
    n, a = om.actual_size()
    g = gm.geometry()
    res = 0.05
    assert float(meta["Resolution"]) == res and meta["PatchSize"] == "64"
    assert [int(meta[k]) for k in ("WidthInPatches", "HeightInPatches", "WidthInGridCells", "HeightInGridCells")] \
        == a[8:12]
    assert float(meta["BottomLeft"]["X"]) == g["min_x"] + res * a[4]
    assert float(meta["TopRight"]["Y"]) == g["min_y"] + res * a[7]
    assert meta["PoseGraphNodeIdxMin"] == "0" and meta["PoseGraphNodeIdxMax"] == str(len(poses) - 1)


def test_latest_map_keeps_patches_across_rebuilds(ctx, world):
    """ConstructMapFromScans' Reset keeps patches allocated
    (H/grid_map/grid_map_patch.hpp:194-203): a latest map rebuilt over a
    sliding window crops to every patch any window touched, as the reference's
    SaveLatestMap image does."""
    ang = scene.beam_angles(181)
    poses = [(0.25 * k - 1.5, 0.1 * k - 0.5, 0.05 * k) for k in range(14)]
    rs = [scene.ray_cast(world, p, ang) for p in poses]
    d = [ctx.scan(r, ang) for r in rs]
    o = [ob.OScan(r, ang) for r in rs]
    gm = ctx.map(0.05, 32, 0, 0)
    om = ob.OMap(0.05, 32, 0, 0)
    bp, obp = abi.BuilderParams(*BP), ob.BuilderParams(*BP)
    for k in range(len(poses)):
        lo = max(0, k - 4)
        gm.construct(d[lo:k + 1], poses[lo:k + 1], bp)
        om.construct(poses[lo:k + 1], o[lo:k + 1], obp)
        same_map(gm, om, f"frame{k}")
        assert np.array_equal(io.draw_image(gm, poses), om.draw_image(poses)), k


def test_after_loop_closure_maps_draw(ctx, world):
    """AfterLoopClosure's fused rebuild moves and keeps the patch flags of
    every local map like ConstructMapFromScans one by one"""
    poses = _trajectory(24, seed=6)
    dscans, oscans = _nodes(ctx, world, poses, 181)
    ranges = [(0, 7), (8, 15), (16, 23)]
    gms, oms = _local_maps(ctx, ranges, poses, dscans, oscans, ps=32)
    new = _perturb(poses, seed=7)
    ctx.construct_maps(gms, ranges, dscans, new, abi.BuilderParams(*BP))
    obp = ob.BuilderParams(*BP)
    for i, ((lo, hi), gm, om) in enumerate(zip(ranges, gms, oms)):
        om.construct(new[lo:hi + 1], oscans[lo:hi + 1], obp)
        same_map(gm, om, f"map{i}")
        img = io.draw_image(gm, new, draw_trajectory=True, node_min=lo, node_max=hi)
        assert np.array_equal(img, om.draw_image(new, draw_trajectory=True, node_min=lo, node_max=hi)), i


def test_render_region_matches_full_render(ctx, world):
    """lgs_map_render_gray_region == the matching window of lgs_map_render_gray"""
    _, _, _, gm, _ = _pair(ctx, world, n=8, seed=9)
    g = gm.geometry()
    full = gm.render_gray()[::-1]          # unflip: row y = cell row y
    x0, y0, w, h = 5, 7, g["w"] - 13, g["h"] - 9
    reg = gm.render_gray_region(x0, y0, w, h, flip=False)
    assert np.array_equal(reg, full[y0:y0 + h, x0:x0 + w])
    assert np.array_equal(gm.render_gray_region(x0, y0, w, h, flip=True), reg[::-1])


def test_empty_map_has_no_image(ctx):
    gm = ctx.map(0.05, 64, 128, 128)
    n, a = gm.actual_size()
    assert n == 0 and a == [0] * 12
    with pytest.raises(abi.LgsError):
        io.draw_image(gm, [(0.0, 0.0, 0.0)])
