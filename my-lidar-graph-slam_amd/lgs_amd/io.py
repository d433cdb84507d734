"""ctypes binding of include/lgs_io.h (liblgs_slam_hip.so): the Carmen log
reader, the pose-graph LM optimizer, the robust losses and the map / pose-graph
savers.  Plumbing for tests: the work runs in the C++
host library (and, for the map image, on the device through liblgs_hip.so).
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Optional, Sequence

import numpy as np

from . import abi
from .abi import Pose2D, ScanHost

LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "liblgs_slam_hip.so")
_P = C.c_void_p
_D = C.POINTER(C.c_double)

LM_SPARSE_CHOLESKY = 0
LM_CONJUGATE_GRADIENT = 1
LOSSES = dict(huber=0, cauchy=1, fair=2, geman_mcclure=3, welsch=4, dcs=5, squared=6)


class PoseGraphEdge(C.Structure):
    _fields_ = [("start_node_index", C.c_int), ("end_node_index", C.c_int), ("relative_pose", Pose2D),
                ("information", C.c_double * 9)]


class LMParams(C.Structure):
    _fields_ = [("solver", C.c_int), ("num_iterations_max", C.c_int), ("error_tolerance", C.c_double),
                ("lambda_", C.c_double), ("loss_kind", C.c_int), ("loss_scale", C.c_double)]


class MapSaveOptions(C.Structure):
    _fields_ = [("draw_trajectory", C.c_int), ("trajectory_node_index_min", C.c_int),
                ("trajectory_node_index_max", C.c_int), ("draw_scan", C.c_int), ("scan_pose", Pose2D),
                ("scan", C.POINTER(ScanHost)), ("save_metadata", C.c_int)]


_PROTOS = [
    ("lgs_carmen_load", C.c_longlong, [C.c_char_p, _D, C.c_longlong, C.c_char_p, C.c_longlong,
                                       C.POINTER(C.c_longlong),
                                       C.POINTER(C.c_int)]),
    ("lgs_pose_graph_optimize_lm", C.c_int, [C.POINTER(LMParams), C.POINTER(Pose2D), C.c_int,
                                             C.POINTER(PoseGraphEdge), C.c_int, C.POINTER(C.c_int), _D]),
    ("lgs_robust_loss", C.c_int, [C.c_int, C.c_double, _D, C.c_int, _D]),
    ("lgs_map_draw_image", C.c_int, [_P, _P, C.POINTER(Pose2D), C.c_int, C.POINTER(MapSaveOptions),
                                     C.POINTER(C.c_uint8), C.c_size_t, C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    ("lgs_map_save", C.c_int, [_P, _P, C.POINTER(Pose2D), C.c_int, C.POINTER(MapSaveOptions), C.c_char_p]),
    ("lgs_pose_graph_save", C.c_int, [C.POINTER(C.c_int), C.POINTER(Pose2D), _D, C.c_int,
                                      C.POINTER(PoseGraphEdge), C.c_int, C.c_char_p]),
    ("lgs_png_write_rgb8", C.c_int, [C.c_char_p, C.POINTER(C.c_uint8), C.c_int, C.c_int]),
]
SYMBOLS = [p[0] for p in _PROTOS]
_lib: Optional[C.CDLL] = None


def load() -> C.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"host library missing: {LIB_PATH} (run __graft_entry__.build())")
        abi.load()   # liblgs_hip.so first (the host library links it)
        lib = C.CDLL(LIB_PATH)
        for name, res, args in _PROTOS:
            fn = getattr(lib, name)
            fn.restype, fn.argtypes = res, args
        _lib = lib
    return _lib


def _dp(a):
    return a.ctypes.data_as(_D)


def carmen_load(text: str):
    """CarmenLogReader::Load -> (flat fp64 record stream, sensor ids, record count)"""
    L = load()
    raw = text.encode()
    n = C.c_int()
    nid = C.c_longlong()
    need = L.lgs_carmen_load(raw, None, 0, None, 0, C.byref(nid), C.byref(n))
    if need < 0:
        raise ValueError("CarmenLogReader failed")
    out = np.zeros(max(1, need))
    ids = C.create_string_buffer(max(1, nid.value))
    L.lgs_carmen_load(raw, _dp(out), need, ids, len(ids), None, C.byref(n))
    names = ids.raw.split(b"\0")[: n.value]
    return out[:need], [s.decode() for s in names], n.value


def edges_array(edges):
    """edges: [(start, end, (x, y, theta), info 3x3)]"""
    arr = (PoseGraphEdge * max(1, len(edges)))()
    for k, (s, e, z, info) in enumerate(edges):
        arr[k].start_node_index, arr[k].end_node_index = s, e
        arr[k].relative_pose = Pose2D(*z)
        arr[k].information[:] = [float(v) for v in np.asarray(info, dtype=np.float64).reshape(9)]
    return arr


def optimize_lm(poses, edges, solver=LM_SPARSE_CHOLESKY, iters=10, tol=1e-3, lam=1e-4, loss="huber",
                scale=1.0):
    """PoseGraphOptimizerLM::Optimize -> (poses [n, 3], iterations, total error, lambda after)"""
    L = load()
    n = len(poses)
    p = (Pose2D * max(1, n))(*[Pose2D(*q) for q in poses])
    prm = LMParams(solver, iters, tol, lam, LOSSES[loss] if isinstance(loss, str) else loss, scale)
    it, tot = C.c_int(), C.c_double()
    rc = L.lgs_pose_graph_optimize_lm(C.byref(prm), p, n, edges_array(edges), len(edges), C.byref(it),
                                      C.byref(tot))
    if rc != 0:
        raise RuntimeError(f"lgs_pose_graph_optimize_lm: status {rc}")
    return np.array([[q.x, q.y, q.theta] for q in p[:n]]), it.value, tot.value, prm.lambda_


def robust_loss(kind, scale, t):
    t = np.ascontiguousarray(t, dtype=np.float64)
    out = np.zeros(2 * len(t))
    rc = load().lgs_robust_loss(LOSSES[kind] if isinstance(kind, str) else kind, scale, _dp(t), len(t), _dp(out))
    if rc != 0:
        raise RuntimeError(f"lgs_robust_loss: status {rc}")
    return out[0::2].copy(), out[1::2].copy()


def save_pose_graph(indices, poses, timestamps, edges, file_name: str):
    n = len(poses)
    idx = (C.c_int * max(1, n))(*indices)
    p = (Pose2D * max(1, n))(*[Pose2D(*q) for q in poses])
    ts = np.ascontiguousarray(timestamps if n else [0.0], dtype=np.float64)
    rc = load().lgs_pose_graph_save(idx, p, _dp(ts), n, edges_array(edges), len(edges), file_name.encode())
    if rc != 0:
        raise RuntimeError(f"lgs_pose_graph_save: status {rc}")


def write_png(file_name: str, rgb: np.ndarray):
    rgb = np.ascontiguousarray(rgb, dtype=np.uint8)
    h, w, _ = rgb.shape
    rc = load().lgs_png_write_rgb8(file_name.encode(), rgb.ctypes.data_as(C.POINTER(C.c_uint8)), w, h)
    if rc != 0:
        raise RuntimeError(f"lgs_png_write_rgb8: status {rc}")


def _options(draw_trajectory, node_min, node_max, scan, scan_pose, save_metadata, keep):
    o = MapSaveOptions()
    o.draw_trajectory, o.trajectory_node_index_min, o.trajectory_node_index_max = int(draw_trajectory), node_min, \
        node_max
    o.save_metadata = int(save_metadata)
    if scan is not None:
        r, a, rel = scan
        r = np.ascontiguousarray(r, dtype=np.float64)
        a = np.ascontiguousarray(a, dtype=np.float64)
        sh = ScanHost(_dp(r), _dp(a), len(r), Pose2D(*rel), 0.0, 1e9)
        keep += [r, a, sh]
        o.draw_scan, o.scan_pose, o.scan = 1, Pose2D(*scan_pose), C.pointer(sh)
    return o


def draw_image(m: "abi.Map", node_poses, draw_trajectory=False, node_min=0, node_max=-1, scan=None,
               scan_pose=(0.0, 0.0, 0.0)):
    """MapSaver::SaveMapCore's image, [h, w, 3] uint8 (PNG row order).
    scan = (ranges, angles, relative sensor pose)"""
    L = load()
    k = len(node_poses)
    p = (Pose2D * max(1, k))(*[Pose2D(*q) for q in node_poses])
    keep = []
    o = _options(draw_trajectory, node_min, node_max if node_max >= 0 else k - 1, scan, scan_pose, False, keep)
    w, h = C.c_int(), C.c_int()
    m.ctx.check(L.lgs_map_draw_image(m.ctx.h, m.h, p, k, C.byref(o), None, 0, C.byref(w), C.byref(h)),
                "map_draw_image")
    img = np.zeros((h.value, w.value, 3), dtype=np.uint8)
    m.ctx.check(L.lgs_map_draw_image(m.ctx.h, m.h, p, k, C.byref(o), img.ctypes.data_as(C.POINTER(C.c_uint8)),
                                     img.size, C.byref(w), C.byref(h)), "map_draw_image")
    return img


def save_map(m: "abi.Map", node_poses, file_name: str, draw_trajectory=False, node_min=0, node_max=-1,
             scan=None, scan_pose=(0.0, 0.0, 0.0), save_metadata=True):
    L = load()
    k = len(node_poses)
    p = (Pose2D * max(1, k))(*[Pose2D(*q) for q in node_poses])
    keep = []
    o = _options(draw_trajectory, node_min, node_max if node_max >= 0 else k - 1, scan, scan_pose, save_metadata,
                 keep)
    m.ctx.check(L.lgs_map_save(m.ctx.h, m.h, p, k, C.byref(o), file_name.encode()), "map_save")


def read_png_rgb8(path: str) -> np.ndarray:
    """Decode an 8-bit RGB, non-interlaced PNG (filters 0-4) -> [h, w, 3] (test helper)"""
    import struct
    import zlib
    data = open(path, "rb").read()
    assert data[:8] == b"\x89PNG\r\n\x1a\n"
    pos, idat, w, h = 8, b"", 0, 0
    while pos < len(data):
        ln, typ = struct.unpack(">I4s", data[pos:pos + 8])
        body = data[pos + 8:pos + 8 + ln]
        crc = struct.unpack(">I", data[pos + 8 + ln:pos + 12 + ln])[0]
        assert zlib.crc32(typ + body) & 0xFFFFFFFF == crc, typ
        if typ == b"IHDR":
            w, h, bd, ct, _, _, il = struct.unpack(">IIBBBBB", body)
            assert (bd, ct, il) == (8, 2, 0)
        elif typ == b"IDAT":
            idat += body
        pos += 12 + ln
    raw = np.frombuffer(zlib.decompress(idat), dtype=np.uint8).reshape(h, 1 + 3 * w)
    out = np.zeros((h, 3 * w), dtype=np.int32)
    prev = np.zeros(3 * w, dtype=np.int32)
    for y in range(h):
        f, line = raw[y, 0], raw[y, 1:].astype(np.int32)
        if f == 0:
            out[y], prev = line, line
            continue
        cur = np.zeros(3 * w, dtype=np.int32)
        for i in range(3 * w):
            a = cur[i - 3] if i >= 3 else 0
            b = prev[i]
            c = prev[i - 3] if i >= 3 else 0
            if f == 0:
                pr = 0
            elif f == 1:
                pr = a
            elif f == 2:
                pr = b
            elif f == 3:
                pr = (a + b) // 2
            else:
                p = a + b - c
                pa, pb, pc = abs(p - a), abs(p - b), abs(p - c)
                pr = a if (pa <= pb and pa <= pc) else (b if pb <= pc else c)
            cur[i] = (line[i] + pr) & 0xFF
        out[y], prev = cur, cur
    return out.reshape(h, w, 3).astype(np.uint8)
