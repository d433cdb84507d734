"""ctypes binding of the CPU oracle (oracle/build/liblgs_oracle.so).

TEST INFRASTRUCTURE ONLY: the oracle is the parity checker, never the thing
measured or shipped.  Only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg load it.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_SO = os.path.join(ROOT, "oracle", "build", "liblgs_oracle.so")


class Pose(C.Structure):
    _fields_ = [("x", C.c_double), ("y", C.c_double), ("theta", C.c_double)]


class Scan(C.Structure):
    _fields_ = [("ranges", C.POINTER(C.c_double)), ("angles", C.POINTER(C.c_double)), ("n", C.c_int),
                ("rel_sensor_pose", Pose), ("min_range", C.c_double), ("max_range", C.c_double)]


class CostGE(C.Structure):
    _fields_ = [("usable_range_min", C.c_double), ("usable_range_max", C.c_double),
                ("hit_and_missed_dist", C.c_double), ("occupancy_threshold", C.c_double),
                ("kernel_size", C.c_int), ("scaling_factor", C.c_double), ("standard_deviation", C.c_double)]


class RtcsmParams(C.Structure):
    _fields_ = [("low_resolution", C.c_int), ("range_x", C.c_double), ("range_y", C.c_double),
                ("range_theta", C.c_double), ("scan_range_max", C.c_double)]


class Grid(C.Structure):
    _fields_ = [("cells", C.POINTER(C.c_double)), ("w", C.c_int), ("h", C.c_int),
                ("min_x", C.c_double), ("min_y", C.c_double), ("res", C.c_double)]


class Summary(C.Structure):
    _fields_ = [("pose_found", C.c_int), ("normalized_cost", C.c_double), ("initial_pose", Pose),
                ("estimated_pose", Pose), ("covariance", C.c_double * 9), ("score_max", C.c_double),
                ("score_threshold", C.c_double), ("best_win", C.c_int * 3), ("win", C.c_int * 3),
                ("steps", C.c_double * 3), ("sensor_pose", Pose), ("best_sensor_pose", Pose),
                ("coarse_evals", C.c_int64), ("fine_blocks", C.c_int64)]


class Map(C.Structure):
    _fields_ = [("res", C.c_double), ("patch_size", C.c_int), ("npx", C.c_int), ("npy", C.c_int),
                ("w", C.c_int), ("h", C.c_int), ("min_x", C.c_double), ("min_y", C.c_double),
                ("cells", C.POINTER(C.c_double)), ("hit_count", C.POINTER(C.c_uint32)),
                ("miss_count", C.POINTER(C.c_uint32)), ("patch_alloc", C.POINTER(C.c_uint8))]


class Node(C.Structure):
    _fields_ = [("pose", Pose), ("scan", Scan)]


class BuilderParams(C.Structure):
    _fields_ = [("usable_range_min", C.c_double), ("usable_range_max", C.c_double),
                ("prob_hit", C.c_double), ("prob_miss", C.c_double)]


class LinsolveParams(C.Structure):
    _fields_ = [("num_iterations_max", C.c_int), ("convergence_threshold", C.c_double),
                ("usable_range_min", C.c_double), ("usable_range_max", C.c_double),
                ("translation_regularizer", C.c_double), ("rotation_regularizer", C.c_double),
                ("cost_usable_range_min", C.c_double), ("cost_usable_range_max", C.c_double)]


class BBParams(C.Structure):
    _fields_ = [("node_height_max", C.c_int), ("range_x", C.c_double), ("range_y", C.c_double),
                ("range_theta", C.c_double), ("scan_range_max", C.c_double),
                ("score_usable_range_min", C.c_double), ("score_usable_range_max", C.c_double)]


_D = C.POINTER(C.c_double)
_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(ORACLE_SO):
            raise RuntimeError(f"oracle not built: {ORACLE_SO}")
        L = C.CDLL(ORACLE_SO)
        L.orc_compound.restype = Pose
        L.orc_compound.argtypes = [Pose, Pose]
        L.orc_inverse_compound.restype = Pose
        L.orc_inverse_compound.argtypes = [Pose, Pose]
        L.orc_move_backward.restype = Pose
        L.orc_move_backward.argtypes = [Pose, Pose]
        L.orc_sliding_window_max.argtypes = [_D, C.c_int, _D, C.c_int, C.c_int, C.c_int]
        L.orc_bresenham.restype = C.c_int
        L.orc_bresenham.argtypes = [C.c_int] * 4 + [C.POINTER(C.c_int), C.c_int]
        L.orc_precompute_grid_map.argtypes = [_D, C.c_int, C.c_int, C.c_int, _D]
        L.orc_bayes_update.restype = C.c_double
        L.orc_scan_interpolate.restype = C.c_int
        L.orc_scan_interpolate.argtypes = [_D, _D, C.c_int, C.c_double, C.c_double, _D, _D, C.c_int]
        L.orc_bayes_update.argtypes = [C.c_double, C.c_double]
        L.orc_rtcsm_search_step.argtypes = [C.c_double, C.POINTER(Scan), C.c_double, _D, _D, _D]
        L.orc_rtcsm_scan_indices.restype = C.c_int
        L.orc_rtcsm_scan_indices.argtypes = [C.POINTER(Grid), Pose, C.POINTER(Scan), C.c_double,
                                             C.POINTER(C.c_int)]
        L.orc_rtcsm_optimize_pose.restype = C.c_int
        L.orc_rtcsm_optimize_pose.argtypes = [C.POINTER(Grid), C.POINTER(Grid), C.POINTER(RtcsmParams),
                                              C.POINTER(CostGE), C.POINTER(Scan), Pose, C.c_double,
                                              C.POINTER(Summary)]
        L.orc_rtcsm_optimize_pose_query.restype = C.c_int
        L.orc_rtcsm_optimize_pose_query.argtypes = [C.POINTER(Grid), C.POINTER(RtcsmParams), C.POINTER(CostGE),
                                                    C.POINTER(Scan), Pose, C.POINTER(Summary)]
        L.orc_rtcsm_dense_scores.restype = C.c_int
        L.orc_rtcsm_dense_scores.argtypes = [C.POINTER(Grid), C.POINTER(Grid), C.POINTER(RtcsmParams),
                                             C.POINTER(Scan), Pose, _D, _D, C.POINTER(C.c_int)]
        L.orc_cost_ge_cost.restype = C.c_double
        L.orc_cost_ge_cost.argtypes = [C.POINTER(Grid), C.POINTER(CostGE), C.POINTER(Scan), Pose]
        L.orc_cost_ge_covariance.argtypes = [C.POINTER(Grid), C.POINTER(CostGE), C.POINTER(Scan), Pose, _D]
        L.orc_map_init.restype = C.c_int
        L.orc_map_init.argtypes = [C.POINTER(Map), C.c_double, C.c_int, C.c_int, C.c_int, C.c_double,
                                   C.c_double]
        L.orc_map_free.argtypes = [C.POINTER(Map)]
        L.orc_map_resize.argtypes = [C.POINTER(Map)] + [C.c_double] * 4
        L.orc_map_expand.argtypes = [C.POINTER(Map)] + [C.c_double] * 5
        L.orc_construct_map_from_scans.restype = C.c_int
        L.orc_construct_map_from_scans.argtypes = [C.POINTER(Map), C.POINTER(Node), C.c_int,
                                                   C.POINTER(BuilderParams)]
        L.orc_integrate_scan.restype = C.c_int
        L.orc_integrate_scan.argtypes = [C.POINTER(Map), Pose, C.POINTER(Scan), C.POINTER(BuilderParams)]
        L.orc_map_actual_size.restype = C.c_int
        L.orc_map_actual_size.argtypes = [C.POINTER(Map), C.POINTER(C.c_int)]
        L.orc_map_draw_image.restype = C.c_int
        L.orc_map_draw_image.argtypes = [C.POINTER(Map), C.POINTER(Pose), C.c_int, C.c_int, C.c_int, C.c_int,
                                         C.POINTER(Scan), Pose, C.POINTER(C.c_uint8), C.POINTER(C.c_int),
                                         C.POINTER(C.c_int)]
        L.orc_sq_smoothed_value.restype = C.c_double
        L.orc_sq_smoothed_value.argtypes = [C.POINTER(Grid), C.c_double, C.c_double]
        L.orc_sq_cost.restype = C.c_double
        L.orc_sq_cost.argtypes = [C.POINTER(Grid), C.c_double, C.c_double, C.POINTER(Scan), Pose]
        L.orc_linsolve_step.restype = Pose
        L.orc_linsolve_step.argtypes = [C.POINTER(Grid), C.POINTER(LinsolveParams), C.POINTER(Scan), Pose]
        L.orc_sq_covariance.restype = None
        L.orc_sq_covariance.argtypes = [C.POINTER(Grid), C.c_double, C.c_double, C.POINTER(Scan), Pose,
                                        C.POINTER(C.c_double)]
        L.orc_linsolve_optimize_pose.restype = C.c_int
        L.orc_linsolve_optimize_pose.argtypes = [C.POINTER(Grid), C.POINTER(LinsolveParams), C.POINTER(Scan),
                                                 Pose, C.POINTER(Summary), C.POINTER(Pose)]
        L.orc_solve3_colpiv_qr.argtypes = [_D, _D, _D]
        L.orc_pixel_accurate_score.restype = C.c_double
        L.orc_pixel_accurate_score.argtypes = [C.POINTER(Grid), C.POINTER(BBParams), C.POINTER(Scan), Pose]
        L.orc_precompute_grid_maps.argtypes = [_D, C.c_int, C.c_int, C.c_int, C.POINTER(_D)]
        L.orc_bb_optimize_pose.restype = C.c_int
        L.orc_bb_optimize_pose.argtypes = [C.POINTER(Grid), C.POINTER(Grid), C.POINTER(BBParams),
                                           C.POINTER(CostGE), C.POINTER(Scan), Pose, C.c_double,
                                           C.POINTER(Summary)]
        L.orc_bb_optimize_pose_query.restype = C.c_int
        L.orc_bb_optimize_pose_query.argtypes = [C.POINTER(Grid), C.POINTER(BBParams), C.POINTER(CostGE),
                                                 C.POINTER(Scan), Pose, C.POINTER(Summary)]
        _lib = L
    return _lib


def dp(a):
    return a.ctypes.data_as(_D)


class OScan:
    """Keeps numpy buffers alive behind an oracle Scan struct."""

    def __init__(self, ranges, angles, rel=(0.0, 0.0, 0.0), min_range=0.0, max_range=30.0):
        self.r = np.ascontiguousarray(ranges, dtype=np.float64)
        self.a = np.ascontiguousarray(angles, dtype=np.float64)
        self.s = Scan(dp(self.r), dp(self.a), len(self.r), Pose(*rel), min_range, max_range)


class OGrid:
    def __init__(self, cells, min_x, min_y, res):
        self.c = np.ascontiguousarray(cells, dtype=np.float64)
        h, w = self.c.shape
        self.g = Grid(dp(self.c), w, h, min_x, min_y, res)


def precompute(cells, win):
    c = np.ascontiguousarray(cells, dtype=np.float64)
    h, w = c.shape
    out = np.zeros_like(c)
    lib().orc_precompute_grid_map(dp(c), w, h, int(win), dp(out))
    return out


def scan_interpolate(ranges, angles, dist_scans, dist_empty):
    """ScanInterpolator::Interpolate -> (ranges, angles) arrays."""
    r = np.ascontiguousarray(ranges, dtype=np.float64)
    a = np.ascontiguousarray(angles, dtype=np.float64)
    cap = 4 * len(r) + 16
    while True:
        orr, oa = np.zeros(cap), np.zeros(cap)
        m = lib().orc_scan_interpolate(dp(r), dp(a), len(r), dist_scans, dist_empty, dp(orr), dp(oa), cap)
        if m <= cap:
            return orr[:m], oa[:m]
        cap = m


def precompute_pyramid(cells, node_height_max):
    """PrecomputeGridMaps: [window-max map with window 2^h for h = 0..H]"""
    c = np.ascontiguousarray(cells, dtype=np.float64)
    h, w = c.shape
    outs = [np.zeros_like(c) for _ in range(node_height_max + 1)]
    ptrs = (_D * len(outs))(*[dp(o) for o in outs])
    lib().orc_precompute_grid_maps(dp(c), w, h, int(node_height_max), ptrs)
    return outs


def bresenham(x0, y0, x1, y1):
    cap = max(abs(x1 - x0), abs(y1 - y0)) + 2
    buf = (C.c_int * (2 * cap))()
    n = lib().orc_bresenham(x0, y0, x1, y1, buf, cap)
    return [(buf[2 * i], buf[2 * i + 1]) for i in range(n)]


class OMap:
    """orc_map with the reference's patch geometry."""

    def __init__(self, res, patch_size, ncx, ncy, center=(0.0, 0.0)):
        self.m = Map()
        rc = lib().orc_map_init(C.byref(self.m), res, patch_size, ncx, ncy, center[0], center[1])
        assert rc == 0

    def cells(self):
        m = self.m
        return np.ctypeslib.as_array(m.cells, shape=(m.h, m.w)).copy()

    def hits(self):
        m = self.m
        return np.ctypeslib.as_array(m.hit_count, shape=(m.h, m.w)).copy()

    def misses(self):
        m = self.m
        return np.ctypeslib.as_array(m.miss_count, shape=(m.h, m.w)).copy()

    def geometry(self):
        m = self.m
        return dict(w=m.w, h=m.h, min_x=m.min_x, min_y=m.min_y, npx=m.npx, npy=m.npy)

    def patches(self):
        """Patch::IsAllocated per patch, [npy, npx]"""
        m = self.m
        return np.ctypeslib.as_array(m.patch_alloc, shape=(m.npy, m.npx)).copy()

    def actual_size(self):
        """GridMap::ComputeActualMapSize -> (count, 12 ints)"""
        out = (C.c_int * 12)()
        n = lib().orc_map_actual_size(C.byref(self.m), out)
        return n, list(out)

    def draw_image(self, node_poses, draw_trajectory=False, node_min=0, node_max=-1, scan=None,
                   scan_pose=(0.0, 0.0, 0.0)):
        """MapSaver::SaveMapCore's image (flipped), [h, w, 3] uint8, or None"""
        n, a = self.actual_size()
        if n == 0:
            return None
        k = len(node_poses)
        nodes = (Pose * max(1, k))(*[Pose(*p) for p in node_poses])
        buf = np.zeros(a[10] * a[11] * 3, dtype=np.uint8)
        w, h = C.c_int(), C.c_int()
        rc = lib().orc_map_draw_image(C.byref(self.m), nodes, k, int(draw_trajectory), node_min,
                                      node_max if node_max >= 0 else k - 1,
                                      C.byref(scan.s) if scan is not None else None, Pose(*scan_pose),
                                      buf.ctypes.data_as(C.POINTER(C.c_uint8)), C.byref(w), C.byref(h))
        assert rc == 0
        return buf.reshape(h.value, w.value, 3)

    def integrate(self, pose, oscan: OScan, bp: BuilderParams):
        lib().orc_integrate_scan(C.byref(self.m), Pose(*pose), C.byref(oscan.s), C.byref(bp))

    def construct(self, poses, oscans, bp: BuilderParams):
        n = len(poses)
        nodes = (Node * n)(*[Node(Pose(*p), s.s) for p, s in zip(poses, oscans)])
        lib().orc_construct_map_from_scans(C.byref(self.m), nodes, n, C.byref(bp))

    def __del__(self):
        try:
            lib().orc_map_free(C.byref(self.m))
        except Exception:
            pass
