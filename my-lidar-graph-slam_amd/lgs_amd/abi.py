"""ctypes binding of the C-ABI in include/lgs_hip.h (liblgs_hip.so).

This is plumbing for tests and bench.py: every compute call goes through the
HIP library.  There is no CPU fallback -- if liblgs_hip.so is missing or no
device is present, the calls raise.
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Optional, Sequence

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "liblgs_hip.so")

LGS_OK = 0
LGS_OPT_GUARD_EPS = 1
LGS_OPT_FORCE_DENSE = 2
LGS_OPT_INJECT_INDEX = 3
LGS_OPT_GUARD_CAP = 4
LGS_OPT_PROFILE = 5
LGS_OPT_PROFILE_MASK = 7
LGS_OPT_SPIN_SYNC = 8
LGS_OPT_SUPER_PRUNE = 9
LGS_OPT_LANES_MIN_BATCH = 11
LGS_OPT_RAY_CHUNK_KEYS = 13
LGS_OPT_POISON_WS = 15   # diagnostics only
LGS_OPT_SKIP_MASK = 10   # diagnostics only
LGS_OPT_LINSOLVE_SPLIT = 17
LGS_OPT_HANDOFF_SPIN_US = 18
LGS_OPT_PEER_COPY = 19
LGS_OPT_PRUNE_MIN_SUPER = 21
LGS_OPT_COOP_TILES = 22
LGS_OPT_SORT_BARRIER_US = 23
LGS_OPT_FINE_STAGED = 24
LGS_OPT_SMALL_WINDOW = 25
LGS_OPT_POST_RECORDS = 26
LGS_OPT_FUSED_PLANES = 27
LGS_OPT_PRIORITY_TAIL = 28
LGS_OPT_HV_FULL = 29
LGS_OPT_SPLIT_CHUNKS = 30
LGS_OPT_DEVICE_HITS = 31
LGS_OPT_SEED_WIDE = 32
LGS_OPT_ZERO_TILES = 33
LGS_OPT_DEVICE_TIMING = 34   # correlative chunks' kernels timed on the device (s_memrealtime spans)
LGS_OPT_LEAN_PROJECT = 35    # batched chunks: only superblock bases projected; consumers form their rows
KERNEL_IDS = ["k_project", "k_coarse", "k_seed", "k_select", "k_fine", "k_replay", "k_cost", "k_precompute",
              "k_linsolve", "k_ray_emit", "k_ray_apply", "k_super", "k_super_planes", "k_bb_score",
              "k_bb_expand", "k_coarse_aux", "k_match_small"]   # lgs_ctx_kernel_stats order


class Pose2D(C.Structure):
    _fields_ = [("x", C.c_double), ("y", C.c_double), ("theta", C.c_double)]

    def tuple(self):
        return (self.x, self.y, self.theta)


class ScanHost(C.Structure):
    _fields_ = [
        ("ranges", C.POINTER(C.c_double)),
        ("angles", C.POINTER(C.c_double)),
        ("n", C.c_int),
        ("rel_sensor_pose", Pose2D),
        ("min_range", C.c_double),
        ("max_range", C.c_double),
    ]


class RtcsmParams(C.Structure):
    _fields_ = [
        ("low_resolution", C.c_int),
        ("range_x", C.c_double),
        ("range_y", C.c_double),
        ("range_theta", C.c_double),
        ("scan_range_max", C.c_double),
    ]


class CostGEParams(C.Structure):
    _fields_ = [
        ("usable_range_min", C.c_double),
        ("usable_range_max", C.c_double),
        ("hit_and_missed_dist", C.c_double),
        ("occupancy_threshold", C.c_double),
        ("kernel_size", C.c_int),
        ("scaling_factor", C.c_double),
        ("standard_deviation", C.c_double),
    ]


class RtcsmSummary(C.Structure):
    _fields_ = [
        ("pose_found", C.c_int),
        ("normalized_cost", C.c_double),
        ("initial_pose", Pose2D),
        ("estimated_pose", Pose2D),
        ("covariance", C.c_double * 9),
        ("score_max", C.c_double),
        ("score_threshold", C.c_double),
        ("best_win", C.c_int * 3),
        ("win", C.c_int * 3),
        ("steps", C.c_double * 3),
        ("best_sensor_pose", Pose2D),
        ("coarse_blocks", C.c_int64),
        ("fine_blocks", C.c_int64),
        ("guard_hits", C.c_int),
        ("fixups", C.c_int),
        ("slow_path", C.c_int),
    ]


class BBParams(C.Structure):
    """lgs_bb_params: ScanMatcherBranchBound ctor (nodeHeightMax, rangeX/Y/Theta,
    scanRangeMax) + ScorePixelAccurate (usableRangeMin/Max)."""
    _fields_ = [("node_height_max", C.c_int), ("range_x", C.c_double), ("range_y", C.c_double),
                ("range_theta", C.c_double), ("scan_range_max", C.c_double),
                ("score_usable_range_min", C.c_double), ("score_usable_range_max", C.c_double)]


class BuilderParams(C.Structure):
    _fields_ = [("usable_range_min", C.c_double), ("usable_range_max", C.c_double),
                ("prob_hit", C.c_double), ("prob_miss", C.c_double)]


class MapGeometry(C.Structure):
    _fields_ = [("resolution", C.c_double), ("patch_size", C.c_int), ("num_patches_x", C.c_int),
                ("num_patches_y", C.c_int), ("num_cells_x", C.c_int), ("num_cells_y", C.c_int),
                ("min_x", C.c_double), ("min_y", C.c_double)]

    def dict(self):
        return dict(w=self.num_cells_x, h=self.num_cells_y, min_x=self.min_x, min_y=self.min_y,
                    npx=self.num_patches_x, npy=self.num_patches_y)

    def res(self):
        return self.resolution


class LinsolveParams(C.Structure):
    """lgs_linsolve_params: ScanMatcherLinearSolver ctor order, then CostSquareError's usable range."""
    _fields_ = [("num_iterations_max", C.c_int), ("convergence_threshold", C.c_double),
                ("usable_range_min", C.c_double), ("usable_range_max", C.c_double),
                ("translation_regularizer", C.c_double), ("rotation_regularizer", C.c_double),
                ("cost_usable_range_min", C.c_double), ("cost_usable_range_max", C.c_double)]


class LinsolveSummary(C.Structure):
    _fields_ = [("pose_found", C.c_int), ("iterations", C.c_int), ("normalized_cost", C.c_double),
                ("initial_pose", Pose2D), ("estimated_pose", Pose2D), ("covariance", C.c_double * 9),
                ("sensor_pose", Pose2D), ("best_sensor_pose", Pose2D), ("cost", C.c_double)]


class LoopQuery(C.Structure):
    _fields_ = [("map", C.c_void_p), ("coarse", C.c_void_p), ("local_map_node_pose", Pose2D),
                ("local_map_node_index", C.c_int), ("first_candidate", C.c_int), ("num_candidates", C.c_int)]


class LoopCandidate(C.Structure):
    _fields_ = [("scan", C.c_void_p), ("node_pose", Pose2D), ("node_index", C.c_int), ("pad", C.c_int)]


class LoopResult(C.Structure):
    _fields_ = [("found", C.c_int), ("start_node_index", C.c_int), ("end_node_index", C.c_int), ("pad", C.c_int),
                ("relative_pose", Pose2D), ("start_node_pose", Pose2D), ("estimated_pose", Pose2D),
                ("covariance", C.c_double * 9), ("score", C.c_double), ("normalized_cost", C.c_double)]


LOOP_RESULT_DOUBLES = 22   # sizeof(lgs_loop_result) / 8


class KernelStat(C.Structure):
    _fields_ = [("name", C.c_char * 32), ("launches", C.c_int64), ("total_ms", C.c_double),
                ("algo_bytes", C.c_double), ("dispatch_ms", C.c_double)]


# (name, restype, argtypes) for every symbol of include/lgs_hip.h
_P = C.c_void_p
_PROTOS = [
    ("lgs_abi_version", C.c_int, []),
    ("lgs_ctx_create", C.c_int, [C.c_int, C.POINTER(_P)]),
    ("lgs_ctx_destroy", None, [_P]),
    ("lgs_ctx_last_error", C.c_char_p, [_P]),
    ("lgs_ctx_synchronize", C.c_int, [_P]),
    ("lgs_ctx_stream", _P, [_P]),
    ("lgs_ctx_set_option", C.c_int, [_P, C.c_int, C.c_double]),
    ("lgs_ctx_kernel_stats", C.c_int, [_P, C.POINTER(KernelStat), C.c_int]),
    ("lgs_ctx_reset_stats", C.c_int, [_P]),
    ("lgs_ctx_match_counters", C.c_int, [_P, C.POINTER(C.c_int64)]),
    ("lgs_grid_create", C.c_int, [_P, C.c_int, C.c_int, C.c_double, C.c_double, C.c_double, C.POINTER(_P)]),
    ("lgs_grid_wrap", C.c_int, [_P, _P, C.c_int, C.c_int, C.c_double, C.c_double, C.c_double, C.POINTER(_P)]),
    ("lgs_grid_destroy", None, [_P]),
    ("lgs_grid_upload", C.c_int, [_P, _P, C.POINTER(C.c_double)]),
    ("lgs_grid_upload_patches", C.c_int, [_P, _P, C.POINTER(_P), C.c_int, C.c_int, C.c_int, C.c_int, C.c_int]),
    ("lgs_grid_download", C.c_int, [_P, _P, C.POINTER(C.c_double)]),
    ("lgs_grid_fill", C.c_int, [_P, _P, C.c_double]),
    ("lgs_grid_info", C.c_int, [_P, C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_double),
                                 C.POINTER(C.c_double), C.POINTER(C.c_double)]),
    ("lgs_grid_device_ptr", _P, [_P]),
    ("lgs_grid_precompute_max", C.c_int, [_P, _P, C.c_int, _P]),
    ("lgs_scan_create", C.c_int, [_P, C.POINTER(ScanHost), C.POINTER(_P)]),
    ("lgs_scan_destroy", None, [_P]),
    ("lgs_rtcsm_optimize_pose", C.c_int, [_P, _P, _P, C.POINTER(RtcsmParams), C.POINTER(CostGEParams), _P,
                                          Pose2D, C.c_double, C.POINTER(RtcsmSummary)]),
    ("lgs_rtcsm_optimize_pose_query", C.c_int, [_P, _P, C.POINTER(RtcsmParams), C.POINTER(CostGEParams), _P,
                                                Pose2D, C.POINTER(RtcsmSummary)]),
    ("lgs_rtcsm_optimize_pose_query_batch", C.c_int, [_P, C.POINTER(_P), C.POINTER(RtcsmParams),
                                                      C.POINTER(CostGEParams), C.POINTER(_P), C.POINTER(Pose2D),
                                                      C.c_int, C.POINTER(RtcsmSummary)]),
    ("lgs_rtcsm_optimize_pose_batch", C.c_int, [_P, _P, _P, C.POINTER(RtcsmParams), C.POINTER(CostGEParams),
                                                C.POINTER(_P), C.POINTER(Pose2D), C.c_int, C.c_double,
                                                C.POINTER(RtcsmSummary)]),
    ("lgs_rtcsm_dense_scores", C.c_int, [_P, _P, _P, C.POINTER(RtcsmParams), _P, Pose2D,
                                         C.POINTER(C.c_double), C.POINTER(C.c_double), C.POINTER(C.c_int)]),
    ("lgs_cost_greedy_endpoint", C.c_int, [_P, _P, C.POINTER(CostGEParams), _P, Pose2D,
                                           C.POINTER(C.c_double)]),
    ("lgs_scan_get", C.c_int, [_P, C.POINTER(C.c_int), C.POINTER(C.c_double), C.POINTER(C.c_double)]),
    ("lgs_scan_interpolate", C.c_int, [_P, _P, C.c_double, C.c_double, C.POINTER(_P)]),
    ("lgs_map_create", C.c_int, [_P, C.c_double, C.c_int, C.c_int, C.c_int, C.c_double, C.c_double,
                                 C.POINTER(_P)]),
    ("lgs_map_destroy", None, [_P]),
    ("lgs_map_get_geometry", C.c_int, [_P, C.POINTER(MapGeometry)]),
    ("lgs_map_grid", C.c_int, [_P, C.POINTER(_P)]),
    ("lgs_map_update_scan", C.c_int, [_P, _P, _P, Pose2D, C.POINTER(BuilderParams)]),
    ("lgs_map_construct_from_scans", C.c_int, [_P, _P, C.POINTER(_P), C.POINTER(Pose2D), C.c_int,
                                               C.POINTER(BuilderParams)]),
    ("lgs_map_append_scan", C.c_int, [_P, _P, _P, C.POINTER(_P), C.POINTER(Pose2D), C.c_int,
                                      C.POINTER(BuilderParams)]),
    ("lgs_maps_construct_from_scans", C.c_int, [_P, C.POINTER(_P), C.POINTER(C.c_int), C.POINTER(C.c_int),
                                                C.c_int, C.POINTER(_P), C.POINTER(Pose2D), C.c_int,
                                                C.POINTER(BuilderParams)]),
    ("lgs_map_construct_global", C.c_int, [_P, C.c_double, C.c_int, C.POINTER(_P), C.POINTER(Pose2D), C.c_int,
                                           C.POINTER(BuilderParams), C.POINTER(_P)]),
    ("lgs_map_render_gray", C.c_int, [_P, _P, C.POINTER(C.c_uint8)]),
    ("lgs_map_render_gray_region", C.c_int, [_P, _P, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                             C.POINTER(C.c_uint8)]),
    ("lgs_map_download_patches", C.c_int, [_P, _P, C.POINTER(C.c_uint8)]),
    ("lgs_map_actual_size", C.c_int, [_P, _P, C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    ("lgs_map_download", C.c_int, [_P, _P, C.POINTER(C.c_double), C.POINTER(C.c_uint32),
                                   C.POINTER(C.c_uint32)]),
    ("lgs_grid_precompute_pyramid", C.c_int, [_P, _P, C.c_int, C.POINTER(_P)]),
    ("lgs_bb_optimize_pose_batch", C.c_int, [_P, _P, C.POINTER(_P), C.POINTER(BBParams), C.POINTER(CostGEParams),
                                             C.POINTER(_P), C.POINTER(Pose2D), C.c_int, C.c_double,
                                             C.POINTER(RtcsmSummary)]),
    ("lgs_bb_optimize_pose_query", C.c_int, [_P, _P, C.POINTER(BBParams), C.POINTER(CostGEParams), _P, Pose2D,
                                             C.POINTER(RtcsmSummary)]),
    ("lgs_loop_detect_bb", C.c_int, [_P, C.POINTER(BBParams), C.POINTER(CostGEParams), C.c_double,
                                     C.POINTER(LoopQuery), C.c_int, C.POINTER(LoopCandidate), C.c_int,
                                     C.POINTER(LoopResult)]),
    ("lgs_loop_detect_rtcsm", C.c_int, [_P, C.POINTER(RtcsmParams), C.POINTER(CostGEParams), C.c_double,
                                        C.POINTER(LoopQuery), C.c_int, C.POINTER(LoopCandidate), C.c_int,
                                        C.POINTER(LoopResult)]),
    ("lgs_loop_detect_rtcsm_multi", C.c_int, [C.POINTER(_P), C.c_int, C.POINTER(RtcsmParams),
                                              C.POINTER(CostGEParams), C.c_double, C.POINTER(LoopQuery), C.c_int,
                                              C.POINTER(LoopCandidate), C.c_int, C.POINTER(LoopResult)]),
    ("lgs_loop_shard_bounds", C.c_int, [C.c_int, C.c_int, C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    ("lgs_loop_records_allgather", C.c_int, [_P, _P, C.c_int, C.c_int, C.c_int, C.POINTER(LoopResult),
                                             C.POINTER(LoopResult)]),
    ("lgs_rccl_unique_id", C.c_int, [C.POINTER(C.c_ubyte)]),
    ("lgs_rccl_comm_init", C.c_int, [_P, C.POINTER(C.c_ubyte), C.c_int, C.c_int, C.POINTER(_P)]),
    ("lgs_rccl_comm_destroy", C.c_int, [_P]),
    ("lgs_linsolve_optimize_pose", C.c_int, [_P, _P, C.POINTER(LinsolveParams), _P, Pose2D,
                                             C.POINTER(LinsolveSummary), C.POINTER(C.c_double)]),
    ("lgs_linsolve_optimize_pose_batch", C.c_int, [_P, _P, C.POINTER(LinsolveParams), C.POINTER(_P),
                                                   C.POINTER(Pose2D), C.c_int, C.POINTER(LinsolveSummary)]),
    ("lgs_cost_square_error", C.c_int, [_P, _P, C.c_double, C.c_double, _P, Pose2D, C.POINTER(C.c_double),
                                        C.POINTER(C.c_double)]),
    ("lgs_debug_keysort", C.c_int, [_P, _P, _P, C.c_longlong, C.c_int, C.c_int]),
    ("lgs_debug_map_rebuilds", C.c_int, [_P, C.POINTER(C.c_longlong), C.POINTER(C.c_longlong)]),
    ("lgs_debug_copy_counters", C.c_int, [_P, C.POINTER(C.c_longlong), C.POINTER(C.c_longlong)]),
    ("lgs_debug_offset_checks", C.c_int, [_P, C.c_int, C.POINTER(C.c_ulonglong)]),
    ("lgs_debug_item_buffer", C.c_int, [_P, C.c_int, C.c_int, _P, C.c_size_t, C.POINTER(C.c_size_t)]),
    ("lgs_debug_libm", C.c_int, [_P, C.c_int, _P, C.c_int, _P]),
]

SYMBOLS = [p[0] for p in _PROTOS]

_lib: Optional[C.CDLL] = None


def load(path: str = None) -> C.CDLL:
    """Load liblgs_hip.so and bind prototypes.  Raises if missing (no fallback).
    LGS_LIB overrides the path (A/B builds of the same library, tools/ab_build.sh)."""
    global _lib
    if _lib is not None:
        return _lib
    path = path or os.environ.get("LGS_LIB") or LIB_PATH
    if not os.path.exists(path):
        raise RuntimeError(f"HIP extension missing: {path} (run __graft_entry__.build())")
    lib = C.CDLL(path)
    for name, res, args in _PROTOS:
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def dptr(a: np.ndarray):
    assert a.dtype == np.float64 and a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(C.POINTER(C.c_double))


class LgsError(RuntimeError):
    pass


class Context:
    """One lgs_ctx: a device + HIP stream + scratch arena."""

    def __init__(self, device: int = 0):
        self.lib = load()
        h = _P()
        rc = self.lib.lgs_ctx_create(device, C.byref(h))
        if rc != LGS_OK:
            raise LgsError(f"lgs_ctx_create(device={device}) failed with status {rc}")
        self.h = h
        # A/B runs: LGS_CTX_OPTIONS="ID=VALUE,ID=VALUE" applied to every new context
        for kv in filter(None, os.environ.get("LGS_CTX_OPTIONS", "").split(",")):
            k, v = kv.split("=")
            self.set_option(int(k), float(v))

    def check(self, rc: int, what: str):
        if rc != LGS_OK:
            msg = self.lib.lgs_ctx_last_error(self.h)
            raise LgsError(f"{what}: status {rc}: {msg.decode() if msg else ''}")

    def set_option(self, opt: int, value: float):
        self.check(self.lib.lgs_ctx_set_option(self.h, opt, float(value)), "set_option")

    def kernel_stats(self) -> dict:
        """{name: dict(launches, total_ms, algo_bytes)} since the last reset."""
        buf = (KernelStat * len(KERNEL_IDS))()
        n = self.lib.lgs_ctx_kernel_stats(self.h, buf, len(KERNEL_IDS))
        if n < 0:
            self.check(-n, "kernel_stats")
        return {buf[i].name.decode(): dict(launches=buf[i].launches, total_ms=buf[i].total_ms,
                                           algo_bytes=buf[i].algo_bytes, dispatch_ms=buf[i].dispatch_ms)
                for i in range(n)}

    def reset_stats(self):
        self.check(self.lib.lgs_ctx_reset_stats(self.h), "reset_stats")

    def match_counters(self) -> dict:
        """matches / coarse blocks scored / dense coarse blocks / pruned matches
        since the last reset_stats (lgs_ctx_match_counters)"""
        buf = (C.c_int64 * 4)()
        self.check(self.lib.lgs_ctx_match_counters(self.h, buf), "match_counters")
        return dict(matches=buf[0], coarse_blocks=buf[1], coarse_blocks_dense=buf[2], pruned=buf[3])

    def synchronize(self):
        self.check(self.lib.lgs_ctx_synchronize(self.h), "synchronize")

    def close(self):
        if getattr(self, "h", None):
            self.lib.lgs_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- grids ----
    def grid(self, w: int, h: int, min_x: float, min_y: float, res: float) -> "Grid":
        g = _P()
        self.check(self.lib.lgs_grid_create(self.h, w, h, min_x, min_y, res, C.byref(g)), "grid_create")
        return Grid(self, g, w, h, min_x, min_y, res)

    def grid_from_array(self, cells: np.ndarray, min_x: float, min_y: float, res: float) -> "Grid":
        cells = np.ascontiguousarray(cells, dtype=np.float64)
        h, w = cells.shape
        g = self.grid(w, h, min_x, min_y, res)
        g.upload(cells)
        return g

    def grid_from_patches(self, patches, npx: int, npy: int, patch_size: int, min_x: float, min_y: float,
                          res: float, cell_bytes: int = 16, value_offset: int = 8,
                          into: Optional["Grid"] = None) -> "Grid":
        """lgs_grid_upload_patches: `patches` is a row-major list (py * npx + px)
        of host arrays holding patch_size^2 cells of cell_bytes bytes each (the
        fp64 value at value_offset), or None for an unallocated patch."""
        g = into or self.grid(npx * patch_size, npy * patch_size, min_x, min_y, res)
        keep = [None if p is None else np.ascontiguousarray(p) for p in patches]
        for p in keep:
            if p is not None and p.nbytes != patch_size * patch_size * cell_bytes:
                raise ValueError("patch array size does not match patch_size^2 * cell_bytes")
        table = (_P * max(1, len(keep)))(*[None if p is None else p.ctypes.data for p in keep])
        self.check(self.lib.lgs_grid_upload_patches(self.h, g.h, table, npx, npy, patch_size, cell_bytes,
                                                    value_offset), "grid_upload_patches")
        return g

    def wrap_device(self, ptr: int, w: int, h: int, min_x: float, min_y: float, res: float) -> "Grid":
        g = _P()
        self.check(self.lib.lgs_grid_wrap(self.h, _P(ptr), w, h, min_x, min_y, res, C.byref(g)), "grid_wrap")
        return Grid(self, g, w, h, min_x, min_y, res, owned=False)

    def precompute_max(self, src: "Grid", win: int, out: Optional["Grid"] = None) -> "Grid":
        if out is None:
            out = self.grid(src.w, src.hgt, src.min_x, src.min_y, src.res)
        self.check(self.lib.lgs_grid_precompute_max(self.h, src.h, int(win), out.h), "precompute_max")
        return out

    # ---- scans ----
    def scan(self, ranges, angles, rel_pose=(0.0, 0.0, 0.0), min_range=0.0, max_range=30.0) -> "Scan":
        r = np.ascontiguousarray(ranges, dtype=np.float64)
        a = np.ascontiguousarray(angles, dtype=np.float64)
        hs = ScanHost(dptr(r), dptr(a), len(r), Pose2D(*rel_pose), min_range, max_range)
        s = _P()
        self.check(self.lib.lgs_scan_create(self.h, C.byref(hs), C.byref(s)), "scan_create")
        return Scan(self, s, r, a, rel_pose, min_range, max_range)

    def interpolate(self, scan: "Scan", dist_scans: float = 0.05, dist_threshold_empty: float = 0.25) -> "Scan":
        """ScanInterpolator::Interpolate: a new device scan (launcher defaults 0.05 / 0.25)."""
        s = _P()
        self.check(self.lib.lgs_scan_interpolate(self.h, scan.h, dist_scans, dist_threshold_empty, C.byref(s)),
                   "scan_interpolate")
        n = C.c_int()
        self.check(self.lib.lgs_scan_get(s, C.byref(n), None, None), "scan_get")
        r, a = np.zeros(n.value), np.zeros(n.value)
        self.check(self.lib.lgs_scan_get(s, C.byref(n), dptr(r), dptr(a)), "scan_get")
        return Scan(self, s, r, a, scan.rel_pose, scan.min_range, scan.max_range)

    # ---- matcher ----
    def optimize_pose(self, grid, coarse, params: RtcsmParams, cost: CostGEParams, scan, init,
                      thr: float) -> RtcsmSummary:
        out = RtcsmSummary()
        rc = self.lib.lgs_rtcsm_optimize_pose(self.h, grid.h, coarse.h, C.byref(params), C.byref(cost), scan.h,
                                              Pose2D(*init), float(thr), C.byref(out))
        self.check(rc, "rtcsm_optimize_pose")
        return out

    def optimize_pose_query(self, grid, params: RtcsmParams, cost: CostGEParams, scan, init) -> RtcsmSummary:
        out = RtcsmSummary()
        rc = self.lib.lgs_rtcsm_optimize_pose_query(self.h, grid.h, C.byref(params), C.byref(cost), scan.h,
                                                    Pose2D(*init), C.byref(out))
        self.check(rc, "rtcsm_optimize_pose_query")
        return out

    def optimize_pose_query_batch(self, grids, params: RtcsmParams, cost: CostGEParams, scans, inits):
        """n independent OptimizePose(query) calls as one batched pipeline;
        grids: one map per query (or a single map for all)."""
        n = len(scans)
        if not isinstance(grids, (list, tuple)):
            grids = [grids] * n
        garr = (_P * n)(*[g.h for g in grids])
        sarr = (_P * n)(*[s.h for s in scans])
        poses = (Pose2D * n)(*[Pose2D(*p) for p in inits])
        out = (RtcsmSummary * n)()
        rc = self.lib.lgs_rtcsm_optimize_pose_query_batch(self.h, garr, C.byref(params), C.byref(cost), sarr,
                                                          poses, n, out)
        self.check(rc, "rtcsm_optimize_pose_query_batch")
        return list(out)

    def optimize_pose_batch(self, grid, coarse, params, cost, scans: Sequence["Scan"], inits, thr: float):
        n = len(scans)
        arr = (_P * n)(*[s.h for s in scans])
        poses = (Pose2D * n)(*[Pose2D(*p) for p in inits])
        out = (RtcsmSummary * n)()
        rc = self.lib.lgs_rtcsm_optimize_pose_batch(self.h, grid.h, coarse.h, C.byref(params), C.byref(cost),
                                                    arr, poses, n, float(thr), out)
        self.check(rc, "rtcsm_optimize_pose_batch")
        return list(out)

    def dense_scores(self, grid, coarse, params, scan, init):
        dims = (C.c_int * 7)()
        self.check(self.lib.lgs_rtcsm_dense_scores(self.h, grid.h, coarse.h, C.byref(params), scan.h,
                                                   Pose2D(*init), None, None, dims), "dense_scores(dims)")
        wx, wy, wt, ncx, ncy, nfx, nfy = list(dims)
        T = 2 * wt + 1
        cs = np.zeros((T, ncx, ncy))
        fs = np.zeros((T, nfx, nfy))
        self.check(self.lib.lgs_rtcsm_dense_scores(self.h, grid.h, coarse.h, C.byref(params), scan.h,
                                                   Pose2D(*init), dptr(cs), dptr(fs), dims), "dense_scores")
        return list(dims), cs, fs

    # ---- loop-closure batch ----
    def loop_detect(self, params: RtcsmParams, cost: CostGEParams, thr: float, queries, candidates,
                    shards: Sequence["Context"] = ()):
        """queries: [(map Grid, coarse Grid|None, node_pose, node_index, first, count)];
        candidates: [(Scan, node_pose, node_index)] -> ctypes LoopResult array (one per candidate).
        shards: further contexts (GPUs) to split the candidates over
        (lgs_loop_detect_rtcsm_multi; this context is shard 0)."""
        qs = (LoopQuery * max(1, len(queries)))()
        for i, (m, c, pose, idx, first, cnt) in enumerate(queries):
            qs[i] = LoopQuery(m.h, c.h if c is not None else None, Pose2D(*pose), idx, first, cnt)
        cs = (LoopCandidate * max(1, len(candidates)))()
        for i, (s, pose, idx) in enumerate(candidates):
            cs[i] = LoopCandidate(s.h, Pose2D(*pose), idx, 0)
        out = (LoopResult * max(1, len(candidates)))()
        if shards:
            hs = (_P * (1 + len(shards)))(self.h, *[c.h for c in shards])
            self.check(self.lib.lgs_loop_detect_rtcsm_multi(hs, len(hs), C.byref(params), C.byref(cost), float(thr),
                                                            qs, len(queries), cs, len(candidates), out),
                       "loop_detect_rtcsm_multi")
            return out
        self.check(self.lib.lgs_loop_detect_rtcsm(self.h, C.byref(params), C.byref(cost), float(thr), qs,
                                                  len(queries), cs, len(candidates), out), "loop_detect_rtcsm")
        return out

    # ---- the loop batch over several processes (RCCL) ----
    def rccl_comm(self, world: int = 1, rank: int = 0, unique_id: Optional[bytes] = None):
        """An ncclComm_t of `world` ranks on this context's device (lgs_rccl_comm_init);
        unique_id: the 128 bytes of lgs_rccl_unique_id, made on one rank (new if None)."""
        if unique_id is None:
            buf = (C.c_ubyte * 128)()
            self.check(self.lib.lgs_rccl_unique_id(buf), "rccl_unique_id")
        else:
            buf = (C.c_ubyte * 128).from_buffer_copy(unique_id)
        comm = _P()
        self.check(self.lib.lgs_rccl_comm_init(self.h, buf, world, rank, C.byref(comm)), "rccl_comm_init")
        return comm

    def rccl_comm_destroy(self, comm):
        self.check(self.lib.lgs_rccl_comm_destroy(comm), "rccl_comm_destroy")

    def loop_records_allgather(self, comm, rank: int, world: int, n: int, local):
        """lgs_loop_records_allgather: this rank's block of LoopResult records ->
        all n records in candidate order."""
        cnt = len(local)
        loc = (LoopResult * max(1, cnt))(*local) if cnt else (LoopResult * 1)()
        out = (LoopResult * max(1, n))()
        self.check(self.lib.lgs_loop_records_allgather(self.h, comm, rank, world, n, loc, out),
                   "loop_records_allgather")
        return out

    # ---- branch-and-bound matcher ----
    def precompute_pyramid(self, src: "Grid", node_height_max: int):
        """PrecomputeGridMaps: [window-max grid with window 2^h for h = 0..H]"""
        out = [self.grid(src.w, src.hgt, src.min_x, src.min_y, src.res) for _ in range(node_height_max + 1)]
        arr = (_P * len(out))(*[g.h for g in out])
        self.check(self.lib.lgs_grid_precompute_pyramid(self.h, src.h, int(node_height_max), arr),
                   "grid_precompute_pyramid")
        return out

    def bb_optimize_pose_batch(self, grid, pyramid, params: "BBParams", cost: CostGEParams, scans, inits,
                               thr: float):
        n = len(scans)
        parr = (_P * len(pyramid))(*[g.h for g in pyramid])
        sarr = (_P * n)(*[s.h for s in scans])
        poses = (Pose2D * n)(*[Pose2D(*p) for p in inits])
        out = (RtcsmSummary * max(1, n))()
        self.check(self.lib.lgs_bb_optimize_pose_batch(self.h, grid.h, parr, C.byref(params), C.byref(cost), sarr,
                                                       poses, n, float(thr), out), "bb_optimize_pose_batch")
        return list(out)[:n]

    def bb_optimize_pose_query(self, grid, params: "BBParams", cost: CostGEParams, scan, init) -> RtcsmSummary:
        out = RtcsmSummary()
        self.check(self.lib.lgs_bb_optimize_pose_query(self.h, grid.h, C.byref(params), C.byref(cost), scan.h,
                                                       Pose2D(*init), C.byref(out)), "bb_optimize_pose_query")
        return out

    def loop_detect_bb(self, params: "BBParams", cost: CostGEParams, thr: float, queries, candidates):
        """as loop_detect, with LoopDetectorBranchBound (the coarse entry of a query is ignored)"""
        qs = (LoopQuery * max(1, len(queries)))()
        for i, (m, c, pose, idx, first, cnt) in enumerate(queries):
            qs[i] = LoopQuery(m.h, None, Pose2D(*pose), idx, first, cnt)
        cs = (LoopCandidate * max(1, len(candidates)))()
        for i, (s, pose, idx) in enumerate(candidates):
            cs[i] = LoopCandidate(s.h, Pose2D(*pose), idx, 0)
        out = (LoopResult * max(1, len(candidates)))()
        self.check(self.lib.lgs_loop_detect_bb(self.h, C.byref(params), C.byref(cost), float(thr), qs,
                                               len(queries), cs, len(candidates), out), "loop_detect_bb")
        return out

    # ---- Gauss-Newton refine (K4) ----
    def linsolve(self, grid, params: LinsolveParams, scan, init, trajectory: bool = False):
        """ScanMatcherLinearSolver::OptimizePose; returns the summary and, with
        trajectory=True, [(x, y, theta, cost)] after every OptimizeStep."""
        out = LinsolveSummary()
        traj = np.zeros(4 * max(1, params.num_iterations_max)) if trajectory else None
        self.check(self.lib.lgs_linsolve_optimize_pose(self.h, grid.h, C.byref(params), scan.h, Pose2D(*init),
                                                       C.byref(out), dptr(traj) if trajectory else None),
                   "linsolve_optimize_pose")
        if trajectory:
            return out, [tuple(traj[4 * k: 4 * k + 4]) for k in range(out.iterations)]
        return out

    def linsolve_batch(self, grid, params: LinsolveParams, scans, inits):
        n = len(scans)
        arr = (_P * n)(*[s.h for s in scans])
        poses = (Pose2D * n)(*[Pose2D(*p) for p in inits])
        out = (LinsolveSummary * n)()
        self.check(self.lib.lgs_linsolve_optimize_pose_batch(self.h, grid.h, C.byref(params), arr, poses, n, out),
                   "linsolve_optimize_pose_batch")
        return list(out)

    def cost_square_error(self, grid, umin: float, umax: float, scan, sensor_pose, covariance: bool = False):
        v = C.c_double()
        cov = (C.c_double * 9)() if covariance else None
        self.check(self.lib.lgs_cost_square_error(self.h, grid.h, umin, umax, scan.h, Pose2D(*sensor_pose),
                                                  C.byref(v), cov), "cost_square_error")
        return (v.value, list(cov)) if covariance else v.value

    # ---- occupancy maps (K3) ----
    def map(self, res: float, patch_size: int, ncx: int, ncy: int, center=(0.0, 0.0)) -> "Map":
        h = _P()
        self.check(self.lib.lgs_map_create(self.h, res, patch_size, ncx, ncy, center[0], center[1],
                                           C.byref(h)), "map_create")
        return Map(self, h)

    def construct_maps(self, maps, ranges, scans, poses, bp: "BuilderParams"):
        """GridMapBuilder::AfterLoopClosure's rebuild: maps[i] from pose-graph
        nodes ranges[i] = (idx_min, idx_max) inclusive; node k = (scans[k], poses[k])."""
        nm, n = len(maps), len(scans)
        mh = (_P * nm)(*[m.h for m in maps])
        lo = (C.c_int * nm)(*[int(a) for a, _ in ranges])
        hi = (C.c_int * nm)(*[int(b) for _, b in ranges])
        arr = (_P * n)(*[s.h for s in scans])
        ps = (Pose2D * n)(*[Pose2D(*p) for p in poses])
        self.check(self.lib.lgs_maps_construct_from_scans(self.h, mh, lo, hi, nm, arr, ps, n, C.byref(bp)),
                   "maps_construct_from_scans")

    def construct_global_map(self, res: float, patch_size: int, scans, poses, bp: "BuilderParams") -> "Map":
        """GridMapBuilder::ConstructGlobalMap: a new map from all nodes."""
        n = len(scans)
        arr = (_P * n)(*[s.h for s in scans])
        ps = (Pose2D * n)(*[Pose2D(*p) for p in poses])
        h = _P()
        self.check(self.lib.lgs_map_construct_global(self.h, res, patch_size, arr, ps, n, C.byref(bp), C.byref(h)),
                   "map_construct_global")
        return Map(self, h)

    DEBUG_BUFFERS = {"sbound": (0, np.float64), "part_c": (1, np.float64), "part_k": (2, np.int64),
                     "L": (3, np.float64), "tedge": (4, np.int32), "cbase": (5, np.int32), "idx": (6, np.int32),
                     "cscore": (7, np.float64), "planes": (8, np.float64), "super": (9, np.float16)}

    def debug_buffer(self, name: str, item: int = 0) -> np.ndarray:
        """Diagnostics: an intermediate buffer of one item of the last
        correlative batch (lgs_debug_item_buffer); "L" = [Lp, pad x7, Lc0..Lc3]."""
        which, dt = self.DEBUG_BUFFERS[name]
        n = C.c_size_t()
        self.check(self.lib.lgs_debug_item_buffer(self.h, item, which, None, 0, C.byref(n)), "debug_item_buffer")
        out = np.zeros(n.value // np.dtype(dt).itemsize, dtype=dt)
        self.check(self.lib.lgs_debug_item_buffer(self.h, item, which, out.ctypes.data_as(_P), out.nbytes,
                                                  C.byref(n)),
                   "debug_item_buffer")
        return out

    def debug_libm(self, op: int, x) -> np.ndarray:
        """Diagnostics: the device's glibc sincos (op 0, rows of (sin, cos)) or
        pow(x, 3.0) (op 1) on the GPU (lgs_debug_libm)."""
        x = np.ascontiguousarray(x, dtype=np.float64)
        out = np.zeros((len(x), 2) if op == 0 else len(x), dtype=np.float64)
        self.check(self.lib.lgs_debug_libm(self.h, op, x.ctypes.data_as(_P), len(x), out.ctypes.data_as(_P)),
                   "debug_libm")
        return out

    def copy_counters(self) -> dict:
        """Diagnostics: cross-context map copies made onto this context by
        lgs_loop_detect_rtcsm_multi (lgs_debug_copy_counters)."""
        a, b = C.c_longlong(), C.c_longlong()
        self.check(self.lib.lgs_debug_copy_counters(self.h, C.byref(a), C.byref(b)), "debug_copy_counters")
        return {"direct": a.value, "staged": b.value}

    def offset_checks(self, reset: bool = True) -> dict:
        """Checked build only (liblgs_hip_checked.so): plane-offset checks and
        violations of the correlative consumers since the last reset
        (lgs_debug_offset_checks); raises in the product build."""
        out = (C.c_ulonglong * 4)()
        self.check(self.lib.lgs_debug_offset_checks(self.h, 1 if reset else 0, out), "debug_offset_checks")
        return {"checked": out[0], "violations": out[1], "first": out[2], "first_base": out[3]}

    def debug_keysort(self, keys, lo: int, bits: int) -> np.ndarray:
        """Diagnostics: the K3 stable radix sort (csrc/k_sort.hip) of host u32
        keys on bits [lo, lo + bits) (lgs_debug_keysort)."""
        k = np.ascontiguousarray(keys, dtype=np.uint32)
        out = np.zeros_like(k)
        self.check(self.lib.lgs_debug_keysort(self.h, k.ctypes.data_as(_P), out.ctypes.data_as(_P), len(k), lo, bits),
                   "debug_keysort")
        return out

    def cost_greedy_endpoint(self, grid, cost: CostGEParams, scan, pose) -> float:
        v = C.c_double()
        self.check(self.lib.lgs_cost_greedy_endpoint(self.h, grid.h, C.byref(cost), scan.h, Pose2D(*pose),
                                                     C.byref(v)), "cost_greedy_endpoint")
        return v.value


class Grid:
    def __init__(self, ctx: Context, h, w, hh, min_x, min_y, res, owned=True, map_view=None):
        self.ctx, self.h = ctx, h
        self.map_view = map_view      # owning Map for lgs_map_grid views (handle not ours)
        self.w, self.hgt = w, hh
        self.min_x, self.min_y, self.res = min_x, min_y, res
        self.owned = owned

    def upload(self, cells: np.ndarray):
        cells = np.ascontiguousarray(cells, dtype=np.float64)
        assert cells.shape == (self.hgt, self.w)
        self.ctx.check(self.ctx.lib.lgs_grid_upload(self.ctx.h, self.h, dptr(cells)), "grid_upload")

    def download(self) -> np.ndarray:
        out = np.zeros((self.hgt, self.w))
        self.ctx.check(self.ctx.lib.lgs_grid_download(self.ctx.h, self.h, dptr(out)), "grid_download")
        return out

    def device_ptr(self) -> int:
        return self.ctx.lib.lgs_grid_device_ptr(self.h)

    def close(self):
        if self.h:
            if self.map_view is None:
                self.ctx.lib.lgs_grid_destroy(self.h)  # frees the handle; cells only if owned
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Map:
    """lgs_map: GridMap<BinaryBayesGridCell<double>> with device-resident cells."""

    def __init__(self, ctx: Context, h):
        self.ctx, self.h = ctx, h

    def geometry(self) -> dict:
        g = MapGeometry()
        self.ctx.check(self.ctx.lib.lgs_map_get_geometry(self.h, C.byref(g)), "map_geometry")
        return g.dict()

    def grid(self) -> "Grid":
        """Non-owning grid view (valid until the next geometry change)."""
        gh = _P()
        self.ctx.check(self.ctx.lib.lgs_map_grid(self.h, C.byref(gh)), "map_grid")
        mg = MapGeometry()
        self.ctx.check(self.ctx.lib.lgs_map_get_geometry(self.h, C.byref(mg)), "map_geometry")
        return Grid(self.ctx, gh, mg.num_cells_x, mg.num_cells_y, mg.min_x, mg.min_y, mg.resolution,
                    owned=False, map_view=self)

    def update_scan(self, scan: "Scan", robot_pose, bp: BuilderParams):
        self.ctx.check(self.ctx.lib.lgs_map_update_scan(self.ctx.h, self.h, scan.h, Pose2D(*robot_pose),
                                                        C.byref(bp)), "map_update_scan")

    def construct(self, scans, poses, bp: BuilderParams):
        n = len(scans)
        arr = (_P * n)(*[s.h for s in scans])
        ps = (Pose2D * n)(*[Pose2D(*p) for p in poses])
        self.ctx.check(self.ctx.lib.lgs_map_construct_from_scans(self.ctx.h, self.h, arr, ps, n, C.byref(bp)),
                       "map_construct_from_scans")

    def append_scan(self, latest: "Map", scans, poses, bp: BuilderParams):
        """GridMapBuilder::AppendScan: scans[-1] inserted into this (local) map,
        `latest` rebuilt from all of `scans` (lgs_map_append_scan)."""
        n = len(scans)
        arr = (_P * n)(*[s.h for s in scans])
        ps = (Pose2D * n)(*[Pose2D(*p) for p in poses])
        self.ctx.check(self.ctx.lib.lgs_map_append_scan(self.ctx.h, self.h, latest.h, arr, ps, n, C.byref(bp)),
                       "map_append_scan")

    def rebuilds(self) -> dict:
        """Diagnostics: incremental and full latest-map rebuilds of this map
        (lgs_debug_map_rebuilds)."""
        a, b = C.c_longlong(), C.c_longlong()
        self.ctx.check(self.ctx.lib.lgs_debug_map_rebuilds(self.h, C.byref(a), C.byref(b)), "debug_map_rebuilds")
        return {"incremental": a.value, "full": b.value}

    def render_gray(self) -> np.ndarray:
        """MapSaver::DrawMap gray image (rows flipped up-down), uint8 [h, w]."""
        g = self.geometry()
        img = np.zeros((g["h"], g["w"]), dtype=np.uint8)
        if img.size:
            self.ctx.check(self.ctx.lib.lgs_map_render_gray(self.ctx.h, self.h,
                                                            img.ctypes.data_as(C.POINTER(C.c_uint8))),
                           "map_render_gray")
        return img

    def render_gray_region(self, x0, y0, w, h, flip=True) -> np.ndarray:
        """DrawMap of the w x h cells at (x0, y0), uint8 [h, w] (lgs_map_render_gray_region)."""
        img = np.zeros((h, w), dtype=np.uint8)
        self.ctx.check(self.ctx.lib.lgs_map_render_gray_region(self.ctx.h, self.h, x0, y0, w, h, int(flip),
                                                               img.ctypes.data_as(C.POINTER(C.c_uint8))),
                       "map_render_gray_region")
        return img

    def patches(self) -> np.ndarray:
        """Patch::IsAllocated per patch, uint8 [npy, npx]."""
        g = self.geometry()
        f = np.zeros((g["npy"], g["npx"]), dtype=np.uint8)
        if f.size:
            self.ctx.check(self.ctx.lib.lgs_map_download_patches(self.ctx.h, self.h,
                                                                 f.ctypes.data_as(C.POINTER(C.c_uint8))),
                           "map_download_patches")
        return f

    def actual_size(self):
        """GridMap::ComputeActualMapSize -> (allocated patches, 12 ints)."""
        n = C.c_int()
        out = (C.c_int * 12)()
        self.ctx.check(self.ctx.lib.lgs_map_actual_size(self.ctx.h, self.h, C.byref(n), out), "map_actual_size")
        return n.value, list(out)

    def download(self):
        g = self.geometry()
        cells = np.zeros((g["h"], g["w"]))
        hits = np.zeros((g["h"], g["w"]), dtype=np.uint32)
        misses = np.zeros((g["h"], g["w"]), dtype=np.uint32)
        self.ctx.check(self.ctx.lib.lgs_map_download(self.ctx.h, self.h, dptr(cells),
                                                     hits.ctypes.data_as(C.POINTER(C.c_uint32)),
                                                     misses.ctypes.data_as(C.POINTER(C.c_uint32))),
                       "map_download")
        return cells, hits, misses

    def close(self):
        if self.h:
            self.ctx.lib.lgs_map_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Scan:
    def __init__(self, ctx, h, ranges, angles, rel_pose, min_range, max_range):
        self.ctx, self.h = ctx, h
        self.ranges, self.angles = ranges, angles
        self.rel_pose, self.min_range, self.max_range = rel_pose, min_range, max_range

    def close(self):
        if self.h:
            self.ctx.lib.lgs_scan_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
