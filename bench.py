#!/usr/bin/env python3
"""Benchmark of the MI355X hot path (BASELINE.json configs 2-5).

Default workload ("match", BASELINE.json's metric, config 2): one step = one
ScanMatcher::OptimizePose(query) through the C-ABI
(lgs_rtcsm_optimize_pose_query): coarse-map precompute of the 1000x1000 @ 5 cm
grid, exhaustive +-2 m / +-30 deg correlative search for a 1081-beam scan,
greedy-endpoint cost and covariance.  Grid and scans are resident in HBM before
the timed region.  With --gpus N (one process per GPU, torchrun) every rank
matches its own scans (replicas, weak scaling) and the winning poses are
all-gathered over RCCL inside the timed region.

Other workloads (--workload):
  refine  config 3: ScanMatcherLinearSolver, 1081 beams, 50 iterations (one
          refine per step, synchronous; replicas across ranks)
  loop    config 5: LoopDetectorRealTimeCorrelative::Detect over 512
          candidates (32 local maps x 16 nodes, JSON loop window), sharded in
          contiguous blocks across ranks + all-gather of result records
          (strong scaling: the 512 candidates are split)
  stream  config 4: per scan, match against the latest map + local-map insert
          + latest-map rebuild from the last 10 scans (replicas)

Rank 0 prints ONE JSON line (DESIGN.md §6 explains every field).
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "my-lidar-graph-slam_amd"))

from lgs_amd import abi, scene  # noqa: E402

METRIC = "scans/sec + p50 scan-match ms, 1081-beam vs 1000×1000@5cm grid, 1/2/4/8 GPU"
PARAMS = (5, 4.0, 4.0, 1.0471976, 20.0)          # LowRes, rangeX, rangeY, rangeTheta, ScanRangeMax
LOOP_PARAMS = (5, 5.0, 5.0, 1.0, 20.0)           # launcher_settings_default.json:107-113
BB_PARAMS = (6, 2.0, 2.0, 1.0, 20.0, 0.01, 20.0)  # LoopDetectorBranchBound (launcher_settings_default.json:128-146)
COST = (0.01, 20.0, 0.075, 0.1, 1, 0.05, 1.0)    # launcher-built CostGreedyEndpoint members
LINSOLVE = (50, 0.0, 0.01, 20.0, 1e-3, 1e-3, 0.01, 20.0)   # config 3
STREAM_WINDOWS = {"json": (0.2, 0.2, 0.5), "config2": (4.0, 4.0, 1.0471976)}   # search range x, y, theta
BUILDER = (0.01, 20.0, 0.6, 0.45)                # GridMapBuilder usable range, pHit, pMiss
HBM_PEAK_GBS = 8000.0                            # MI355X_MICROARCH.md: 8.0 TB/s spec


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None, help="default: 200 (match/refine), 4 (loop), 500 (stream)")
    ap.add_argument("--warmup", type=int, default=None)
    ap.add_argument("--workload", default="match", choices=["match", "refine", "loop", "loop_bb", "stream", "rebuild"])
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="bounded CPU-baseline budget")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--spin-sync", type=int, default=1, help="1 spin on the stream when waiting, 0 blocking wait")
    ap.add_argument("--skip-kernels", default="",
                    help="diagnostics only: comma-separated kernel names not launched (results invalid)")
    ap.add_argument("--super-prune", type=int, default=1,
                    help="A/B: 1 superblock pruning of the coarse stage, 0 score every coarse block")
    ap.add_argument("--streams", type=int, default=2,
                    help="match workload: concurrent HIP streams (lgs contexts) per GPU, one host thread each")
    ap.add_argument("--batch", type=int, default=128,
                    help="match workload: queries per call (lgs_rtcsm_optimize_pose_query_batch runs them as "
                         "64-query chunks, two in flight; 1 = one lgs_rtcsm_optimize_pose_query call per scan)")
    ap.add_argument("--lanes-min-batch", type=int, default=None,
                    help="A/B: LGS_OPT_LANES_MIN_BATCH (pruned coarse stage kernel choice by batch size)")
    ap.add_argument("--latency-calls", type=int, default=100,
                    help="match workload: lone OptimizePose(query) calls timed for p50/p90 (0 = skip, e.g. under "
                         "rocprofv3 so that the trace holds the batched launches only)")
    ap.add_argument("--interp", type=int, default=1,
                    help="stream workload: 1 (default, the launcher's UseScanInterpolator) interpolates every "
                         "scan (lgs_scan_interpolate, DistScans 0.05 / DistThresholdEmpty 0.25), 0 raw scans")
    ap.add_argument("--dropin-line", type=int, default=1,
                    help="match workload: also time INTEGRATION.md's drop-in query path (Flatten of a patch map + "
                         "upload + match, C++) and report it as 'dropin'")
    ap.add_argument("--fused", type=int, default=1,
                    help="stream workload (C++ driver): GridMapBuilder::AppendScan as one fused call (1) or as "
                         "the insert + the latest-map rebuild (0)")
    ap.add_argument("--driver", default="cpp", choices=["cpp", "py"],
                    help="stream workload: the frontend loop in C++ over the adapter (default) or in Python")
    ap.add_argument("--ctx-option", type=lambda v: (int(v.split("=")[0]), float(v.split("=")[1])), default=None,
                    help="stream workload (C++ driver), A/B: ID=VALUE, one lgs_ctx option on the device context")
    ap.add_argument("--window", default="json", choices=sorted(STREAM_WINDOWS),
                    help="stream workload: search window (json = the launcher's frontend 0.2 m/0.2 m/0.5 rad, "
                         "config2 = +-2 m/+-30 deg)")
    ap.add_argument("--pmc", default=os.path.join(ROOT, "profiles", "pmc_summary.json"),
                    help="rocprofv3 PMC summary (tools/pmc_summary.py) of THIS library build: roofline.traffic "
                         "is taken from it only when its lib_sha256 matches liblgs_hip.so, else null; other "
                         "workloads read <pmc>_<workload>.json beside it")
    ap.add_argument("--loop-line", type=int, default=1,
                    help="match workload: also run config 5 (512 loop candidates sharded over the ranks, strong "
                         "scaling) after the timed region and report it as 'config5_strong_scaling'")
    ap.add_argument("--distinct-maps", type=int, default=0,
                    help="match workload: 1 = every query of a call against its own copy of the map (distinct "
                         "device buffers: the per-query coarse-map precompute is not served from the cache)")
    ap.add_argument("--sub-lines", type=int, default=1,
                    help="match workload: also report configs 4 (config4_stream), 3 (config3_refine) and f2 "
                         "(f2_rebuild) after the timed region, each with its own CPU baseline and kernel times")
    ap.add_argument("--timed-events", default="dominant", choices=["dominant", "all", "none"],
                    help="kernel timing inside the timed region: the roofline kernel only (default; with "
                         "--device-timing 1 on the match workload: every kernel of the chunks, which costs two "
                         "atomics per workgroup), every kernel, or none (A/B of the timing overhead)")
    ap.add_argument("--device-timing", type=int, default=1,
                    help="1 (default) = time the correlative chunks' kernels on the device (LGS_OPT_DEVICE_TIMING: "
                         "first workgroup start to last workgroup end, s_memrealtime -- the span rocprofv3's kernel "
                         "trace reports); 0 = HIP events on the stream (their begin fires when the stream reaches "
                         "the launch, before the kernel gets its CUs)")
    a = ap.parse_args()
    d_steps = dict(match=200, refine=200, loop=12, loop_bb=12, stream=10000 if a.driver == "cpp" else 500,
                   rebuild=20)[a.workload]
    d_warm = dict(match=10, refine=5, loop=1, loop_bb=2, stream=10, rebuild=2)[a.workload]
    a.steps = d_steps if a.steps is None else a.steps
    a.warmup = d_warm if a.warmup is None else a.warmup
    return a


class Dist:
    """torch.distributed (RCCL) when launched by torchrun with WORLD_SIZE > 1.

    LGS_BENCH_REHEARSE=1 (rehearsal of the multi-rank path on a one-GPU box):
    every rank uses GPU 0 and the collectives run over gloo on host tensors."""

    def __init__(self, gpus: int = 1):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        if self.world != gpus:
            sys.stderr.write(f"bench.py: --gpus {gpus} but WORLD_SIZE={self.world}\n")
            sys.exit(2)
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        self.rehearse = os.environ.get("LGS_BENCH_REHEARSE") == "1"
        # LGS_BENCH_DIST=1: the RCCL process group even at world size 1 (checks,
        # on a one-GPU box, the torch-first HIP runtime sharing of the N>1 path)
        force = os.environ.get("LGS_BENCH_DIST") == "1"
        self.d = None
        if self.rehearse:
            self.local = 0
        if self.world > 1 or force:
            import torch
            import torch.distributed as tdist
            if self.world == 1:   # LGS_BENCH_DIST without a launcher: a one-rank env:// rendezvous
                for k, v in (("RANK", "0"), ("LOCAL_RANK", "0"), ("WORLD_SIZE", "1"), ("MASTER_ADDR", "127.0.0.1"),
                             ("MASTER_PORT", "29531")):
                    os.environ.setdefault(k, v)
            if self.rehearse:
                tdist.init_process_group("gloo")
            else:
                torch.cuda.set_device(self.local)
                tdist.init_process_group("nccl", device_id=torch.device("cuda", self.local))
            self.d = tdist

    def device(self):
        if not self.d:
            return None
        return "cpu" if self.rehearse else f"cuda:{self.local}"

    def barrier(self):
        if self.d:
            self.d.barrier()

    def max(self, v: float) -> float:
        if not self.d:
            return v
        import torch
        t = torch.tensor([v], dtype=torch.float64, device=self.device())
        self.d.all_reduce(t, op=self.d.ReduceOp.MAX)
        return float(t.item())

    def all_gather_rows(self, a: np.ndarray):
        if not self.d:
            return a
        import torch
        local = torch.from_numpy(np.ascontiguousarray(a)).to(self.device())
        out = torch.empty((self.world,) + tuple(local.shape), dtype=local.dtype, device=local.device)
        if self.rehearse:
            parts = [torch.empty_like(local) for _ in range(self.world)]
            self.d.all_gather(parts, local)
            return torch.stack(parts).numpy()
        self.d.all_gather_into_tensor(out, local)
        torch.cuda.synchronize()
        return out.cpu().numpy()

    def close(self):
        if self.d:
            self.d.destroy_process_group()


def lib_sha256() -> str:
    import hashlib
    with open(abi.LIB_PATH, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()


def pmc_for(pmc_path, trace_kernel, workload):
    """Counter bytes per launch of `trace_kernel` from a PMC summary of THIS
    build and THIS workload (tools/pmc_summary.py records the library's
    sha256 and the bench workload profiled), else None.
    gfx950 FETCH_SIZE counts half the bytes of wide coalesced reads
    (MI355X_MICROARCH.md §HBM): 'traffic' doubles it; the raw sum is kept too."""
    if workload != "match":
        # other workloads' passes sit beside the match summary as pmc_summary_<workload>.json
        root, ext = os.path.splitext(pmc_path)
        pmc_path = f"{root}_{workload}{ext}"
    try:
        pmc = json.load(open(pmc_path))
    except (OSError, ValueError):
        return None
    if pmc.get("lib_sha256") != lib_sha256() or pmc.get("workload", "match") != workload:
        return None
    kernels = pmc.get("kernels", {})
    e = kernels.get(trace_kernel)
    if not e:   # the launched variant (k_coarse_list_c, the chunked list kernel since r04)
        cands = [k for k in kernels if k.startswith(trace_kernel)]
        e = kernels[cands[0]] if len(cands) == 1 else None
    if not e or "fetch_bytes_per_launch" not in e or "write_bytes_per_launch" not in e:
        return None
    return dict(traffic=2.0 * e["fetch_bytes_per_launch"] + e["write_bytes_per_launch"],
                raw=e["fetch_bytes_per_launch"] + e["write_bytes_per_launch"], avg_us=e.get("avg_us"),
                l2_hit_rate=e.get("l2_hit_rate"), profile=os.path.relpath(pmc_path, ROOT))


def roofline_from(stats, kernel, pmc_path, trace_kernel, bound, workload="match", bytes_scale=1.0,
                  time_key="total_ms", exec_key=None):
    """Roofline of the dominant kernel: achieved = ALGORITHMIC bytes per launch
     / event-timed average launch duration; frac against the
    8 TB/s HBM peak.  frac_hbm_counters = the PMC-counted HBM bytes of the same
    kernel (from this build's profile) over the same time; null without one.
    bytes_scale rescales the library's per-launch accounting (k_super counts
    8 B per superblock lookup, the fp64 planes' width; the 8-bit units read 1 B).
    time_key: "total_ms" (events, or the device execution span) or
    "dispatch_ms" (device-timed, dispatch-inclusive); exec_key adds the
    execution-span figure beside it."""
    k = stats.get(kernel)
    if not k or not k["launches"] or not k["algo_bytes"] or not k.get(time_key):
        return None
    per_launch = bytes_scale * k["algo_bytes"] / k["launches"]
    avg_ms = k[time_key] / k["launches"]
    achieved = per_launch / (avg_ms * 1e-3) / 1e9
    p = pmc_for(pmc_path, trace_kernel, workload)
    traffic = round(p["traffic"]) if p else None
    frac_hbm = round(traffic / (avg_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4) if p else None
    ex = None
    if exec_key and k.get(exec_key):
        ex_ms = k[exec_key] / k["launches"]
        ex = dict(avg_launch_ms=round(ex_ms, 5), frac=round(per_launch / (ex_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4))
    return dict(bound=bound, achieved=round(achieved, 1), peak=HBM_PEAK_GBS, unit="GB/s",
                frac=round(achieved / HBM_PEAK_GBS, 4), traffic=traffic, time_basis=time_key, execution=ex,
                frac_algorithmic=round(achieved / HBM_PEAK_GBS, 4), frac_hbm_counters=frac_hbm,
                traffic_raw_fetch_plus_write=round(p["raw"]) if p else None,
                l2_hit_rate=p["l2_hit_rate"] if p else None, pmc_profile=p["profile"] if p else None,
                pmc_avg_launch_us=p["avg_us"] if p else None,
                kernel=trace_kernel, avg_launch_ms=round(avg_ms, 5), algo_bytes_per_launch=per_launch)


def coarse_stage(stats):
    """The whole batched coarse stage: k_coarse_list (the 'k_coarse' kernel of
    the roofline, every coarse lookup) plus the work-list passes around it
    (k_keep, k_unsafe_list: 'k_coarse_aux'), per k_coarse launch, with the
    same algorithmic bytes."""
    k, a = stats.get("k_coarse"), stats.get("k_coarse_aux")
    if not k or not a or not k["launches"] or not k["algo_bytes"]:
        return None
    ms = (k["total_ms"] + a["total_ms"]) / k["launches"]
    per = k["algo_bytes"] / k["launches"]
    return dict(kernels="k_keep + k_coarse_list + k_unsafe_list", ms_per_launch=round(ms, 5),
                aux_ms_per_launch=round(a["total_ms"] / k["launches"], 5),
                frac=round(per / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4))


def set_timed_events(ctx, args, dominant, extra=(), chunk_kernels=False):
    """Kernel timing during the timed region (LGS_OPT_PROFILE_MASK); the
    coarse kernel's work-list passes (k_coarse_aux) are timed with it, and
    the `extra` kernels (config 5: k_super, which outweighs k_coarse there).
    With --device-timing the correlative chunks' launches are timed on the
    device (LGS_OPT_DEVICE_TIMING); chunk_kernels: then every kernel of the
    chunks is timed (no events, two atomics per workgroup), so that the line
    can name the largest kernel by its share of the timed region."""
    dom = 1 << abi.KERNEL_IDS.index(dominant)
    if dominant == "k_coarse":
        dom |= 1 << abi.KERNEL_IDS.index("k_coarse_aux")
    for k in extra:
        dom |= 1 << abi.KERNEL_IDS.index(k)
    every = (1 << len(abi.KERNEL_IDS)) - 1
    if args.device_timing and chunk_kernels:
        dom = every
    mask = {"dominant": dom, "all": every, "none": 0}[args.timed_events]
    ctx.set_option(abi.LGS_OPT_DEVICE_TIMING, 1 if args.device_timing else 0)
    ctx.set_option(abi.LGS_OPT_PROFILE_MASK, mask)
    ctx.reset_stats()


# the launched kernel(s) behind each timing id of a config-2 chunk (rocprofv3 names)
TRACE_NAMES = dict(k_project="k_beams (lean batches; k_project<16> materialises)", k_super="k_super_oct<5, 2>", k_seed="k_seed_members + k_seed_super<2>",
                   k_coarse_aux="k_keep + k_unsafe_list", k_coarse="k_coarse_list_c", k_select="k_select<256>",
                   k_fine="k_fine_regs", k_replay="k_replay", k_cost="k_cost<1>",
                   k_precompute="k_precompute_planes<5, 8>", k_super_planes="k_super_hv<1>")


def timed_region_kernels(stats):
    """Per-kernel device times of the timed region (every kernel of the
    chunks, device-timed): launches, average ms, share of the summed kernel
    time; and the largest kernel by that share."""
    tot = sum(v["total_ms"] for v in stats.values() if v["launches"])
    if tot <= 0:
        return None, None
    rows = {k: dict(trace_name=TRACE_NAMES.get(k, k), launches=v["launches"],
                    avg_ms=round(v["total_ms"] / v["launches"], 5), share=round(v["total_ms"] / tot, 4))
            for k, v in sorted(stats.items(), key=lambda kv: -kv[1]["total_ms"]) if v["launches"]}
    top = max(rows, key=lambda k: rows[k]["share"])
    return rows, dict(kernel=top, trace_name=rows[top]["trace_name"], share=rows[top]["share"],
                      avg_ms=rows[top]["avg_ms"])


def bench_map(world, ang):
    w, h, mx, my = scene.map_geometry(1000, 100, 0.05)
    cells = scene.approx_occupancy_map(world, scene.arc_poses(10), ang, w, h, mx, my, 0.05)
    return cells, mx, my


def random_scans(world, ang, rng, n, jitter=(0.3, 0.3, 0.2)):
    scans, inits, truths = [], [], []
    for _ in range(n):
        true = (rng.uniform(-1.5, 1.5), rng.uniform(-1.5, 1.5), rng.uniform(-np.pi, np.pi))
        scans.append(scene.ray_cast(world, true, ang))
        inits.append((true[0] + rng.uniform(-jitter[0], jitter[0]), true[1] + rng.uniform(-jitter[1], jitter[1]),
                      true[2] + rng.uniform(-jitter[2], jitter[2])))
        truths.append(true)
    return scans, inits, truths


def oracle_lib():
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_bind as ob
    return ob


class FbIn(C.Structure):
    _fields_ = [("device", C.c_int), ("n_scans", C.c_int), ("warmup", C.c_int), ("n_beams", C.c_int),
                ("n_segs", C.c_int), ("interp", C.c_int), ("latest_scans", C.c_int), ("fused", C.c_int),
                ("low_res", C.c_int),
                ("range_x", C.c_double), ("range_y", C.c_double), ("range_theta", C.c_double),
                ("scan_range_max", C.c_double), ("segs", C.POINTER(C.c_double)), ("angles", C.POINTER(C.c_double)),
                ("truths", C.POINTER(C.c_double)), ("odo", C.POINTER(C.c_double)), ("n_dump", C.c_int),
                ("opt_id", C.c_int), ("opt_value", C.c_double), ("profile_warmup", C.c_int)]


class FbOut(C.Structure):
    _fields_ = [("est", C.POINTER(C.c_double)), ("guess", C.POINTER(C.c_double)),
                ("dump_ranges", C.POINTER(C.c_double)), ("total_s", C.c_double), ("phase_s", C.c_double * 4),
                ("steps_timed", C.c_int), ("not_found", C.c_int), ("kstats", C.POINTER(abi.KernelStat)),
                ("kstats_cap", C.c_int), ("kstats_n", C.c_int)]


class DropinIn(C.Structure):
    _fields_ = [("device", C.c_int), ("w", C.c_int), ("h", C.c_int), ("patch_size", C.c_int),
                ("min_x", C.c_double), ("min_y", C.c_double), ("res", C.c_double),
                ("cells", C.POINTER(C.c_double)), ("n_beams", C.c_int), ("n_queries", C.c_int),
                ("ranges", C.POINTER(C.c_double)), ("angles", C.POINTER(C.c_double)),
                ("inits", C.POINTER(C.c_double)), ("low_res", C.c_int), ("range_x", C.c_double),
                ("range_y", C.c_double), ("range_theta", C.c_double), ("scan_range_max", C.c_double)]


class DropinOut(C.Structure):
    _fields_ = [("flatten_s", C.c_double), ("upload_s", C.c_double), ("match_uploaded_s", C.c_double),
                ("match_resident_s", C.c_double), ("same", C.c_int), ("patch_ingest_s", C.c_double),
                ("match_patch_s", C.c_double), ("same_patch", C.c_int), ("allocated_patches", C.c_int)]


def bench_drivers():
    """liblgs_frontend_bench.so: C++ loops over the adapter (host/frontend_bench.cpp)."""
    lib = C.CDLL(os.path.join(ROOT, "my-lidar-graph-slam_amd", "lgs_amd", "liblgs_frontend_bench.so"))
    lib.lgs_frontend_bench.argtypes = [C.POINTER(FbIn), C.POINTER(FbOut)]
    lib.lgs_dropin_bench.argtypes = [C.POINTER(DropinIn), C.POINTER(DropinOut)]
    return lib


def dptr(a):
    return a.ctypes.data_as(C.POINTER(C.c_double))


def dropin_line(args, D, n_queries=32):
    """INTEGRATION.md §2's drop-in query path for the unchanged reference
    frontend: Flatten of a patch-based GridMapType (1000x1000, PatchSize 100,
    virtual Value() per cell) + upload per query, beside the match on the
    resident map (C++ driver, lgs_dropin_bench)."""
    world = scene.make_world()
    ang = scene.beam_angles(1081)
    cells, mx, my = bench_map(world, ang)
    rng = np.random.default_rng(5 + D.rank)
    scans, inits, _ = random_scans(world, ang, rng, n_queries)
    r = np.ascontiguousarray(np.stack(scans), dtype=np.float64)
    ini = np.ascontiguousarray(np.array(inits, dtype=np.float64))
    c = np.ascontiguousarray(cells, dtype=np.float64)
    a = np.ascontiguousarray(ang)
    h, w = c.shape
    din = DropinIn(D.local, w, h, 100, mx, my, 0.05, dptr(c), len(ang), n_queries, dptr(r), dptr(a), dptr(ini),
                   *PARAMS)
    dout = DropinOut()
    rc = bench_drivers().lgs_dropin_bench(C.byref(din), C.byref(dout))
    if rc != 0:
        raise RuntimeError(f"lgs_dropin_bench failed with status {rc}")
    ms = lambda v: round(1e3 * v / n_queries, 4)   # noqa: E731
    return dict(queries=n_queries, per_query_ms=ms(dout.patch_ingest_s + dout.match_patch_s),
                patch_ingest_ms=ms(dout.patch_ingest_s), match_patch_ms=ms(dout.match_patch_s),
                same_poses=bool(dout.same_patch and dout.same), allocated_patches=dout.allocated_patches,
                patches=(h // 100) * (w // 100),
                flatten_path=dict(per_query_ms=ms(dout.flatten_s + dout.upload_s + dout.match_uploaded_s),
                                  flatten_ms=ms(dout.flatten_s), upload_ms=ms(dout.upload_s),
                                  match_uploaded_ms=ms(dout.match_uploaded_s)),
                match_resident_ms=ms(dout.match_resident_s),
                note="unchanged reference frontend: a GridMapType copy per OptimizePose, ingested patch-natively "
                     "(lgs_grid_upload_patches: only allocated patches' raw 16-byte cells cross PCIe); "
                     "flatten_path = the Flatten + dense upload ingest it replaces")


def timed(budget_s, items, fn):
    """CPU baseline: run fn over items until the budget is spent (>= 3 items)."""
    times = []
    t_start = time.perf_counter()
    for it in items:
        t0 = time.perf_counter()
        fn(it)
        times.append(time.perf_counter() - t0)
        if time.perf_counter() - t_start > budget_s and len(times) >= 3:
            break
    return len(times) / sum(times), times


# --------------------------------------------------------------------- match
def cpu_model():
    """The host CPU's model string (/proc/cpuinfo), for the cpu_baseline lines."""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or "unknown"


def cpu_threads():
    """Host cores the CPU baseline may use: the box's share (OMP_NUM_THREADS is
    set to it on the GPU box), else every core."""
    return max(1, int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1)))


def cpu_throughput(budget_s, items, fn, threads):
    """Oracle throughput with `threads` independent workers (ctypes releases the
    GIL inside the C oracle, so the workers run in parallel)."""
    import threading
    lock = threading.Lock()
    queue = list(items)
    times = []
    t_start = time.perf_counter()

    def worker():
        while True:
            with lock:
                if not queue or (time.perf_counter() - t_start > budget_s and len(times) >= threads):
                    return
                it = queue.pop(0)
            t0 = time.perf_counter()
            fn(it)
            with lock:
                times.append(time.perf_counter() - t0)

    th = [threading.Thread(target=worker) for _ in range(threads)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    wall = time.perf_counter() - t_start
    return len(times) / wall, times


def run_match(args, D, ctx):
    """S concurrent streams per GPU (one lgs_ctx each, driven from its own host
    thread), each running batches of B complete OptimizePose(query) matches
    (lgs_rtcsm_optimize_pose_query_batch: every query precomputes its own
    coarse map; one launch per pipeline stage for the B queries).  A step is
    one batch; value = scans/s over all ranks and streams."""
    import threading
    world = scene.make_world()
    ang = scene.beam_angles(1081)
    cells, mx, my = bench_map(world, ang)
    rng = np.random.default_rng(1000 + D.rank)
    # a fixed set of 256 scans: the workload (and coarse_blocks_scored_mean) does
    # not depend on --steps / --warmup
    scans, inits, truths = random_scans(world, ang, rng, 256)
    S = max(1, args.streams)
    ctxs = [ctx] + [abi.Context(D.local) for _ in range(S - 1)]
    state = []
    B = max(1, args.batch)
    # --distinct-maps: every query of a call matches against its own copy of
    # the map (distinct device buffers), so no query's coarse-map precompute
    # reads a map another query of the batch already brought into L2/MALL
    nmaps = B if args.distinct_maps else 1
    for c in ctxs:
        c.set_option(abi.LGS_OPT_SUPER_PRUNE, args.super_prune)
        c.set_option(abi.LGS_OPT_SPIN_SYNC, args.spin_sync)
        if args.lanes_min_batch is not None:
            c.set_option(abi.LGS_OPT_LANES_MIN_BATCH, args.lanes_min_batch)
        gs = [c.grid_from_array(cells, mx, my, 0.05) for _ in range(nmaps)]
        state.append((c, gs if args.distinct_maps else gs[0], [c.scan(r, ang) for r in scans]))
    P, cost = abi.RtcsmParams(*PARAMS), abi.CostGEParams(*COST)
    n = len(scans)

    def call(c, g, ds, k):
        """step k: scans k*B .. k*B + B - 1 (cyclic over the generated scans)"""
        if B == 1:
            j = k % n
            return [c.optimize_pose_query(g[0] if isinstance(g, list) else g, P, cost, ds[j], inits[j])], [j]
        js = [(k * B + i) % n for i in range(B)]
        return c.optimize_pose_query_batch(g, P, cost, [ds[j] for j in js], [inits[j] for j in js]), js

    for c, g, ds in state:
        for k in range(args.warmup):
            call(c, g, ds, k)
        set_timed_events(c, args, "k_coarse", chunk_kernels=True)
        if args.skip_kernels:   # after the warmup: skipped stages then read valid stale scratch
            c.set_option(abi.LGS_OPT_SKIP_MASK,
                         sum(1 << abi.KERNEL_IDS.index(k) for k in args.skip_kernels.split(",")))
    results = np.zeros((args.steps * B, 7))
    lat = [[] for _ in range(S)]

    def stream(i):
        c, g, ds = state[i]
        for k in range(i, args.steps, S):
            ts = time.perf_counter()
            outs, js = call(c, g, ds, args.warmup + k)
            lat[i].append(time.perf_counter() - ts)
            for q, (out, j) in enumerate(zip(outs, js)):
                e = out.estimated_pose
                results[k * B + q] = (e.x, e.y, e.theta, out.score_max, out.coarse_blocks, out.fine_blocks, j)

    D.barrier()
    for c, _, _ in state:
        c.synchronize()
    th = [threading.Thread(target=stream, args=(i,)) for i in range(S)]
    t0 = time.perf_counter()
    for t in th:
        t.start()
    for t in th:
        t.join()
    D.all_gather_rows(results)       # winning poses of every rank, over RCCL
    elapsed = D.max(time.perf_counter() - t0)
    D.barrier()
    stats = {}
    for c, _, _ in state:            # k_coarse launches of every stream, event-timed on their own streams
        for k, v in c.kernel_stats().items():
            a = stats.setdefault(k, dict(launches=0, total_ms=0.0, algo_bytes=0.0, dispatch_ms=0.0))
            for f in a:
                a[f] += v[f]
    # single-stream latency and the per-kernel table: a separate, fully
    # event-timed pass on one stream (outside the timed region)
    c0, g0, ds0 = state[0]
    c0.set_option(abi.LGS_OPT_PROFILE_MASK, 0)
    lat1 = []
    for k in range(args.latency_calls):
        j = (args.warmup + k) % n
        ts = time.perf_counter()
        c0.optimize_pose_query(g0[0] if isinstance(g0, list) else g0, P, cost, ds0[j], inits[j])
        lat1.append(time.perf_counter() - ts)
    c0.set_option(abi.LGS_OPT_PROFILE, 1)
    c0.set_option(abi.LGS_OPT_DEVICE_TIMING, 1 if args.device_timing else 0)
    # one stream: a chunk's tail on the priority stream would overlap the next
    # chunk's plane builds, and the table is of kernels alone
    prio = 1 if "28=1" in os.environ.get("LGS_CTX_OPTIONS", "") else 0   # the timed region's setting
    c0.set_option(abi.LGS_OPT_PRIORITY_TAIL, 0)
    c0.reset_stats()
    iso_calls = min(max(1, 1024 // B), args.steps)   # ~16 coarse launches
    for k in range(iso_calls):
        call(c0, g0, ds0, args.warmup + k)
    all_stats = c0.kernel_stats()
    c0.set_option(abi.LGS_OPT_PROFILE, 0)
    c0.set_option(abi.LGS_OPT_PRIORITY_TAIL, prio)
    if "k_coarse" not in stats:
        stats = all_stats
    err = [max(abs(results[k, 0] - truths[int(results[k, 6])][0]),
               abs(results[k, 1] - truths[int(results[k, 6])][1])) for k in range(args.steps * B)]
    cpu = None
    value = args.steps * B * D.world / elapsed
    if D.rank == 0 and not args.no_cpu and D.world == 1:
        ob = oracle_lib()
        g = ob.OGrid(cells, mx, my, 0.05)
        prm, oc = ob.RtcsmParams(*PARAMS), ob.CostGE(*COST)

        def one(k):
            out = ob.Summary()
            ob.lib().orc_rtcsm_optimize_pose_query(C.byref(g.g), C.byref(prm), C.byref(oc),
                                                   C.byref(ob.OScan(scans[k % n], ang).s),
                                                   ob.Pose(*inits[k % n]), C.byref(out))
        T = cpu_threads()
        rate, times = cpu_throughput(args.cpu_seconds, range(4 * T), one, T)
        cpu = dict(value=round(rate, 4), unit="scans/s", cores=T, kind="port", cpu_model=cpu_model(),
                   sample=f"{len(times)} config-2 scans through the oracle's OptimizePose(query) (C restatement, "
                          f"-O3 -ffp-contract=off, the reference's -O3) on {T} threads, one independent scan per thread; "
                          f"single-scan p50 {1e3 * np.median(times):.1f} ms",
                   speedup=round(value / rate, 1),
                   single_core_scans_per_s=round(1.0 / float(np.median(times)), 4),
                   speedup_vs_single_core=round(value * float(np.median(times)), 1))
    lat_ms = np.array([x for l in lat for x in l]) * 1e3
    trk, top = timed_region_kernels(stats) if args.device_timing else (None, None)
    line = dict(
        metric=METRIC, value=round(value, 2), unit="scans/s", n_gpus=D.world, steps=args.steps,
        warmup=args.warmup, ms_per_step=round(1e3 * elapsed / args.steps, 4), higher_is_better=True,
        scaling="weak", vs_baseline=None, dtype="f64",
        data="synthetic: 24 m room + 40 boxes, analytic ray-cast 1081-beam scans, 10-scan occupancy map",
        config=dict(workload="config2: 1081-beam scan, +-2 m/+-30 deg correlative match (OptimizePose(query)) "
                             "vs 1000x1000@5cm grid, PatchSize 100",
                    beams=1081, grid=[1000, 1000], resolution=0.05, low_resolution=5,
                    search_range=[4.0, 4.0, 1.0471976], scans_per_rank=args.steps * B, batch=B,
                    streams_per_gpu=S, distinct_map_buffers=bool(args.distinct_maps),
                    parallelism=f"replicas x{D.world} (independent scans per rank), {S} concurrent HIP streams "
                                f"per GPU, each issuing calls of {B} OptimizePose(query) matches "
                                f"(one launch per stage per 64-query chunk) + RCCL all-gather of poses"),
        # latency of one lone OptimizePose(query) call (what the frontend waits for)
        p50_scan_match_ms=round(1e3 * float(np.median(lat1)), 4) if lat1 else None,
        p90_scan_match_ms=round(1e3 * float(np.percentile(lat1, 90)), 4) if lat1 else None,
        # latency of one batched call under the timed load
        p50_batch_call_ms=round(float(np.percentile(lat_ms, 50)), 4),
        # the correlative-score kernel over the timed region (the rubric's
        # basis), device-timed by default (LGS_OPT_DEVICE_TIMING, DESIGN.md
        # §6): `avg_launch_ms` is dispatch-inclusive -- from the end of the
        # chunk's previous launch on the stream (k_keep) to the kernel's last
        # workgroup, i.e. its execution plus the wait for CUs held by the
        # other streams' kernels, what rocprofv3's dispatch duration counts
        # (tools/trace_coarse.py's "timed" group of the committed trace) --
        # and `execution` is the first-workgroup-start to last-workgroup-end
        # span of the same launches; roofline_isolated is the same kernel
        # timed alone, the one-stream pass after the timed region (the
        # trace's "alone" group).  Events when device timing is off.
        roofline=(roofline_from(stats, "k_coarse", args.pmc, "k_coarse_list", "l2-gather", time_key="dispatch_ms",
                                exec_key="total_ms") if args.device_timing
                  else roofline_from(stats, "k_coarse", args.pmc, "k_coarse_list", "l2-gather")), cpu_baseline=cpu,
        # the superblock-bound pass (1 B per angle x superblock x beam of the
        # 8-bit superblock units, r06), timed the same way
        roofline_super=(roofline_from(stats, "k_super", args.pmc, "k_super_oct<5, 2>", "l2-gather",
                                      bytes_scale=0.125, time_key="dispatch_ms", exec_key="total_ms")
                        if args.device_timing else
                        roofline_from(stats, "k_super", args.pmc, "k_super_oct<5, 2>", "l2-gather", bytes_scale=0.125)),
        timing=("device: s_memrealtime stamps of sampled workgroups per launch (LGS_OPT_DEVICE_TIMING); "
                "avg_launch_ms dispatch-inclusive, execution = first start to last end"
                if args.device_timing else "HIP events on each launch's stream"),
        timed_region_kernels=trk, largest_kernel=top,
        roofline_isolated=roofline_from(all_stats, "k_coarse", args.pmc, "k_coarse_list", "l2-gather"),
        coarse_stage=coarse_stage(all_stats),
        pose_err_max_m=round(float(max(err)), 4), timed_events=args.timed_events,
        super_prune=bool(args.super_prune),
        coarse_blocks_scored_mean=round(float(results[:, 4].mean()), 1),
        fine_blocks_refined_mean=round(float(results[:, 5].mean()), 1))
    for c in ctxs[1:]:
        c.close()
    return line, all_stats, value


# -------------------------------------------------------------------- refine
def run_refine(args, D, ctx):
    world = scene.make_world()
    ang = scene.beam_angles(1081)
    cells, mx, my = bench_map(world, ang)
    rng = np.random.default_rng(2000 + D.rank)
    # (256 scans: the device-filling batch below takes one per CU)
    scans, inits, _ = random_scans(world, ang, rng, 256, jitter=(0.05, 0.05, 0.03))
    grid = ctx.grid_from_array(cells, mx, my, 0.05)
    dscans = [ctx.scan(r, ang) for r in scans]
    lp = abi.LinsolveParams(*LINSOLVE)
    for k in range(args.warmup):
        ctx.linsolve(grid, lp, dscans[k % len(dscans)], inits[k % len(dscans)])
    set_timed_events(ctx, args, "k_linsolve")
    lat = []
    D.barrier()
    t0 = time.perf_counter()
    for k in range(args.steps):
        j = (args.warmup + k) % len(dscans)
        ts = time.perf_counter()
        ctx.linsolve(grid, lp, dscans[j], inits[j])
        lat.append(time.perf_counter() - ts)
    elapsed = D.max(time.perf_counter() - t0)
    stats = ctx.kernel_stats()
    ctx.set_option(abi.LGS_OPT_PROFILE, 0)
    # batched throughput (one workgroup per refine)
    def batch_rate_of(nb):
        ctx.linsolve_batch(grid, lp, dscans[:nb], inits[:nb])
        tb = time.perf_counter()
        ctx.linsolve_batch(grid, lp, dscans[:nb], inits[:nb])
        return nb / (time.perf_counter() - tb)
    batch_rate = batch_rate_of(min(64, len(dscans)))
    # a batch that fills the device: one 512-thread workgroup per refine, one per CU
    batch_rate_full = batch_rate_of(min(256, len(dscans)))
    cpu = None
    if D.rank == 0 and not args.no_cpu and D.world == 1:
        ob = oracle_lib()
        g = ob.OGrid(cells, mx, my, 0.05)
        olp = ob.LinsolveParams(*LINSOLVE)

        def one(k):
            out = ob.Summary()
            ob.lib().orc_linsolve_optimize_pose(C.byref(g.g), C.byref(olp), C.byref(ob.OScan(scans[k], ang).s),
                                                ob.Pose(*inits[k]), C.byref(out), None)
        rate, times = timed(args.cpu_seconds, range(min(len(scans), 64)), one)
        cpu = dict(value=round(rate, 3), unit="refines/s", cores=1, kind="port", cpu_model=cpu_model(),
                   sample=f"{len(times)} config-3 refines through the oracle (1 thread), "
                          f"p50 {1e3 * np.median(times):.1f} ms")
    k = stats.get("k_linsolve", {})
    lat_ms = np.array(lat) * 1e3
    value = args.steps * D.world / elapsed
    line = dict(
        metric="refines/sec, ScanMatcherLinearSolver 1081 beams x 50 iterations vs 1000x1000@5cm",
        value=round(value, 2), unit="refines/s", n_gpus=D.world, steps=args.steps, warmup=args.warmup,
        ms_per_step=round(1e3 * elapsed / args.steps, 4), higher_is_better=True, scaling="weak",
        vs_baseline=None, dtype="f64", data="synthetic (as config 2), seeds within 5 cm / 0.03 rad",
        config=dict(workload="config3: Gauss-Newton refine (LinearSolver + CostSquareError), 50 iterations",
                    beams=1081, grid=[1000, 1000], iterations=50, parallelism=f"replicas x{D.world}"),
        p50_refine_ms=round(float(np.percentile(lat_ms, 50)), 4),
        batched_refines_per_s_per_gpu=round(batch_rate, 1),
        batched_refines_per_s_per_gpu_256=round(batch_rate_full, 1),
        roofline=None, cpu_baseline=cpu,
        kernel_avg_ms=round(k["total_ms"] / k["launches"], 5) if k.get("launches") else None)
    return line, stats, value


# ---------------------------------------------------------------------- loop
def run_loop(args, D, ctx):
    """config 5; --workload loop_bb: the same batch through the reference's
    default loop detector, LoopDetectorBranchBound."""
    from lgs_amd import loopbatch
    bb = args.workload == "loop_bb"
    world = scene.make_world()
    bp = abi.BuilderParams(*BUILDER)

    def build(poses, ang):   # local maps built on the device (K3), 600x600 @ 5 cm
        m = ctx.map(0.05, 100, 600, 600)
        m.construct([ctx.scan(scene.ray_cast(world, p, ang), ang) for p in poses], poses, bp)
        cells, _, _ = m.download()
        g = m.geometry()
        return cells, g["min_x"], g["min_y"], 0.05

    maps, cands = scene.loop_problem(world, build, n_maps=32, nodes_per_map=16, n_beams=1081, seed=5,
                                     perturb=(0.8, 0.3) if bb else (2.0, 0.4), arc_scans=10)
    cost = abi.CostGEParams(*COST)
    if bb:
        fn = loopbatch.hip_detect_fn_bb(ctx, maps, cands, abi.BBParams(*BB_PARAMS), cost, 0.6)
    else:
        fn = loopbatch.hip_detect_fn(ctx, maps, cands, abi.RtcsmParams(*LOOP_PARAMS), cost, 0.6)
    # N > 1 on GPUs: the records' all-gather through the library's own RCCL
    # collective (lgs_loop_records_allgather); the gloo rehearsal keeps torch
    gather = None
    if D.world > 1 and not D.rehearse:
        gather = loopbatch.RcclGather(ctx, D.rank, D.world, D.d)

    def one_step():
        if gather is not None:
            return loopbatch.run_sharded_rccl(cands, fn, gather)
        return loopbatch.run_sharded(cands, fn, D.rank, D.world, D.d, D.device())

    for _ in range(args.warmup):
        one_step()
    dominant = "k_bb_score" if bb else "k_coarse"
    set_timed_events(ctx, args, dominant, extra=() if bb else ("k_super",))
    D.barrier()
    t0 = time.perf_counter()
    step_s = []
    for _ in range(args.steps):
        ts = time.perf_counter()
        rec = one_step()
        step_s.append(time.perf_counter() - ts)
    elapsed = D.max(time.perf_counter() - t0)
    if gather is not None:
        gather.close()
    stats = ctx.kernel_stats()
    ctx.set_option(abi.LGS_OPT_PROFILE, 0)
    found = len(loopbatch.loop_results(rec))
    cpu = None
    if D.rank == 0 and not args.no_cpu and D.world == 1:
        ob = oracle_lib()
        grids = {}
        prm, oc = ob.RtcsmParams(*LOOP_PARAMS), ob.CostGE(*COST)
        bprm = ob.BBParams(*BB_PARAMS)

        def one_bb(i):
            c = cands[i]
            if c.query not in grids:   # the pyramid once per map (LocalMapInfo caches it)
                m = maps[c.query]
                keep = [ob.OGrid(x, m.min_x, m.min_y, 0.05) for x in ob.precompute_pyramid(m.cells, BB_PARAMS[0])]
                grids[c.query] = (ob.OGrid(m.cells, m.min_x, m.min_y, 0.05), keep,
                                  (ob.Grid * len(keep))(*[k.g for k in keep]))
            g, _, arr = grids[c.query]
            s = ob.Summary()
            ob.lib().orc_bb_optimize_pose(C.byref(g.g), arr, C.byref(bprm), C.byref(oc),
                                          C.byref(ob.OScan(c.ranges, c.angles).s), ob.Pose(*c.pose), 0.6,
                                          C.byref(s))

        def one(i):
            if bb:
                return one_bb(i)
            c = cands[i]
            if c.query not in grids:
                m = maps[c.query]
                grids[c.query] = (ob.OGrid(m.cells, m.min_x, m.min_y, 0.05),
                                  ob.OGrid(ob.precompute(m.cells, 5), m.min_x, m.min_y, 0.05))
            g, cg = grids[c.query]
            s = ob.Summary()
            ob.lib().orc_rtcsm_optimize_pose(C.byref(g.g), C.byref(cg.g), C.byref(prm), C.byref(oc),
                                             C.byref(ob.OScan(c.ranges, c.angles).s), ob.Pose(*c.pose), 0.6,
                                             C.byref(s))
        rate, times = timed(args.cpu_seconds, range(0, len(cands), 37), one)
        cpu = dict(value=round(rate, 4), unit="candidates/s", cores=1, kind="port", cpu_model=cpu_model(),
                   sample=f"{len(times)} config-5 candidates through the oracle's "
                          f"{'ScanMatcherBranchBound' if bb else 'RTCSM'} OptimizePose "
                          f"({'pyramid' if bb else 'coarse map'} precomputed per map, as LocalMapInfo caches it; "
                          f"1 thread), p50 {1e3 * np.median(times):.1f} ms")
    value = args.steps * len(cands) / elapsed
    line = dict(
        metric=("loop-closure candidates/sec, LoopDetectorBranchBound, 512 candidates (32 maps x 16 nodes), "
                "1081 beams, +-1 m/+-0.5 rad, NodeHeightMax 6" if bb else
                "loop-closure candidates/sec, 512 candidates (32 maps x 16 nodes), 1081 beams, +-2.5 m/+-0.5 rad"),
        value=round(value, 2), unit="candidates/s", n_gpus=D.world, steps=args.steps, warmup=args.warmup,
        ms_per_step=round(1e3 * elapsed / args.steps, 4), higher_is_better=True, scaling="strong",
        vs_baseline=None, dtype="f64", data="synthetic: 32 device-built local maps (600x600 @ 5 cm), 512 scans",
        config=dict(workload=("config5 (f1): LoopDetectorBranchBound::Detect batch" if bb else
                              "config5: LoopDetectorRealTimeCorrelative::Detect batch"), candidates=len(cands),
                    found=found, parallelism=f"candidates sharded in contiguous blocks over {D.world} ranks + "
                                             "one all-gather of 176-B result records (N > 1: the library's "
                                             "lgs_loop_records_allgather, RCCL)"),
        roofline=roofline_from(stats, dominant, args.pmc, "k_bb_score" if bb else "k_coarse_list", "l2-gather",
                               workload="loop_bb" if bb else "loop"),
        # config 5's largest kernel by time is the 9-row superblock-bound pass,
        # not the coarse sums: its own roofline (1 B per angle x superblock x
        # beam of the 8-bit superblock units, r06)
        roofline_super=None if bb else roofline_from(stats, "k_super", args.pmc, "k_super_oct<9, 3>", "l2-gather",
                                                     workload="loop", bytes_scale=0.125),
        coarse_stage=None if bb else coarse_stage(stats),
        step_ms_p10_p50_p90=[round(1e3 * float(np.percentile(step_s, q)), 4) for q in (10, 50, 90)],
        step_spread=round(float((np.percentile(step_s, 90) - np.percentile(step_s, 10)) / np.median(step_s)), 4),
        cpu_baseline=cpu)
    return line, stats, value


# -------------------------------------------------------------------- stream
def run_stream(args, D, ctx):
    """Config 4: odometry-driven frontend over a circular trajectory (0.1 m,
    0.02 rad per scan, odometry noise sigma (0.01 m, 0.005 rad), seed 7)."""
    world = scene.make_world()
    ang = scene.beam_angles(1081)
    rng = np.random.default_rng(7 + D.rank)
    n = args.warmup + args.steps + 1
    truths = [(5.0 * np.cos(0.02 * k), 5.0 * np.sin(0.02 * k), 0.02 * k + np.pi / 2) for k in range(n)]
    ranges = [scene.ray_cast(world, t, ang) for t in truths]
    bp = abi.BuilderParams(*BUILDER)
    win = STREAM_WINDOWS[args.window]
    P, cost = abi.RtcsmParams(5, *win, 20.0), abi.CostGEParams(*COST)
    local = ctx.map(0.05, 100, 200, 200, center=truths[0][:2])
    latest = ctx.map(0.05, 100, 200, 200, center=truths[0][:2])
    raw = [ctx.scan(r, ang) for r in ranges]
    dscans = [None] * n

    def frontend_scan(k):   # ScanInterpolator::Interpolate (launcher default on)
        dscans[k] = ctx.interpolate(raw[k], 0.05, 0.25) if args.interp else raw[k]

    frontend_scan(0)
    est = [truths[0]]
    local.update_scan(dscans[0], est[0], bp)

    def odometry(rng_, last):
        # the true relative motion + noise, composed onto the last estimate
        d = (0.1 + rng_.normal(0, 0.01), rng_.normal(0, 0.01), 0.02 + rng_.normal(0, 0.005))
        c, s = np.cos(last[2]), np.sin(last[2])
        return (last[0] + c * d[0] - s * d[1], last[1] + s * d[0] + c * d[1], last[2] + d[2])

    phase = dict(interpolate=0.0, latest_map=0.0, match=0.0, insert=0.0)

    def step(k):
        t = [time.perf_counter()]
        guess = odometry(rng, est[-1])
        frontend_scan(k)
        t.append(time.perf_counter())
        lo = max(0, k - 10)
        latest.construct(dscans[lo:k], est[lo:k], bp)                       # UpdateLatestMap (10 scans)
        t.append(time.perf_counter())
        out = ctx.optimize_pose_query(latest.grid(), P, cost, dscans[k], guess)
        e = out.estimated_pose
        est.append((e.x, e.y, e.theta))
        t.append(time.perf_counter())
        local.update_scan(dscans[k], est[-1], bp)                           # UpdateGridMap insert
        t.append(time.perf_counter())
        for i, name in enumerate(phase):
            phase[name] += t[i + 1] - t[i]

    for k in range(1, args.warmup + 1):
        step(k)
    set_timed_events(ctx, args, "k_ray_apply")
    D.barrier()
    t0 = time.perf_counter()
    for name in phase:
        phase[name] = 0.0
    for k in range(args.warmup + 1, n):
        step(k)
    elapsed = D.max(time.perf_counter() - t0)
    stats = ctx.kernel_stats()
    ctx.set_option(abi.LGS_OPT_PROFILE, 0)
    steps = n - args.warmup - 1
    breakdown = {f"{name}_ms": round(1e3 * v / steps, 4) for name, v in phase.items()}
    drift = max(abs(est[-1][0] - truths[len(est) - 1][0]), abs(est[-1][1] - truths[len(est) - 1][1]))
    value = steps * D.world / elapsed
    cpu = None
    if D.rank == 0 and not args.no_cpu and D.world == 1:
        # the same frontend through the oracle from step 1 (same odometry draws):
        # its poses must equal the GPU run's, step for step
        ob = oracle_lib()
        orng = np.random.default_rng(7)
        obp = ob.BuilderParams(*BUILDER)
        oprm, ocost = ob.RtcsmParams(5, *win, 20.0), ob.CostGE(*COST)
        olocal = ob.OMap(0.05, 100, 200, 200, center=truths[0][:2])
        olatest = ob.OMap(0.05, 100, 200, 200, center=truths[0][:2])

        def oscan(k):
            r, a = ob.scan_interpolate(ranges[k], ang, 0.05, 0.25) if args.interp else (ranges[k], ang)
            return ob.OScan(r, a)

        oscans = [oscan(0)]
        oest = [truths[0]]
        olocal.integrate(oest[0], oscans[0], obp)
        times = []
        t_start = time.perf_counter()
        for k in range(1, n):
            t1 = time.perf_counter()
            guess = odometry(orng, oest[-1])
            oscans.append(oscan(k))
            lo = max(0, k - 10)
            olatest.construct(oest[lo:k], oscans[lo:k], obp)
            g = olatest.geometry()
            og = ob.OGrid(olatest.cells(), g["min_x"], g["min_y"], 0.05)
            out = ob.Summary()
            ob.lib().orc_rtcsm_optimize_pose_query(C.byref(og.g), C.byref(oprm), C.byref(ocost),
                                                   C.byref(oscans[k].s), ob.Pose(*guess), C.byref(out))
            e = out.estimated_pose
            oest.append((e.x, e.y, e.theta))
            olocal.integrate(oest[-1], oscans[k], obp)
            times.append(time.perf_counter() - t1)
            if time.perf_counter() - t_start > args.cpu_seconds and len(times) >= 3:
                break
        same = all(tuple(a) == tuple(b) for a, b in zip(oest, est))
        cpu = dict(value=round(len(times) / sum(times), 3), unit="scans/s", cores=1, kind="port", cpu_model=cpu_model(),
                   sample=f"the first {len(times)} frontend steps through the oracle (interpolate, 10-scan "
                          f"ConstructMapFromScans, OptimizePose(query), insert; 1 thread); poses identical to "
                          f"the GPU run's for all of them: {same}")
    line = dict(
        metric="frontend scans/sec: match vs latest map + local-map insert + latest-map rebuild, 1081 beams",
        value=round(value, 2), unit="scans/s", n_gpus=D.world, steps=steps, warmup=args.warmup,
        ms_per_step=round(1e3 * elapsed / steps, 4), higher_is_better=True, scaling="weak", vs_baseline=None,
        dtype="f64", data="synthetic circular trajectory, odometry noise (0.01 m, 0.005 rad)",
        config=dict(workload=f"config4: streaming frontend ({args.window} window "
                             f"{'/'.join(str(v) for v in win)})", beams=1081,
                    scan_interpolator=bool(args.interp), latest_map_scans=10, parallelism=f"replicas x{D.world}"),
        final_drift_m=round(float(drift), 4), breakdown_per_step=breakdown,
        roofline=roofline_from(stats, "k_ray_apply", args.pmc, "k_apply", "hbm", workload=args.workload), cpu_baseline=cpu)
    return line, stats, value


def run_stream_cpp(args, D, ctx):
    """Config 4 driven from C++ (host/frontend_bench.cpp lgs_frontend_bench):
    the same frontend as run_stream -- scan upload, ScanInterpolator, latest map
    from the last 10 scans, OptimizePose(query) from the odometry guess,
    local-map insert -- through the reference-shaped adapter classes with no
    Python between calls.  Trajectory: 0.1 m / 0.02 rad per scan on a 5 m
    circle, odometry noise sigma (0.01 m, 0.005 rad), seed 7 + rank.  The CPU
    baseline replays the first steps through the oracle with the driver's own
    guesses and raw ranges; its poses must equal the driver's bit for bit."""
    world = scene.make_world()
    ang = np.ascontiguousarray(scene.beam_angles(1081))
    n = args.warmup + args.steps + 1
    k = np.arange(n, dtype=np.float64)
    truths = np.ascontiguousarray(np.stack([5.0 * np.cos(0.02 * k), 5.0 * np.sin(0.02 * k), 0.02 * k + np.pi / 2], 1))
    rng = np.random.default_rng(7 + D.rank)
    odo = np.zeros((n, 3))
    for i in range(1, n):
        odo[i] = (0.1 + rng.normal(0, 0.01), rng.normal(0, 0.01), 0.02 + rng.normal(0, 0.005))
    win = STREAM_WINDOWS[args.window]
    segs = np.ascontiguousarray(world, dtype=np.float64)
    n_dump = min(n, 400)
    est, guess = np.zeros((n, 3)), np.zeros((n, 3))
    dump = np.zeros((n_dump, len(ang)))
    fin = FbIn(D.local, n, args.warmup, len(ang), len(segs), int(args.interp), 10, int(args.fused), 5, *win, 20.0,
               dptr(segs), dptr(ang),
               dptr(truths), dptr(odo), n_dump, *(args.ctx_option or (0, 0.0)), 1)
    kst = (abi.KernelStat * len(abi.KERNEL_IDS))()
    fout = FbOut(dptr(est), dptr(guess), dptr(dump), kstats=kst, kstats_cap=len(abi.KERNEL_IDS))
    D.barrier()
    rc = bench_drivers().lgs_frontend_bench(C.byref(fin), C.byref(fout))
    if rc != 0:
        raise RuntimeError(f"lgs_frontend_bench failed with status {rc}")
    steps = fout.steps_timed
    elapsed = D.max(fout.total_s)
    value = steps * D.world / elapsed
    # per-kernel HIP-event times of the (untimed) warmup steps, per step
    wsteps = max(1, args.warmup - 1 if args.warmup >= 3 else args.warmup)   # profiled from step 2 (frontend_bench.cpp)
    stats = {kst[i].name.decode(): dict(launches=kst[i].launches, total_ms=kst[i].total_ms,
                                        algo_bytes=kst[i].algo_bytes)
             for i in range(fout.kstats_n) if kst[i].launches}
    kernel_ms_per_step = {k: round(v["total_ms"] / wsteps, 5) for k, v in stats.items()}
    names = ("scan_upload", "interpolate", "match", "append_scan")
    breakdown = {f"{nm}_ms": round(1e3 * fout.phase_s[i] / steps, 4) for i, nm in enumerate(names)}
    drift = float(np.max(np.abs(est[-1, :2] - truths[-1, :2])))
    cpu = replay = None
    if D.rank == 0 and not args.no_cpu and D.world == 1:
        ob = oracle_lib()
        obp = ob.BuilderParams(*BUILDER)
        oprm, ocost = ob.RtcsmParams(5, *win, 20.0), ob.CostGE(*COST)
        olocal = ob.OMap(0.05, 100, 200, 200, center=tuple(truths[0][:2]))
        olatest = ob.OMap(0.05, 100, 200, 200, center=tuple(truths[0][:2]))

        def oscan(j):
            r, a = ob.scan_interpolate(dump[j], ang, 0.05, 0.25) if args.interp else (dump[j], ang)
            return ob.OScan(r, a)

        oscans = [oscan(0)]
        oest = [tuple(truths[0])]
        olocal.integrate(oest[0], oscans[0], obp)
        times = []
        t_start = time.perf_counter()
        o_steps = min(n_dump, 1 + getattr(args, "oracle_steps", n_dump))
        for j in range(1, o_steps):
            t1 = time.perf_counter()
            oscans.append(oscan(j))
            lo = max(0, j - 10)
            olatest.construct(oest[lo:j], oscans[lo:j], obp)
            g = olatest.geometry()
            og = ob.OGrid(olatest.cells(), g["min_x"], g["min_y"], 0.05)
            out = ob.Summary()
            ob.lib().orc_rtcsm_optimize_pose_query(C.byref(og.g), C.byref(oprm), C.byref(ocost),
                                                   C.byref(oscans[j].s), ob.Pose(*guess[j]), C.byref(out))
            e = out.estimated_pose
            oest.append((e.x, e.y, e.theta))
            olocal.integrate(oest[-1], oscans[j], obp)
            times.append(time.perf_counter() - t1)
            if time.perf_counter() - t_start > args.cpu_seconds and len(times) >= 3:
                break
        same = all(tuple(est[j]) == oest[j] for j in range(len(oest)))
        want = min(n_dump - 1, getattr(args, "oracle_steps", n_dump))
        if len(times) < want:
            # the remaining steps of the replay on the host's threads: step j's
            # latest map from the GPU run's poses of steps j - 10 .. j - 1 (the
            # oracle's own, as long as every earlier step was identical)
            n_id, ok = oracle_replay_parallel(ob, dump, est, guess, truths, ang, win, args.interp, len(times) + 1,
                                              want + 1)
            same = same and ok
            replay = dict(steps=len(times) + n_id, poses_identical=bool(same),
                          note=f"steps 1..{len(times)} sequential (the cpu_baseline timing), "
                               f"{len(times) + 1}..{len(times) + n_id} on {cpu_threads()} threads from the GPU run's "
                               f"earlier poses")
        else:
            replay = dict(steps=len(times), poses_identical=bool(same))
        cpu = dict(value=round(len(times) / sum(times), 3), unit="scans/s", cores=1, kind="port", cpu_model=cpu_model(),
                   sample=f"the first {len(times)} frontend steps through the oracle (interpolate, 10-scan "
                          f"ConstructMapFromScans, OptimizePose(query) from the C++ run's guesses, insert; "
                          f"1 thread); poses identical to the GPU run's for all of them: {same}")
    line = dict(
        metric="frontend scans/sec: match vs latest map + local-map insert + latest-map rebuild, 1081 beams",
        value=round(value, 2), unit="scans/s", n_gpus=D.world, steps=steps, warmup=args.warmup,
        ms_per_step=round(1e3 * elapsed / steps, 4), higher_is_better=True, scaling="weak", vs_baseline=None,
        dtype="f64", data="synthetic circular trajectory, odometry noise (0.01 m, 0.005 rad)",
        config=dict(workload=f"config4: streaming frontend, {n - 1}-scan trajectory ({args.window} window "
                             f"{'/'.join(str(v) for v in win)})", beams=1081,
                    scan_interpolator=bool(args.interp), latest_map_scans=10, driver="C++ adapter loop",
                    append_scan="fused (lgs_map_append_scan)" if args.fused else "UpdateScan + ConstructMapFromScans",
                    parallelism=f"replicas x{D.world}"),
        final_drift_m=round(drift, 4), not_found=fout.not_found, breakdown_per_step=breakdown,
        oracle_replay=replay, kernel_ms_per_step=kernel_ms_per_step,
        kernel_ms_per_step_note=f"HIP-event times of the {wsteps} untimed warmup steps (every kernel timed), per step",
        roofline=None, cpu_baseline=cpu)
    return line, stats, value


def oracle_replay_parallel(ob, dump, est, guess, truths, ang, win, interp, j0, j1):
    """Frontend steps j0 .. j1 - 1 through the oracle, their matches on the
    host's threads: this thread rebuilds the latest map step after step as the
    sequential replay does (one map object, so its geometry has the same
    history; step j's map from scans j - 10 .. j - 1 at the GPU run's poses --
    the oracle's own, as long as every earlier step was identical) and hands
    each step's OptimizePose(query) from the GPU run's guess to a worker.
    Returns (steps, every pose bit-identical to the GPU run's)."""
    import concurrent.futures as cf
    obp = ob.BuilderParams(*BUILDER)
    oprm, ocost = ob.RtcsmParams(5, *win, 20.0), ob.CostGE(*COST)
    olatest = ob.OMap(0.05, 100, 200, 200, center=tuple(truths[0][:2]))

    def oscan(j):
        r, a = ob.scan_interpolate(dump[j], ang, 0.05, 0.25) if interp else (dump[j], ang)
        return ob.OScan(r, a)

    def match(j, og, sc):
        out = ob.Summary()
        ob.lib().orc_rtcsm_optimize_pose_query(C.byref(og.g), C.byref(oprm), C.byref(ocost), C.byref(sc.s),
                                               ob.Pose(*guess[j]), C.byref(out))
        e = out.estimated_pose
        return (e.x, e.y, e.theta) == tuple(est[j])

    oscans = [oscan(0)]
    poses = [tuple(truths[0])]
    futs = []
    with cf.ThreadPoolExecutor(max_workers=cpu_threads()) as ex:
        for j in range(1, j1):
            oscans.append(oscan(j))
            lo = max(0, j - 10)
            olatest.construct(poses[lo:j], oscans[lo:j], obp)
            poses.append(tuple(est[j]))
            if j >= j0:
                g = olatest.geometry()
                og = ob.OGrid(olatest.cells(), g["min_x"], g["min_y"], 0.05)
                futs.append(ex.submit(match, j, og, oscans[j]))
        res = [f.result() for f in futs]
    return len(res), all(res)


# ------------------------------------------------------------------- rebuild
def run_rebuild(args, D, ctx):
    """GridMapBuilder::AfterLoopClosure -- every local map rebuilt
    from its nodes after the pose graph moved them (one
    lgs_maps_construct_from_scans call per step), then one ConstructGlobalMap
    outside the timed region.  400 nodes on a 5 m circle (0.1 m apart), 10
    local maps of 40 nodes, 1081 beams, 5 cm, PatchSize 64."""
    world = scene.make_world()
    ang = scene.beam_angles(1081)
    n_nodes, per_map = 400, 40
    truths = [(5.0 * np.cos(0.02 * k), 5.0 * np.sin(0.02 * k), 0.02 * k + np.pi / 2) for k in range(n_nodes)]
    ranges_ = [scene.ray_cast(world, t, ang) for t in truths]
    dscans = [ctx.scan(r, ang) for r in ranges_]
    rng = np.random.default_rng(11 + D.rank)
    # pose-graph corrections: a few variants, applied in turn
    variants = [[(x + rng.normal(0, 0.03), y + rng.normal(0, 0.03), t + rng.normal(0, 0.01)) for x, y, t in truths]
                for _ in range(4)]
    ranges = [(lo, lo + per_map - 1) for lo in range(0, n_nodes, per_map)]
    bp = abi.BuilderParams(*BUILDER)
    maps = [ctx.map(0.05, 64, 0, 0, center=truths[lo][:2]) for lo, _ in ranges]
    ctx.construct_maps(maps, ranges, dscans, truths, bp)
    for k in range(args.warmup):
        ctx.construct_maps(maps, ranges, dscans, variants[k % 4], bp)
    set_timed_events(ctx, args, "k_ray_apply")
    D.barrier()
    t0 = time.perf_counter()
    for k in range(args.steps):
        ctx.construct_maps(maps, ranges, dscans, variants[k % 4], bp)
    elapsed = D.max(time.perf_counter() - t0)
    stats = ctx.kernel_stats()
    ctx.set_option(abi.LGS_OPT_PROFILE, 0)
    t1 = time.perf_counter()
    gm = ctx.construct_global_map(0.05, 64, dscans, variants[0], bp)
    global_ms = 1e3 * (time.perf_counter() - t1)
    gg = gm.geometry()
    cpu = None
    if D.rank == 0 and not args.no_cpu and D.world == 1:
        ob = oracle_lib()
        oscans = [ob.OScan(r, ang) for r in ranges_]
        obp = ob.BuilderParams(*BUILDER)

        def one(i):
            lo, hi = ranges[i]
            om = ob.OMap(0.05, 64, 0, 0, center=truths[lo][:2])
            om.construct(variants[0][lo:hi + 1], oscans[lo:hi + 1], obp)

        rate, times = timed(args.cpu_seconds, range(len(ranges)), one)
        cpu = dict(value=round(rate * per_map, 2), unit="nodes/s", cores=1, kind="port", cpu_model=cpu_model(),
                   sample=f"{len(times)} local maps x {per_map} nodes through the oracle's ConstructMapFromScans "
                          f"(1 thread, as AfterLoopClosure runs), p50 {1e3 * np.median(times):.1f} ms per map")
    value = args.steps * n_nodes * D.world / elapsed
    line = dict(
        metric="AfterLoopClosure rebuild: pose-graph nodes re-ray-cast/sec, 10 local maps x 40 nodes, 1081 beams",
        value=round(value, 2), unit="nodes/s", n_gpus=D.world, steps=args.steps, warmup=args.warmup,
        ms_per_step=round(1e3 * elapsed / args.steps, 4), higher_is_better=True, scaling="weak",
        vs_baseline=None, dtype="f64", data="synthetic 400-node circular trajectory, pose corrections N(0, 3 cm)",
        config=dict(workload="f2: GridMapBuilder::AfterLoopClosure (all local maps, one fused ray-cast pass)",
                    nodes=n_nodes, local_maps=len(maps), beams=1081, parallelism=f"replicas x{D.world}"),
        global_map=dict(ms=round(global_ms, 3), cells=[gg["w"], gg["h"]], nodes=n_nodes),
        roofline=roofline_from(stats, "k_ray_apply", args.pmc, "k_apply", "hbm", workload=args.workload), cpu_baseline=cpu)
    return line, stats, value


SUB_KEYS = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "scaling", "dtype", "config",
            "cpu_baseline", "roofline", "p50_refine_ms", "batched_refines_per_s_per_gpu",
            "batched_refines_per_s_per_gpu_256", "kernel_avg_ms",
            "final_drift_m", "not_found", "breakdown_per_step", "oracle_replay", "kernel_ms_per_step",
            "kernel_ms_per_step_note", "global_map")


def sub_line(args, D, ctx, workload, steps, warmup, cpu_seconds, **extra):
    """Another workload's line inside the default run (its own steps, warmup
    and bounded CPU baseline), with its per-kernel event times."""
    sa = argparse.Namespace(**vars(args))
    sa.workload, sa.steps, sa.warmup, sa.cpu_seconds = workload, steps, warmup, cpu_seconds
    for k, v in extra.items():
        setattr(sa, k, v)
    fn = dict(refine=run_refine, stream=run_stream_cpp, rebuild=run_rebuild)[workload]
    ln, stats, _ = fn(sa, D, ctx)
    sub = {k: ln[k] for k in SUB_KEYS if k in ln}
    if workload != "stream":
        sub["kernels"] = {k: dict(launches=v["launches"], avg_ms=round(v["total_ms"] / max(1, v["launches"]), 5))
                          for k, v in stats.items() if v["launches"]}
    return sub


def spawn_ranks(args) -> None:
    """--gpus N without a launcher: start N ranks (one process per GPU) with
    torch.distributed.run as a CHILD process, before anything here touches the
    GPU, and exit with its status."""
    if args.gpus <= 1 or "WORLD_SIZE" in os.environ:
        return
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    sys.exit(subprocess.call(cmd))


def main():
    args = parse()
    spawn_ranks(args)
    D = Dist(args.gpus)
    ctx = abi.Context(D.local)
    line, stats, _ = dict(match=run_match, refine=run_refine, loop=run_loop, loop_bb=run_loop,
                          stream=run_stream_cpp if args.driver == "cpp" else run_stream,
                          rebuild=run_rebuild)[args.workload](
        args, D, ctx)
    line["kernels"] = {k: dict(launches=v["launches"], avg_ms=round(v["total_ms"] / max(1, v["launches"]), 5))
                       for k, v in stats.items()}
    if args.workload == "match" and args.loop_line:
        # config 5 next to the config-2 replicas line: the 512 loop candidates
        # split over the ranks (strong scaling), measured after the main timed region
        la = argparse.Namespace(**vars(args))
        la.workload, la.steps, la.warmup, la.no_cpu = "loop", 12, 2, True
        ll, _, _ = run_loop(la, D, ctx)
        line["config5_strong_scaling"] = {k: ll[k] for k in ("metric", "value", "unit", "n_gpus", "steps",
                                                              "ms_per_step", "scaling", "config", "roofline",
                                                              "roofline_super", "step_ms_p10_p50_p90", "step_spread")}
    if args.workload == "match" and args.dropin_line:
        line["dropin"] = dropin_line(args, D)
    if args.workload == "match" and args.sub_lines and not args.distinct_maps:
        # config 2 with a distinct map buffer per query
        da = argparse.Namespace(**vars(args))
        da.distinct_maps, da.steps, da.warmup, da.no_cpu, da.latency_calls = 1, 30, 3, True, 0
        dl, dstats, _ = run_match(da, D, ctx)
        line["config2_distinct_maps"] = {k: dl[k] for k in ("value", "unit", "steps", "ms_per_step", "config",
                                                             "roofline")}
        line["config2_distinct_maps"]["kernels"] = {
            k: dict(launches=v["launches"], avg_ms=round(v["total_ms"] / max(1, v["launches"]), 5))
            for k, v in dstats.items() if v["launches"]}
    if args.workload == "match" and args.sub_lines:
        # configs 4 and 3 and f2 next to the headline, on the same run
        # (replicas over the ranks; CPU baselines on rank 0 at N = 1)
        # (BASELINE config 4: a 10k-scan trajectory -- every config-4 line
        # times 10,000 steps after 100 warm-up steps)
        line["config4_stream"] = sub_line(args, D, ctx, "stream", 10000, 100, 8.0, oracle_steps=200, window="json",
                                          interp=1, fused=1, driver="cpp", ctx_option=None)
        # SURVEY §8(d)'s config-4 variants: the per-scan match at the config-2
        # window (+-2 m / +-30 deg), and with the interpolator off (N = 1081)
        line["config4_stream_config2_window"] = sub_line(args, D, ctx, "stream", 10000, 20, 4.0, oracle_steps=200,
                                                         window="config2", interp=1, fused=1, driver="cpp",
                                                         ctx_option=None)
        line["config4_stream_raw_scans"] = sub_line(args, D, ctx, "stream", 10000, 100, 4.0, oracle_steps=200,
                                                    window="json", interp=0, fused=1, driver="cpp", ctx_option=None)
        line["config3_refine"] = sub_line(args, D, ctx, "refine", 100, 5, 3.0)
        line["f2_rebuild"] = sub_line(args, D, ctx, "rebuild", 10, 2, 3.0)
    if D.rank == 0:
        print(json.dumps(line), flush=True)
    D.close()


if __name__ == "__main__":
    main()
