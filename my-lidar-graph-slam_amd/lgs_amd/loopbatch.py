"""Loop-closure candidate batch sharded over GPUs.

LoopDetectorRealTimeCorrelative::Detect (C/mapping/loop_detector_real_time_correlative.cpp:26-92)
matches every candidate node of every query against the query's local map;
candidates are independent (:38, :66), so with one process per GPU:

  * rank r takes the contiguous block [start_r, start_r + count_r) of the
    candidate list (query-major, node order inside a query: the reference's
    iteration order);
  * it uploads only the local maps its block references and computes their
    coarse maps once (:52-60), then runs lgs_loop_detect_rtcsm on its block
    -- no collective on the data path;
  * one all_gather of fixed 176-byte result records (uint8 rows, padded to the
    largest block) restores the full, ordered list on every rank; results with
    found == 0 are dropped WITHOUT reordering, because the order of loop edges
    feeds the pose-graph optimizer (C/mapping/lidar_graph_slam.cpp:252-282).

`detect_fn(sub_queries, cand_lo, cand_hi) -> np.uint8 [count, 176]` does the
per-rank matching; `hip_detect_fn` is the product implementation (C-ABI);
tests inject an oracle-based one to exercise the sharding on CPU (gloo).
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import Callable, List, Optional, Sequence, Tuple

import numpy as np

from . import abi

RECORD_BYTES = C.sizeof(abi.LoopResult)   # 176


@dataclass
class LocalMap:
    """LoopDetectionQuery::mLocalMapInfo (dense cells) + mLocalMapNode."""
    cells: np.ndarray          # (H, W) fp64, 0.0 = unknown
    min_x: float
    min_y: float
    res: float
    node_pose: Tuple[float, float, float]
    node_index: int


@dataclass
class Candidate:
    """One poseGraphNode of a query: scan + pose (initial guess) + index."""
    query: int
    ranges: np.ndarray
    angles: np.ndarray
    pose: Tuple[float, float, float]
    node_index: int


def shard_bounds(n: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous block of rank r: sizes differ by at most one."""
    base, rem = divmod(n, world)
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


def sub_queries(cands: Sequence[Candidate], lo: int, hi: int) -> List[Tuple[int, int, int]]:
    """[(query index, first local candidate, count)] covering [lo, hi) in order.
    Candidates must be query-major (all of query q before q+1)."""
    out: List[Tuple[int, int, int]] = []
    for i in range(lo, hi):
        q = cands[i].query
        if out and out[-1][0] == q:
            out[-1] = (q, out[-1][1], out[-1][2] + 1)
        else:
            out.append((q, i - lo, 1))
    return out


def hip_detect_fn(ctx: "abi.Context", maps: Sequence[LocalMap], cands: Sequence[Candidate],
                  params: "abi.RtcsmParams", cost: "abi.CostGEParams", threshold: float
                  ) -> Callable[[List[Tuple[int, int, int]], int, int], np.ndarray]:
    """Per-rank matcher on the GPU: uploads the maps its block needs once."""
    grids = {}
    scans = {}

    def fn(subq, lo, hi):
        queries, cl = [], []
        for q, first, count in subq:
            if q not in grids:
                m = maps[q]
                g = ctx.grid_from_array(m.cells, m.min_x, m.min_y, m.res)
                grids[q] = (g, ctx.precompute_max(g, params.low_resolution))
            g, coarse = grids[q]
            queries.append((g, coarse, maps[q].node_pose, maps[q].node_index, first, count))
        for i in range(lo, hi):
            c = cands[i]
            if i not in scans:
                scans[i] = ctx.scan(c.ranges, c.angles)
            cl.append((scans[i], c.pose, c.node_index))
        out = ctx.loop_detect(params, cost, threshold, queries, cl)
        return np.frombuffer(bytes(out), dtype=np.uint8)[: (hi - lo) * RECORD_BYTES].reshape(hi - lo, RECORD_BYTES)

    return fn


def hip_detect_fn_bb(ctx: "abi.Context", maps: Sequence[LocalMap], cands: Sequence[Candidate],
                     params: "abi.BBParams", cost: "abi.CostGEParams", threshold: float
                     ) -> Callable[[List[Tuple[int, int, int]], int, int], np.ndarray]:
    """As hip_detect_fn with LoopDetectorBranchBound (C/mapping/loop_detector_branch_bound.cpp:26-117):
    lgs_loop_detect_bb builds each query's map pyramid itself."""
    grids = {}
    scans = {}

    def fn(subq, lo, hi):
        queries, cl = [], []
        for q, first, count in subq:
            if q not in grids:
                m = maps[q]
                grids[q] = ctx.grid_from_array(m.cells, m.min_x, m.min_y, m.res)
            queries.append((grids[q], None, maps[q].node_pose, maps[q].node_index, first, count))
        for i in range(lo, hi):
            c = cands[i]
            if i not in scans:
                scans[i] = ctx.scan(c.ranges, c.angles)
            cl.append((scans[i], c.pose, c.node_index))
        out = ctx.loop_detect_bb(params, cost, threshold, queries, cl)
        return np.frombuffer(bytes(out), dtype=np.uint8)[: (hi - lo) * RECORD_BYTES].reshape(hi - lo, RECORD_BYTES)

    return fn


def run_sharded(cands: Sequence[Candidate], detect_fn, rank: int = 0, world: int = 1, dist=None,
                device=None) -> np.ndarray:
    """All candidates' records (uint8 [n, 176]) in candidate order, on every rank."""
    n = len(cands)
    lo, hi = shard_bounds(n, world, rank)
    local = detect_fn(sub_queries(cands, lo, hi), lo, hi) if hi > lo else np.zeros((0, RECORD_BYTES), np.uint8)
    assert local.shape == (hi - lo, RECORD_BYTES)
    if world == 1:
        return local
    import torch
    rows = shard_bounds(n, world, 0)[1]        # largest block
    buf = torch.zeros((rows, RECORD_BYTES), dtype=torch.uint8)
    buf[: hi - lo] = torch.from_numpy(local.copy())
    if device is not None and str(device).startswith("cuda"):
        # RCCL: one all-gather into one device tensor, one copy back
        out = torch.empty((world * rows, RECORD_BYTES), dtype=torch.uint8, device=device)
        dist.all_gather_into_tensor(out, buf.to(device))
        allrows = out.cpu().numpy().reshape(world, rows, RECORD_BYTES)
    else:
        if device is not None:
            buf = buf.to(device)
        gathered = [torch.empty_like(buf) for _ in range(world)]
        dist.all_gather(gathered, buf)
        allrows = np.stack([g.cpu().numpy() for g in gathered])
    parts = []
    for r in range(world):
        a, b = shard_bounds(n, world, r)
        parts.append(allrows[r, : b - a])
    return np.concatenate(parts, axis=0)


class RcclGather:
    """The all-gather of the records through the library's C-ABI
    (lgs_loop_records_allgather: one ncclAllGather of fixed-size rows on the
    context's stream, RCCL over xGMI) instead of torch: one communicator per
    rank, its unique id made on rank 0 and broadcast over `dist` once."""

    def __init__(self, ctx: "abi.Context", rank: int, world: int, dist=None):
        self.ctx, self.rank, self.world = ctx, rank, world
        uid = None
        if rank == 0:
            buf = (C.c_ubyte * 128)()
            ctx.check(ctx.lib.lgs_rccl_unique_id(buf), "rccl_unique_id")
            uid = bytes(buf)
        if world > 1:
            box = [uid]
            dist.broadcast_object_list(box, src=0)
            uid = box[0]
        self.comm = ctx.rccl_comm(world, rank, uid)

    def __call__(self, n: int, lo: int, hi: int, local: np.ndarray) -> np.ndarray:
        loc = (abi.LoopResult * max(1, hi - lo)).from_buffer_copy(
            local.tobytes() if hi > lo else bytes(RECORD_BYTES))
        out = (abi.LoopResult * max(1, n))()
        self.ctx.check(self.ctx.lib.lgs_loop_records_allgather(self.ctx.h, self.comm, self.rank, self.world, n,
                                                               loc, out), "loop_records_allgather")
        return np.frombuffer(bytes(out), dtype=np.uint8)[: n * RECORD_BYTES].reshape(n, RECORD_BYTES)

    def close(self):
        if self.comm:
            self.ctx.rccl_comm_destroy(self.comm)
            self.comm = None


def run_sharded_rccl(cands: Sequence[Candidate], detect_fn, gather: RcclGather) -> np.ndarray:
    """run_sharded with the records gathered by the C-ABI collective."""
    n = len(cands)
    lo, hi = shard_bounds(n, gather.world, gather.rank)
    local = detect_fn(sub_queries(cands, lo, hi), lo, hi) if hi > lo else np.zeros((0, RECORD_BYTES), np.uint8)
    assert local.shape == (hi - lo, RECORD_BYTES)
    return gather(n, lo, hi, local)


def decode(records: np.ndarray) -> List[abi.LoopResult]:
    raw = records.tobytes()
    return [abi.LoopResult.from_buffer_copy(raw[i * RECORD_BYTES:(i + 1) * RECORD_BYTES])
            for i in range(records.shape[0])]


def loop_results(records: np.ndarray) -> List[abi.LoopResult]:
    """LoopDetectionResultVector: found records, order preserved (:77-88)."""
    return [r for r in decode(records) if r.found]
