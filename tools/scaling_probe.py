#!/usr/bin/env python3
"""Multi-GPU readiness of the config-5 loop batch, measured on ONE GPU
(DESIGN.md §7).

bench.py's config-5 line splits 512 candidates (32 local maps x 16 nodes) in
contiguous blocks over N ranks (lgs_amd/loopbatch.run_sharded) and all-gathers
the 176-byte records.  Without an 8-GPU node this measures the pieces of the
N-rank step that do not need one:

  1. per-rank work: every rank's block (64 candidates at N = 8) timed on this
     GPU through the same path a rank runs (hip_detect_fn: Python packaging,
     ctypes, lgs_loop_detect_rtcsm, record copy), after a warm-up that uploaded
     the maps the block references -- the critical path is the slowest rank;
  2. the all-gather of 512 records: gloo on the host CPU (world 2/4/8 CPU
     processes, started BEFORE anything touches the GPU), the host-side upper
     bound; RCCL over xGMI is the driver's to measure;
  3. predicted strong scaling: T1 / (max_r T_r + T_allgather).

Writes one JSON object (stdout, and --out)."""
import argparse
import json
import os
import socket
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "my-lidar-graph-slam_amd"))
sys.path.insert(0, ROOT)

RECORD_BYTES = 176


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _gloo_worker(rank, world, port, n, iters, q):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rows = -(-n // world)
    buf = torch.zeros((rows, RECORD_BYTES), dtype=torch.uint8)
    out = [torch.empty_like(buf) for _ in range(world)]
    for _ in range(10):
        dist.all_gather(out, buf)
    dist.barrier()
    ts = []
    for _ in range(iters):
        t0 = time.perf_counter()
        dist.all_gather(out, buf)
        ts.append(time.perf_counter() - t0)
    if rank == 0:
        q.put(ts)
    dist.barrier()
    dist.destroy_process_group()


def gloo_allgather(world, n=512, iters=200):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_gloo_worker, args=(r, world, port, n, iters, q)) for r in range(world)]
    for p in ps:
        p.start()
    ts = q.get(timeout=120)
    for p in ps:
        p.join(timeout=60)
    return dict(median_ms=round(1e3 * float(np.median(ts)), 4), p90_ms=round(1e3 * float(np.percentile(ts, 90)), 4))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    worlds = (1, 2, 4, 8)
    gloo = {w: gloo_allgather(w) for w in worlds if w > 1}   # before the GPU is touched
    import bench
    from lgs_amd import abi, loopbatch, scene
    ctx = abi.Context(0)
    world = scene.make_world()
    bp = abi.BuilderParams(*bench.BUILDER)

    def build(poses, ang):
        m = ctx.map(0.05, 100, 600, 600)
        m.construct([ctx.scan(scene.ray_cast(world, p, ang), ang) for p in poses], poses, bp)
        cells, _, _ = m.download()
        g = m.geometry()
        return cells, g["min_x"], g["min_y"], 0.05

    maps, cands = scene.loop_problem(world, build, n_maps=32, nodes_per_map=16, n_beams=1081, seed=5,
                                     perturb=(2.0, 0.4), arc_scans=10)
    fn = loopbatch.hip_detect_fn(ctx, maps, cands, abi.RtcsmParams(*bench.LOOP_PARAMS), abi.CostGEParams(*bench.COST),
                                 0.6)
    n = len(cands)
    loopbatch.run_sharded(cands, fn)   # uploads every map (each rank uploads its own in its warm-up)
    shards = {}
    for w in worlds:
        per = []
        for r in range(w):
            lo, hi = loopbatch.shard_bounds(n, w, r)
            sq = loopbatch.sub_queries(cands, lo, hi)
            fn(sq, lo, hi)
            ts = []
            for _ in range(a.reps):
                t0 = time.perf_counter()
                fn(sq, lo, hi)
                ts.append(time.perf_counter() - t0)
            per.append(float(np.median(ts)))
        shards[w] = dict(candidates_per_rank=n // w, rank_ms=[round(1e3 * t, 4) for t in per],
                         max_rank_ms=round(1e3 * max(per), 4))
    # the 8-rank block as ONE chunk (r04) vs two (r05 default, LGS_OPT_SPLIT_CHUNKS)
    lo, hi = loopbatch.shard_bounds(n, 8, 0)
    sq = loopbatch.sub_queries(cands, lo, hi)
    split_ab = {}
    for opt in (0, 1):
        ctx.set_option(abi.LGS_OPT_SPLIT_CHUNKS, opt)
        fn(sq, lo, hi)
        ts = []
        for _ in range(a.reps):
            t0 = time.perf_counter()
            fn(sq, lo, hi)
            ts.append(time.perf_counter() - t0)
        split_ab["two_chunks" if opt else "one_chunk"] = round(1e3 * float(np.median(ts)), 4)
    ctx.set_option(abi.LGS_OPT_SPLIT_CHUNKS, 1)
    # per-rank overhead of an 8-rank step outside the kernels: the whole call
    # (Python packaging + ctypes + lgs_loop_detect_rtcsm + record copy) vs the
    # kernels' event-timed sum, and the C-ABI gather's own work at one rank
    # (records host -> device, ncclAllGather, device -> host, synchronise)
    ctx.set_option(abi.LGS_OPT_PROFILE, 1)
    ctx.reset_stats()
    reps = a.reps
    for _ in range(reps):
        fn(sq, lo, hi)
    kern_ms = sum(v["total_ms"] for v in ctx.kernel_stats().values()) / reps
    ctx.set_option(abi.LGS_OPT_PROFILE, 0)
    gather = loopbatch.RcclGather(ctx, 0, 1)
    rec = fn(sq, lo, hi)
    ts = []
    for _ in range(max(20, reps)):
        t0 = time.perf_counter()
        gather(hi - lo, 0, hi - lo, rec)
        ts.append(time.perf_counter() - t0)
    gather.close()
    overhead = dict(block_call_ms=split_ab["two_chunks"], kernels_event_ms=round(kern_ms, 4),
                    non_kernel_ms=round(split_ab["two_chunks"] - kern_ms, 4),
                    capi_gather_world1_ms=round(1e3 * float(np.median(ts)), 4),
                    note="kernels_event_ms: every kernel of the block's call HIP-event-timed on its stream "
                         "(serialised: the profile mode times each launch), so non_kernel_ms is a lower bound "
                         "of the host/launch share")
    t1 = shards[1]["max_rank_ms"]
    pred = {}
    for w in worlds:
        ag = gloo[w]["median_ms"] if w > 1 else 0.0
        tw = shards[w]["max_rank_ms"] + ag
        pred[w] = dict(step_ms=round(tw, 4), speedup=round(t1 / tw, 3), efficiency=round(t1 / tw / w, 3),
                       candidates_per_s=round(n / tw * 1e3, 1))
    out = dict(workload="config5: 512 candidates (32 maps x 16 nodes), 1081 beams, +-2.5 m / +-0.5 rad",
               shard_on_one_gpu=shards, rank8_block_chunks_ms=split_ab, rank8_overhead=overhead,
               gloo_allgather_512_records=gloo, predicted=pred,
               note="per-rank blocks timed one at a time on ONE MI355X (each rank owns a GPU on a node); "
                    "all-gather = gloo over host TCP (an upper bound of RCCL over xGMI)")
    s = json.dumps(out)
    print(s)
    if a.out:
        with open(a.out, "w") as f:
            f.write(s + "\n")
    ctx.close()


if __name__ == "__main__":
    main()
