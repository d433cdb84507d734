"""LGS_OPT_DEVICE_TIMING: the correlative chunks' kernels
timed on the device -- each workgroup stamps s_memrealtime at its start and
end into per-chunk words (relaxed atomic maxima), copied back with the
chunk's records; a launch's time is its first workgroup's start to its last
workgroup's end, the span a rocprofv3 kernel trace reports.

The timing must not change a single record bit, must produce a sample for
every kernel of the batched chain that stamps (and plausible spans: positive,
below the call's wall time), and launches outside a chunk's main chain
(guard/dense reruns, other paths) keep HIP-event timing.
"""
import time

import numpy as np
import pytest

from conftest import launcher_cost
from lgs_amd import abi
from test_gpu_batch import _queries, _record, small_map  # noqa: F401 (fixture)
from test_gpu_rtcsm import assert_same, oracle_match

pytestmark = pytest.mark.gpu

# kernels of the batched, pruned chain (config-2-like window) that stamp
CHAIN = ("k_precompute", "k_super_planes", "k_project", "k_super", "k_seed", "k_coarse_aux", "k_coarse",
         "k_select", "k_fine", "k_replay", "k_cost")


def test_device_timing_same_records_and_spans(ctx, world, small_map):
    cells, mx, my = small_map
    rng = np.random.default_rng(101)
    ang, qs = _queries(world, rng, 24, 541)
    params = (5, 4.0, 4.0, 1.0, 20.0)
    P, cost = abi.RtcsmParams(*params), launcher_cost()
    g = ctx.grid_from_array(cells, mx, my, 0.05)
    scans = [ctx.scan(r, ang) for r, _ in qs]
    inits = [i for _, i in qs]
    plain = [_record(b) for b in ctx.optimize_pose_query_batch(g, P, cost, scans, inits)]
    try:
        ctx.set_option(abi.LGS_OPT_DEVICE_TIMING, 1)
        ctx.set_option(abi.LGS_OPT_PROFILE, 1)
        ctx.reset_stats()
        t0 = time.perf_counter()
        timed = ctx.optimize_pose_query_batch(g, P, cost, scans, inits)
        wall_ms = 1e3 * (time.perf_counter() - t0)
        stats = ctx.kernel_stats()
    finally:
        ctx.set_option(abi.LGS_OPT_PROFILE, 0)
        ctx.set_option(abi.LGS_OPT_DEVICE_TIMING, 0)
    assert [_record(b) for b in timed] == plain
    for k in CHAIN:
        s = stats[k]
        assert s["launches"] >= 1, (k, s)
        avg = s["total_ms"] / s["launches"]
        assert 0.0 < avg < wall_ms, (k, avg, wall_ms)
    # the correlative-score kernel's algorithmic bytes still come from the records
    assert stats["k_coarse"]["algo_bytes"] > 0
    for j in (0, 13):
        assert_same(timed[j], oracle_match(cells, mx, my, 0.05, params, qs[j][0], ang, inits[j]), f"q{j}")


def test_device_timing_chunks_and_lone_calls(ctx, world, small_map):
    """Two chunks in flight (two banks, 80 queries) and lone calls: one sample
    per chunk launch; lone calls (a batch of one) are device-timed too."""
    cells, mx, my = small_map
    rng = np.random.default_rng(102)
    ang, qs = _queries(world, rng, 80, 361)
    params = (5, 2.0, 2.0, 0.5, 20.0)
    P, cost = abi.RtcsmParams(*params), launcher_cost()
    g = ctx.grid_from_array(cells, mx, my, 0.05)
    scans = [ctx.scan(r, ang) for r, _ in qs]
    inits = [i for _, i in qs]
    plain = [_record(b) for b in ctx.optimize_pose_query_batch(g, P, cost, scans, inits)]
    lone_plain = _record(ctx.optimize_pose_query(g, P, cost, scans[3], inits[3]))
    try:
        ctx.set_option(abi.LGS_OPT_DEVICE_TIMING, 1)
        ctx.set_option(abi.LGS_OPT_PROFILE, 1)
        ctx.reset_stats()
        timed = [_record(b) for b in ctx.optimize_pose_query_batch(g, P, cost, scans, inits)]
        st_batch = ctx.kernel_stats()
        ctx.reset_stats()
        lone = _record(ctx.optimize_pose_query(g, P, cost, scans[3], inits[3]))
        st_lone = ctx.kernel_stats()
    finally:
        ctx.set_option(abi.LGS_OPT_PROFILE, 0)
        ctx.set_option(abi.LGS_OPT_DEVICE_TIMING, 0)
    assert timed == plain and lone == lone_plain
    assert st_batch["k_coarse"]["launches"] == 2      # one per 64-query chunk
    assert st_batch["k_super"]["launches"] == 2
    assert st_lone["k_project"]["launches"] == 1 and st_lone["k_project"]["total_ms"] > 0
