"""Loop-closure batch on the GPU (lgs_loop_detect_rtcsm) vs the oracle's
LoopDetectorRealTimeCorrelative::Detect restatement
(C/mapping/loop_detector_real_time_correlative.cpp:26-125).

found flags, node indices, estimated / relative / start poses and scores are
bit-exact; normalized cost and covariance agree to 1e-5 relative (device exp
vs glibc, as for every greedy-endpoint cost)."""
import numpy as np
import pytest

import test_loopbatch_cpu as small
from loop_oracle import oracle_detect_fn
from lgs_amd import abi, loopbatch, scene

pytestmark = pytest.mark.gpu

LOOP_JSON = (5, 5.0, 5.0, 1.0, 20.0)   # launcher_settings_default.json:107-113 (LoopDetectorRealTimeCorrelative.ScanMatcher)


def compare(dev, orc):
    assert len(dev) == len(orc)
    for d, o in zip(dev, orc):
        assert (d.found, d.start_node_index, d.end_node_index) == (o.found, o.start_node_index, o.end_node_index)
        for f in ("relative_pose", "start_node_pose", "estimated_pose"):
            a, b = getattr(d, f), getattr(o, f)
            assert (a.x, a.y, a.theta) == (b.x, b.y, b.theta), f
        assert d.score == o.score
        assert abs(d.normalized_cost - o.normalized_cost) <= 1e-5 * max(1.0, abs(o.normalized_cost))
        assert np.allclose(list(d.covariance), list(o.covariance), rtol=1e-5, atol=1e-9)


def test_loop_detect_small(ctx):
    maps, cands = small.make_problem()
    p, c = abi.RtcsmParams(*small.PARAMS), abi.CostGEParams(*small.COST)
    dev = loopbatch.run_sharded(cands, loopbatch.hip_detect_fn(ctx, maps, cands, p, c, small.THR))
    orc = loopbatch.run_sharded(cands, oracle_detect_fn(maps, cands, small.PARAMS, small.COST, small.THR))
    compare(loopbatch.decode(dev), loopbatch.decode(orc))
    found = loopbatch.loop_results(dev)
    assert 0 < len(found) < len(cands)


def test_loop_detect_coarse_computed_inside(ctx):
    """coarse == NULL: the C-ABI computes ComputeCoarserMap itself (:52-60)."""
    maps, cands = small.make_problem()
    p, c = abi.RtcsmParams(*small.PARAMS), abi.CostGEParams(*small.COST)
    grids = [ctx.grid_from_array(m.cells, m.min_x, m.min_y, m.res) for m in maps]
    scans = [ctx.scan(x.ranges, x.angles) for x in cands]
    qs, first = [], 0
    for qi, m in enumerate(maps):
        n = sum(1 for x in cands if x.query == qi)
        qs.append((grids[qi], None, m.node_pose, m.node_index, first, n))
        first += n
    out = ctx.loop_detect(p, c, small.THR, qs, [(s, x.pose, x.node_index) for s, x in zip(scans, cands)])
    ref = loopbatch.run_sharded(cands, loopbatch.hip_detect_fn(ctx, maps, cands, p, c, small.THR))
    assert bytes(out)[: len(cands) * loopbatch.RECORD_BYTES] == ref.tobytes()


def test_loop_detect_bad_queries(ctx):
    maps, cands = small.make_problem()
    p, c = abi.RtcsmParams(*small.PARAMS), abi.CostGEParams(*small.COST)
    g = ctx.grid_from_array(maps[0].cells, maps[0].min_x, maps[0].min_y, 0.05)
    s = ctx.scan(cands[0].ranges, cands[0].angles)
    with pytest.raises(abi.LgsError):   # gap in the candidate cover
        ctx.loop_detect(p, c, 0.6, [(g, None, (0, 0, 0), 0, 1, 1)], [(s, (0, 0, 0), 1), (s, (0, 0, 0), 2)])
    with pytest.raises(abi.LgsError):   # threshold outside (0, 1] (:21-22)
        ctx.loop_detect(p, c, 1.5, [(g, None, (0, 0, 0), 0, 0, 1)], [(s, (0, 0, 0), 1)])


def test_loop_detect_config5_json_window(ctx, world):
    """1081-beam candidates, the JSON loop window (+-2.5 m, +-0.5 rad), 500x500 maps."""
    import oracle_bind as ob

    def build(poses, ang):
        m = ob.OMap(0.05, 100, 500, 500)
        for q in poses:
            m.integrate(q, ob.OScan(scene.ray_cast(world, q, ang), ang), ob.BuilderParams(0.01, 20.0, 0.6, 0.45))
        return m.cells(), m.m.min_x, m.m.min_y, 0.05

    maps, cands = scene.loop_problem(world, build, n_maps=2, nodes_per_map=2, n_beams=1081, seed=21,
                                     perturb=(1.0, 0.3), arc_scans=8)
    p, c = abi.RtcsmParams(*LOOP_JSON), abi.CostGEParams(*small.COST)
    ctx.reset_stats()
    dev = loopbatch.run_sharded(cands, loopbatch.hip_detect_fn(ctx, maps, cands, p, c, 0.6))
    orc = loopbatch.run_sharded(cands, oracle_detect_fn(maps, cands, LOOP_JSON, small.COST, 0.6))
    compare(loopbatch.decode(dev), loopbatch.decode(orc))
    # the JSON window has 6 x 6 = 36 superblocks per angle (21 x 21 coarse
    # blocks at LowRes 5): superblock pruning runs, and scores fewer blocks
    # than the dense search (loop_detector_real_time_correlative.cpp:100-125)
    cnt = ctx.match_counters()
    assert cnt["matches"] == len(cands) and cnt["pruned"] == len(cands), cnt
    assert cnt["coarse_blocks"] < cnt["coarse_blocks_dense"], cnt
    ctx.set_option(abi.LGS_OPT_FORCE_DENSE, 1)
    try:
        ctx.reset_stats()
        dense = loopbatch.run_sharded(cands, loopbatch.hip_detect_fn(ctx, maps, cands, p, c, 0.6))
        cd = ctx.match_counters()
    finally:
        ctx.set_option(abi.LGS_OPT_FORCE_DENSE, 0)
    assert cd["pruned"] == 0 and cd["coarse_blocks"] == cd["coarse_blocks_dense"] == cnt["coarse_blocks_dense"], cd
    assert dense.tobytes() == dev.tobytes()


@pytest.mark.parametrize("n_shards", [2, 3])
def test_loop_detect_multi_context_identical(ctx, n_shards):
    """lgs_loop_detect_rtcsm_multi: the candidates split over more contexts
    (here all on GPU 0, one host thread each, maps and scans copied over) give
    byte-identical records to the one-context call (the
    multi-GPU form of the backend's single Detect call,
    lidar_graph_slam_backend.cpp:39-40)."""
    maps, cands = small.make_problem()
    p, c = abi.RtcsmParams(*small.PARAMS), abi.CostGEParams(*small.COST)
    grids = [ctx.grid_from_array(m.cells, m.min_x, m.min_y, m.res) for m in maps]
    coarse = [ctx.precompute_max(g, small.PARAMS[0]) if i % 2 == 0 else None for i, g in enumerate(grids)]
    scans = [ctx.scan(x.ranges, x.angles) for x in cands]
    qs, first = [], 0
    for qi, m in enumerate(maps):
        n = sum(1 for x in cands if x.query == qi)
        qs.append((grids[qi], coarse[qi], m.node_pose, m.node_index, first, n))
        first += n
    cl = [(s, x.pose, x.node_index) for s, x in zip(scans, cands)]
    one = bytes(ctx.loop_detect(p, c, small.THR, qs, cl))
    others = [abi.Context(0) for _ in range(n_shards - 1)]
    try:
        multi = bytes(ctx.loop_detect(p, c, small.THR, qs, cl, shards=others))
        again = bytes(ctx.loop_detect(p, c, small.THR, qs, cl, shards=others))
        direct = [o.copy_counters() for o in others]
        # the fallback for devices without peer access: maps staged through
        # pinned host memory (forced here, on one device)
        for o in others:
            o.set_option(abi.LGS_OPT_PEER_COPY, 1)
        staged = bytes(ctx.loop_detect(p, c, small.THR, qs, cl, shards=others))
        after = [o.copy_counters() for o in others]
        with pytest.raises(abi.LgsError):   # the single-context contract holds (:21-22)
            ctx.loop_detect(p, c, 1.5, qs, cl, shards=others)
    finally:
        for o in others:
            o.close()
    assert multi == one
    assert again == one
    assert staged == one
    assert all(d["direct"] > 0 and d["staged"] == 0 for d in direct), direct
    assert all(a["staged"] > 0 and a["direct"] == d["direct"] for a, d in zip(after, direct)), (after, direct)
    assert len(cands) >= n_shards


def test_loop_detect_config5_shape(ctx, world):
    """BASELINE config 5 at its own shape: 600x600 @ 5 cm local
    maps built by the oracle's UpdateGridMap, 1081-beam candidates whose
    initial poses are perturbed by U(+-2 m, +-0.4 rad), the JSON loop window
    (+-2.5 m, +-0.5 rad, LowRes 5, threshold 0.6,
    launcher_settings_default.json:102-126), 32 candidates over 8 maps --
    the pruned device batch against the oracle's Detect, record by record
    (loop_detector_real_time_correlative.cpp:26-125)."""
    import oracle_bind as ob

    def build(poses, ang):
        m = ob.OMap(0.05, 100, 600, 600)
        for q in poses:
            m.integrate(q, ob.OScan(scene.ray_cast(world, q, ang), ang), ob.BuilderParams(0.01, 20.0, 0.6, 0.45))
        return m.cells(), m.m.min_x, m.m.min_y, 0.05

    maps, cands = scene.loop_problem(world, build, n_maps=8, nodes_per_map=4, n_beams=1081, seed=33,
                                     perturb=(2.0, 0.4), arc_scans=10)
    assert all(m.cells.shape == (600, 600) for m in maps)
    p, c = abi.RtcsmParams(*LOOP_JSON), abi.CostGEParams(*small.COST)
    ctx.reset_stats()
    dev = loopbatch.run_sharded(cands, loopbatch.hip_detect_fn(ctx, maps, cands, p, c, 0.6))
    cnt = ctx.match_counters()
    orc = loopbatch.run_sharded(cands, oracle_detect_fn(maps, cands, LOOP_JSON, small.COST, 0.6))
    compare(loopbatch.decode(dev), loopbatch.decode(orc))
    found = loopbatch.loop_results(dev)
    assert 0 < len(found) <= len(cands)
    assert cnt["pruned"] == len(cands) and cnt["coarse_blocks"] < cnt["coarse_blocks_dense"], cnt


def test_loop_records_allgather_world1(ctx):
    """lgs_loop_records_allgather over an RCCL communicator of one rank: the
    records of a real loop batch come back byte for byte (the multi-process
    path's collective; N > 1 runs on the driver's nodes)."""
    import ctypes as C

    maps, cands = small.make_problem()
    p, c = abi.RtcsmParams(*small.PARAMS), abi.CostGEParams(*small.COST)
    rec = loopbatch.run_sharded(cands, loopbatch.hip_detect_fn(ctx, maps, cands, p, c, small.THR))
    n = len(cands)
    local = (abi.LoopResult * n).from_buffer_copy(rec.tobytes())
    comm = ctx.rccl_comm(1, 0)
    try:
        out = ctx.loop_records_allgather(comm, 0, 1, n, list(local))
        assert bytes(out) == rec.tobytes()
        assert bytes(ctx.loop_records_allgather(comm, 0, 1, 0, [])) == bytes(C.sizeof(abi.LoopResult))
    finally:
        ctx.rccl_comm_destroy(comm)


def test_run_sharded_rccl_world1(ctx):
    """bench.py's N > 1 loop line gathers through loopbatch.RcclGather (the
    library's lgs_loop_records_allgather): at one rank it returns the records
    run_sharded returns, byte for byte, call after call."""
    maps, cands = small.make_problem()
    p, c = abi.RtcsmParams(*small.PARAMS), abi.CostGEParams(*small.COST)
    fn = loopbatch.hip_detect_fn(ctx, maps, cands, p, c, small.THR)
    want = loopbatch.run_sharded(cands, fn)
    gather = loopbatch.RcclGather(ctx, 0, 1)
    try:
        for _ in range(3):
            assert loopbatch.run_sharded_rccl(cands, fn, gather).tobytes() == want.tobytes()
    finally:
        gather.close()
