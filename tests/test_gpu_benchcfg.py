"""Parity of the configuration bench.py times.

bench.py's default line times lgs_rtcsm_optimize_pose_query_batch on config 2
(1081 beams, +-2 m / +-30 deg, 1000x1000 @ 5 cm, LowRes 5): calls of 128
queries (two 64-query chunks, both buffer banks in flight), 3 lgs_ctx on one
GPU, each driven from its own host thread (bench.py run_match).  This test
runs exactly that -- bench.py's own map, scans and initial guesses -- and
checks the records against the oracle (OptimizePose(query),
C/mapping/scan_matcher_real_time_correlative.cpp:31-145): 16 records per
context, spread over both chunks; every other record against the lone call
(lgs_rtcsm_optimize_pose_query, the k_coarse_rows / k_fine path) field by
field, coarse_blocks included.

The batched kernels' other shapes are covered beside it: a +-4.5 m window
(nsb2 = 100 superblocks per angle: no superblock pruning, the dense batched
k_coarse) and scans with more than 2048 and 4096 valid beams (past the
pruned path's LDS rows: dense k_coarse, generic fine evaluator).
"""
import ctypes as C
import importlib.util
import os
import threading
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

import oracle_bind as ob
from conftest import ROOT, launcher_cost
from lgs_amd import abi, scene
from test_gpu_rtcsm import assert_same, build_map, oracle_match

pytestmark = pytest.mark.gpu


def _bench():
    spec = importlib.util.spec_from_file_location("lgs_bench", os.path.join(ROOT, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def _threads():
    return max(1, min(16, int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))))


def _lone_equal(b, one, tag, blocks=True):
    assert b.pose_found == one.pose_found, tag
    assert list(b.best_win) == list(one.best_win), tag
    assert b.score_max == one.score_max, tag
    assert b.estimated_pose.tuple() == one.estimated_pose.tuple(), tag
    assert b.normalized_cost == one.normalized_cost, tag
    assert list(b.covariance) == list(one.covariance), tag
    if blocks:
        assert b.coarse_blocks == one.coarse_blocks, (tag, b.coarse_blocks, one.coarse_blocks)


@pytest.fixture(scope="module")
def bench_problem(world):
    bm = _bench()
    ang = scene.beam_angles(1081)
    cells, mx, my = bm.bench_map(world, ang)
    scans, inits, truths = bm.random_scans(world, ang, np.random.default_rng(1000), 256)
    return bm, ang, cells, mx, my, scans, inits, truths


def test_bench_configuration_three_contexts(ctx, bench_problem):
    """3 contexts x 3 threads, two 128-query calls each (steps k = i and
    k = i + 3 of bench.py's loop after its 10 warmup calls)."""
    bm, ang, cells, mx, my, scans, inits, _ = bench_problem
    P, cost = abi.RtcsmParams(*bm.PARAMS), abi.CostGEParams(*bm.COST)
    B, S, n = 128, 3, len(scans)
    ctxs = [ctx] + [abi.Context(0) for _ in range(S - 1)]
    try:
        state = [(c, c.grid_from_array(cells, mx, my, 0.05), [c.scan(r, ang) for r in scans]) for c in ctxs]
        for c, _, _ in state:
            c.reset_stats()
        calls = {i: [10 + i, 10 + i + S] for i in range(S)}
        got, errs = {}, []

        def stream(i):
            try:
                c, g, ds = state[i]
                for k in calls[i]:
                    js = [(k * B + q) % n for q in range(B)]
                    got[(i, k)] = (js, c.optimize_pose_query_batch(g, P, cost, [ds[j] for j in js],
                                                                   [inits[j] for j in js]))
            except Exception as e:   # noqa: BLE001 -- reported below
                errs.append((i, e))

        th = [threading.Thread(target=stream, args=(i,)) for i in range(S)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        assert not errs, errs
        for c, _, _ in state:
            mc = c.match_counters()
            assert mc["matches"] == 2 * B and mc["pruned"] == 2 * B, mc   # the pruned work-list path ran
        # 16 records per context against the oracle: both chunks of both calls
        pick = [(i, calls[i][u], q) for i in range(S) for u, qs in enumerate([range(0, 64, 8), range(64, 128, 8)])
                for q in qs]
        assert len(pick) == 16 * S

        def oracle(p):
            i, k, q = p
            j = got[(i, k)][0][q]
            return oracle_match(cells, mx, my, 0.05, bm.PARAMS, scans[j], ang, inits[j])

        with ThreadPoolExecutor(_threads()) as ex:
            ora = list(ex.map(oracle, pick))
        for (i, k, q), o in zip(pick, ora):
            assert_same(got[(i, k)][1][q], o, f"ctx{i} call{k} q{q}")
        # every record against the lone call on its own context (the batch's
        # wide seed -- LGS_OPT_SEED_WIDE -- prunes more than the lone call's
        # one-launch seed: the blocks scored may only shrink on the whole)
        lone_blocks, batch_blocks = [], []
        for (i, k), (js, recs) in got.items():
            c, g, ds = state[i]
            for q, (j, b) in enumerate(zip(js, recs)):
                one = c.optimize_pose_query(g, P, cost, ds[j], inits[j])
                _lone_equal(b, one, f"ctx{i} call{k} q{q}", blocks=False)
                lone_blocks.append(one.coarse_blocks)
                batch_blocks.append(b.coarse_blocks)
            # the superblock pruning scores a small fraction of the ~421 x 17 x 17 blocks
            assert np.mean([b.coarse_blocks for b in recs]) < 0.1 * 421 * 17 * 17
        assert sum(batch_blocks) <= sum(lone_blocks), (sum(batch_blocks), sum(lone_blocks))
    finally:
        for c in ctxs[1:]:
            c.close()


def test_bench_configuration_repeatable(ctx, bench_problem):
    """The same 128-query call twice in a row and after a call with other
    queries: identical records (the banks alternate between calls)."""
    bm, ang, cells, mx, my, scans, inits, _ = bench_problem
    P, cost = abi.RtcsmParams(*bm.PARAMS), abi.CostGEParams(*bm.COST)
    g = ctx.grid_from_array(cells, mx, my, 0.05)
    ds = [ctx.scan(r, ang) for r in scans[:192]]
    rec = lambda outs: [(o.pose_found, list(o.best_win), o.score_max, o.estimated_pose.tuple(),   # noqa: E731
                         o.normalized_cost, list(o.covariance), o.coarse_blocks, o.fine_blocks) for o in outs]
    a = rec(ctx.optimize_pose_query_batch(g, P, cost, ds[:128], inits[:128]))
    b = rec(ctx.optimize_pose_query_batch(g, P, cost, ds[:128], inits[:128]))
    ctx.optimize_pose_query_batch(g, P, cost, ds[64:192], inits[64:192])
    c = rec(ctx.optimize_pose_query_batch(g, P, cost, ds[:128], inits[:128]))
    assert a == b == c


def test_batch_wide_window_dense(ctx, world):
    """+-4.5 m window: 37 x 37 coarse blocks, 100 superblocks per angle
    (nsb2 > 64): the batch is not pruned and runs the dense batched k_coarse."""
    cells, mx, my = build_map(world, 400, 0.05, 100, scene.arc_poses(5), n_beams=541)
    ang = scene.beam_angles(541)
    rng = np.random.default_rng(45)
    params = (5, 9.0, 9.0, 0.2, 20.0)
    P, cost = abi.RtcsmParams(*params), launcher_cost()
    g = ctx.grid_from_array(cells, mx, my, 0.05)
    qs = []
    for _ in range(5):
        true = (rng.uniform(-1, 1), rng.uniform(-1, 1), rng.uniform(-np.pi, np.pi))
        qs.append((scene.ray_cast(world, true, ang), (true[0] + rng.uniform(-0.5, 0.5),
                                                       true[1] + rng.uniform(-0.5, 0.5), true[2] + 0.05)))
    scans = [ctx.scan(r, ang) for r, _ in qs]
    ctx.reset_stats()
    batch = ctx.optimize_pose_query_batch(g, P, cost, scans, [i for _, i in qs])
    mc = ctx.match_counters()
    assert mc["matches"] == 5 and mc["pruned"] == 0, mc
    with ThreadPoolExecutor(_threads()) as ex:
        ora = list(ex.map(lambda q: oracle_match(cells, mx, my, 0.05, params, q[0], ang, q[1]), qs))
    for j, (b, o) in enumerate(zip(batch, ora)):
        assert list(b.win)[:2] == [90, 90]
        assert_same(b, o, f"wide q{j}")


@pytest.mark.parametrize("n_beams", [2500, 4500])
def test_batch_many_valid_beams(ctx, world, n_beams):
    """More valid beams than the pruned path's LDS rows hold (2048; and past
    k_coarse_list's 4096): dense batched k_coarse + the generic fine path."""
    cells, mx, my = build_map(world, 300, 0.05, 100, scene.arc_poses(4), n_beams=541)
    ang = scene.beam_angles(n_beams)
    rng = np.random.default_rng(n_beams)
    params = (5, 0.5, 0.5, 0.2, 20.0)
    P, cost = abi.RtcsmParams(*params), launcher_cost()
    g = ctx.grid_from_array(cells, mx, my, 0.05)
    qs = []
    for k in range(4):
        true = (rng.uniform(-1, 1), rng.uniform(-1, 1), rng.uniform(-np.pi, np.pi))
        r = scene.ray_cast(world, true, ang)
        if k == 1:
            r = np.where(np.arange(n_beams) % 5 == 0, 25.0, r)   # a smaller Nv in the same batch
        qs.append((r, (true[0] + rng.uniform(-0.2, 0.2), true[1] + rng.uniform(-0.2, 0.2), true[2] + 0.03)))
    scans = [ctx.scan(r, ang) for r, _ in qs]
    ctx.reset_stats()
    batch = ctx.optimize_pose_query_batch(g, P, cost, scans, [i for _, i in qs])
    mc = ctx.match_counters()
    assert mc["matches"] == 4 and mc["pruned"] == 0, mc
    with ThreadPoolExecutor(_threads()) as ex:
        ora = list(ex.map(lambda q: oracle_match(cells, mx, my, 0.05, params, q[0], ang, q[1]), qs))
    for j, ((r, init), b, o) in enumerate(zip(qs, batch, ora)):
        assert int(np.sum(r < 20.0)) > 2048 or j == 1
        assert_same(b, o, f"nv q{j}")
        one = ctx.optimize_pose_query(g, P, cost, scans[j], init)
        # (q1 alone has <= 2048 valid beams: its lone match is pruned, the batch's is not)
        _lone_equal(b, one, f"nv lone q{j}", blocks=j != 1)
