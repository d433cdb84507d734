"""GPU parity tests for the batched matcher (lgs_rtcsm_optimize_pose_query_batch
and the batched lgs_rtcsm_optimize_pose_batch / loop paths).

One launch per pipeline stage serves every query of a batch; each query must
still give exactly what a lone OptimizePose(query) gives (and the oracle):
bit-exact argmax window, score and pose, cost/covariance within 1e-5.  The
batches mix scans whose search-angle counts T and valid-beam counts Nv differ
(the kernels size their grids for the largest and per-item workgroups exit),
scans with no valid beam at all, different maps per query, and more queries
than one device batch holds (chunking).
"""
import numpy as np
import pytest

from conftest import launcher_cost
from lgs_amd import abi, scene
from test_gpu_rtcsm import assert_same, build_map, oracle_match

pytestmark = pytest.mark.gpu


def _queries(world, rng, n, n_beams, jitter=(0.3, 0.3, 0.2)):
    ang = scene.beam_angles(n_beams)
    out = []
    for _ in range(n):
        true = (rng.uniform(-1, 1), rng.uniform(-1, 1), rng.uniform(-np.pi, np.pi))
        r = scene.ray_cast(world, true, ang)
        init = (true[0] + rng.uniform(-jitter[0], jitter[0]), true[1] + rng.uniform(-jitter[1], jitter[1]),
                true[2] + rng.uniform(-jitter[2], jitter[2]))
        out.append((r, init))
    return ang, out


@pytest.fixture(scope="module")
def small_map(world):
    return build_map(world, 400, 0.05, 100, scene.arc_poses(5), n_beams=541)


def test_query_batch_matches_single_and_oracle(ctx, world, small_map):
    cells, mx, my = small_map
    rng = np.random.default_rng(7)
    ang, qs = _queries(world, rng, 10, 541)
    # vary T (max range -> angular step) and Nv (beams >= ScanRangeMax are dropped)
    qs[2] = (np.minimum(qs[2][0], 6.0), qs[2][1])
    qs[5] = (np.where(np.arange(541) % 3 == 0, 25.0, qs[5][0]), qs[5][1])
    qs[7] = (np.full(541, 25.0), qs[7][1])          # no valid beam at all
    params = (5, 1.0, 1.0, 0.6, 20.0)
    P, cost = abi.RtcsmParams(*params), launcher_cost()
    g = ctx.grid_from_array(cells, mx, my, 0.05)
    scans = [ctx.scan(r, ang) for r, _ in qs]
    inits = [i for _, i in qs]
    batch = ctx.optimize_pose_query_batch(g, P, cost, scans, inits)
    for j, ((r, init), b) in enumerate(zip(qs, batch)):
        one = ctx.optimize_pose_query(g, P, cost, scans[j], init)
        assert list(b.best_win) == list(one.best_win), j
        assert b.score_max == one.score_max, j
        assert b.estimated_pose.tuple() == one.estimated_pose.tuple(), j
        assert b.normalized_cost == one.normalized_cost, j
        assert list(b.covariance) == list(one.covariance), j
        assert_same(b, oracle_match(cells, mx, my, 0.05, params, r, ang, init), f"q{j}")


def test_query_batch_distinct_maps(ctx, world):
    """Each query carries its own map (same size): its own coarse map."""
    rng = np.random.default_rng(11)
    maps = [build_map(world, 300, 0.05, 100, scene.arc_poses(k + 2), n_beams=361) for k in range(3)]
    ang, qs = _queries(world, rng, 6, 361)
    params = (5, 0.8, 0.8, 0.5, 20.0)
    P, cost = abi.RtcsmParams(*params), launcher_cost()
    grids = [ctx.grid_from_array(c, mx, my, 0.05) for c, mx, my in maps]
    which = [j % 3 for j in range(6)]
    scans = [ctx.scan(r, ang) for r, _ in qs]
    batch = ctx.optimize_pose_query_batch([grids[w] for w in which], P, cost, scans, [i for _, i in qs])
    for j, ((r, init), b) in enumerate(zip(qs, batch)):
        c, mx, my = maps[which[j]]
        assert_same(b, oracle_match(c, mx, my, 0.05, params, r, ang, init), f"q{j}")


def test_query_batch_chunked(ctx, world):
    """More queries than one device batch (kMaxBatch = 64): chunked, same results."""
    cells, mx, my = build_map(world, 200, 0.05, 100, scene.arc_poses(3), n_beams=181)
    rng = np.random.default_rng(3)
    ang, qs = _queries(world, rng, 70, 181, jitter=(0.1, 0.1, 0.1))
    params = (5, 0.4, 0.4, 0.3, 20.0)
    P, cost = abi.RtcsmParams(*params), launcher_cost()
    g = ctx.grid_from_array(cells, mx, my, 0.05)
    scans = [ctx.scan(r, ang) for r, _ in qs]
    batch = ctx.optimize_pose_query_batch(g, P, cost, scans, [i for _, i in qs])
    for j in (0, 1, 63, 64, 69):
        r, init = qs[j]
        assert_same(batch[j], oracle_match(cells, mx, my, 0.05, params, r, ang, init), f"q{j}")


def test_query_batch_fixups_and_dense(ctx, world, small_map):
    """Guard fix-ups (injected index corruption) and the dense mode inside a batch."""
    cells, mx, my = small_map
    rng = np.random.default_rng(5)
    ang, qs = _queries(world, rng, 4, 541)
    params = (5, 1.0, 1.0, 0.6, 20.0)
    P, cost = abi.RtcsmParams(*params), launcher_cost()
    g = ctx.grid_from_array(cells, mx, my, 0.05)
    scans = [ctx.scan(r, ang) for r, _ in qs]
    ora = [oracle_match(cells, mx, my, 0.05, params, r, ang, init) for r, init in qs]
    try:
        ctx.set_option(abi.LGS_OPT_GUARD_EPS, 0.02)
        ctx.set_option(abi.LGS_OPT_INJECT_INDEX, 1)
        for j, b in enumerate(ctx.optimize_pose_query_batch(g, P, cost, scans, [i for _, i in qs])):
            assert b.fixups == 1, j
            assert_same(b, ora[j], f"inject q{j}")
        ctx.set_option(abi.LGS_OPT_INJECT_INDEX, 0)
        ctx.set_option(abi.LGS_OPT_GUARD_EPS, 1e-9)
        ctx.set_option(abi.LGS_OPT_FORCE_DENSE, 1)
        for j, b in enumerate(ctx.optimize_pose_query_batch(g, P, cost, scans, [i for _, i in qs])):
            assert_same(b, ora[j], f"dense q{j}")
    finally:
        ctx.set_option(abi.LGS_OPT_INJECT_INDEX, 0)
        ctx.set_option(abi.LGS_OPT_GUARD_EPS, 1e-9)
        ctx.set_option(abi.LGS_OPT_FORCE_DENSE, 0)


@pytest.mark.parametrize("prune", [1, 0])
def test_query_batch_layouts(ctx, world, small_map, prune):
    """Superblock pruning on and off give the same batch."""
    cells, mx, my = small_map
    rng = np.random.default_rng(9)
    ang, qs = _queries(world, rng, 5, 541)
    params = (5, 1.0, 1.0, 0.6, 20.0)
    P, cost = abi.RtcsmParams(*params), launcher_cost()
    g = ctx.grid_from_array(cells, mx, my, 0.05)
    scans = [ctx.scan(r, ang) for r, _ in qs]
    try:
        ctx.set_option(abi.LGS_OPT_SUPER_PRUNE, prune)
        batch = ctx.optimize_pose_query_batch(g, P, cost, scans, [i for _, i in qs])
    finally:
        ctx.set_option(abi.LGS_OPT_SUPER_PRUNE, 1)
    for j, ((r, init), b) in enumerate(zip(qs, batch)):
        assert_same(b, oracle_match(cells, mx, my, 0.05, params, r, ang, init), f"q{j}")


def test_query_batch_rejects_mixed_sizes(ctx, world):
    a = ctx.grid_from_array(np.zeros((100, 100)), -2.5, -2.5, 0.05)
    b = ctx.grid_from_array(np.zeros((120, 100)), -2.5, -2.5, 0.05)
    ang = scene.beam_angles(91)
    sc = ctx.scan(np.full(91, 2.0), ang)
    with pytest.raises(abi.LgsError):
        ctx.optimize_pose_query_batch([a, b], abi.RtcsmParams(5, 0.4, 0.4, 0.3, 20.0), launcher_cost(),
                                      [sc, sc], [(0, 0, 0), (0, 0, 0)])


@pytest.mark.parametrize("low_res,n_cells", [(5, 400), (4, 400), (2, 300), (8, 400)])
def test_query_planes_equal_supplied_coarse_planes(ctx, world, low_res, n_cells):
    """The query path writes the coarse planes straight from the batched
    precompute; OptimizePose with a caller coarse map builds them by the
    phase-plane copy: identical results, including the number of coarse
    blocks the superblock pruning scored (the pruning is a function of the
    call's inputs only)."""
    cells, mx, my = build_map(world, n_cells, 0.05, 100, scene.arc_poses(5), n_beams=541)
    rng = np.random.default_rng(low_res)
    ang, qs = _queries(world, rng, 4, 541)
    params = (low_res, 1.0, 1.0, 0.5, 20.0)
    P, cost = abi.RtcsmParams(*params), launcher_cost()
    g = ctx.grid_from_array(cells, mx, my, 0.05)
    cg = ctx.precompute_max(g, low_res)
    for j, (r, init) in enumerate(qs):
        sc = ctx.scan(r, ang)
        fused = ctx.optimize_pose_query(g, P, cost, sc, init)
        two = ctx.optimize_pose(g, cg, P, cost, sc, init, 2.2250738585072014e-308)
        assert list(fused.best_win) == list(two.best_win) and fused.score_max == two.score_max, j
        assert fused.coarse_blocks == two.coarse_blocks, (j, fused.coarse_blocks, two.coarse_blocks)
        assert_same(fused, oracle_match(cells, mx, my, 0.05, params, r, ang, init), f"lr{low_res} q{j}")


_FIELDS = ("found", "best_win", "score", "pose", "ncost", "cov", "coarse_blocks", "fine_blocks", "guard_hits",
           "fixups", "slow_path")


def _diff(a, b):
    return [(j, f, x, y) for j, (ra, rb) in enumerate(zip(a, b)) for f, x, y in zip(_FIELDS, ra, rb) if x != y]


def _buffers(ctx, n):
    out = [{b: ctx.debug_buffer(b, j) for b in ("sbound", "part_c", "part_k", "L", "tedge", "cbase", "idx")}
           for j in range(n)]
    for d in out:
        d["L"] = np.concatenate([d["L"][:1], d["L"][8:12]])   # Lp, Lc[0..3] (not the padding between)
    return out


def _buffer_diff(a, b):
    """first differing intermediate buffer of every item (diagnostics)"""
    out = []
    for j, (x, y) in enumerate(zip(a, b)):
        for name in x:
            u, v = x[name], y[name]
            if u.shape != v.shape or not np.array_equal(u.view(np.uint8), v.view(np.uint8)):
                k = int(np.argmax(u.view(np.uint8) != v.view(np.uint8))) // u.itemsize if u.shape == v.shape else -1
                out.append((j, name, k, u[k] if k >= 0 else u.shape, v[k] if k >= 0 else v.shape))
    return out


def _expected_blocks(bufs, ncx, ncy, thr):
    """coarse blocks the keep rule selects, recomputed on the host from an
    item's sbound / Lc / tedge (diagnostics)"""
    nsbx, nsby = (ncx + 3) // 4, (ncy + 3) // 4
    sb = bufs["sbound"].reshape(-1, nsbx * nsby)
    L = bufs["L"][1:5].max()
    tot = 0
    for t in range(sb.shape[0]):
        for i in range(nsbx * nsby):
            a, b = i % nsbx, i // nsbx
            if sb[t, i] > thr and (bufs["tedge"][t] or sb[t, i] >= L):
                tot += min(4, ncx - 4 * a) * min(4, ncy - 4 * b)
    return tot


def _record(out):
    return (out.pose_found, list(out.best_win), out.score_max, out.estimated_pose.tuple(), out.normalized_cost,
            list(out.covariance), out.coarse_blocks, out.fine_blocks, out.guard_hits, out.fixups, out.slow_path)


@pytest.mark.parametrize("poison", [0, 1])
def test_pruning_is_history_independent(ctx, world, small_map, poison):
    """Every record field -- including coarse_blocks, the superblock pruning's
    work and the roofline's algorithmic bytes -- is a function of the call's
    inputs only: call A, then calls that leave other contents in the
    workspace (another T and Nv, a batch, the dense path, the unpruned path),
    then A again.  With LGS_OPT_POISON_WS every workspace byte is 0xFF before
    each batch, so a read-before-write would change the result."""
    cells, mx, my = small_map
    rng = np.random.default_rng(21)
    ang, qs = _queries(world, rng, 4, 541)
    params = (5, 1.0, 1.0, 0.6, 20.0)
    P, cost = abi.RtcsmParams(*params), launcher_cost()
    g = ctx.grid_from_array(cells, mx, my, 0.05)
    scans = [ctx.scan(r, ang) for r, _ in qs]
    short = ctx.scan(np.where(np.arange(541) % 3 == 0, 25.0, np.minimum(qs[0][0], 5.0)), ang)
    ctx.set_option(abi.LGS_OPT_POISON_WS, poison)
    try:
        first = [_record(ctx.optimize_pose_query(g, P, cost, sc, i)) for sc, (_, i) in zip(scans, qs)]
        batch1 = [_record(b) for b in ctx.optimize_pose_query_batch(g, P, cost, scans, [i for _, i in qs])]
        snap1 = _buffers(ctx, len(scans))
        for k in range(3):
            ctx.optimize_pose_query(g, abi.RtcsmParams(5, 0.6, 0.6, 1.0, 20.0), cost, short, (0.1, 0.0, 0.3))
            ctx.optimize_pose_query_batch(g, P, cost, [short] + scans[:k + 1], [(0.0, 0.0, 0.0)] + [i for _, i in qs][:k + 1])
            if k == 1:
                ctx.set_option(abi.LGS_OPT_FORCE_DENSE, 1)
                ctx.optimize_pose_query(g, P, cost, scans[2], qs[2][1])
                ctx.set_option(abi.LGS_OPT_FORCE_DENSE, 0)
            if k == 2:
                ctx.set_option(abi.LGS_OPT_SUPER_PRUNE, 0)
                ctx.optimize_pose_query(g, P, cost, scans[1], qs[1][1])
                ctx.set_option(abi.LGS_OPT_SUPER_PRUNE, 1)
            again = [_record(ctx.optimize_pose_query(g, P, cost, sc, i)) for sc, (_, i) in zip(scans, qs)]
            assert again == first, (k, _diff(again, first))
            batch = [_record(b) for b in ctx.optimize_pose_query_batch(g, P, cost, scans, [i for _, i in qs])]
            if batch != batch1:
                snap = _buffers(ctx, len(scans))
                exp1 = [_expected_blocks(b, 5, 5, 0.0) for b in snap1]
                exp = [_expected_blocks(b, 5, 5, 0.0) for b in snap]
                for row in [k, _diff(batch, batch1), exp1, exp] + _buffer_diff(snap1, snap):
                    print("HISTORY-DIAG", row)
                assert batch == batch1, (k, _diff(batch, batch1), _buffer_diff(snap1, snap), exp1, exp)
    finally:
        ctx.set_option(abi.LGS_OPT_POISON_WS, 0)
        ctx.set_option(abi.LGS_OPT_FORCE_DENSE, 0)
        ctx.set_option(abi.LGS_OPT_SUPER_PRUNE, 1)


def test_scans_first_touched_by_two_contexts_at_once(ctx, world, small_map):
    """Fresh scans (no device copy yet) passed to two contexts' batches at the
    same moment, in opposite orders: whichever call copies a scan first
    publishes it, the other waits until that copy is enqueued and done
    (lgs::CopyFence) -- every record equals the one from scans copied
    beforehand."""
    import threading
    cells, mx, my = small_map
    rng = np.random.default_rng(33)
    ang, qs = _queries(world, rng, 8, 541)
    params = (5, 1.0, 1.0, 0.6, 20.0)
    P, cost = abi.RtcsmParams(*params), launcher_cost()
    other = abi.Context(0)
    try:
        grids = [ctx.grid_from_array(cells, mx, my, 0.05), other.grid_from_array(cells, mx, my, 0.05)]
        inits = [i for _, i in qs]
        ref = [_record(b) for b in ctx.optimize_pose_query_batch(grids[0], P, cost,
                                                                 [ctx.scan(r, ang) for r, _ in qs], inits)]
        for rnd in range(12):
            fresh = [ctx.scan(r, ang) for r, _ in qs]     # created, not yet copied
            got, errs = {}, []
            gate = threading.Barrier(2)

            def run(k):
                try:
                    order = list(range(8)) if k == 0 else list(range(7, -1, -1))
                    gate.wait()
                    c = (ctx, other)[k]
                    outs = c.optimize_pose_query_batch(grids[k], P, cost, [fresh[j] for j in order],
                                                       [inits[j] for j in order])
                    got[k] = {j: _record(o) for j, o in zip(order, outs)}
                except Exception as e:   # noqa: BLE001 -- reported below
                    errs.append((k, repr(e)))

            th = [threading.Thread(target=run, args=(k,)) for k in range(2)]
            for t in th:
                t.start()
            for t in th:
                t.join()
            assert not errs, errs
            for k in range(2):
                for j in range(8):
                    assert got[k][j] == ref[j], (rnd, k, j)
    finally:
        other.close()


@pytest.mark.parametrize("n_cells,low_edge", [(400, False), (401, False), (400, True)])
def test_fine_staged_equals_gathers(ctx, world, n_cells, low_edge):
    """The LDS-staged batched fine evaluator (k_fine_regs, LowRes 5, even W)
    == the per-beam gather one (k_fine_lanes) == the oracle, field for field;
    an odd-width map (401) takes the gather kernel either way, and a map
    cropped at its low edges puts windows across x = 0 / y = 0."""
    cells, mx, my = build_map(world, 600 if low_edge else n_cells, 0.05, 100, scene.arc_poses(5), n_beams=541)
    if low_edge:
        cells, mx, my = cells[40:440, 40:440].copy(), mx + 2.0, my + 2.0
    elif n_cells % 2:
        cells = cells[:, :n_cells]
    rng = np.random.default_rng(n_cells + low_edge)
    ang, qs = _queries(world, rng, 9, 541)
    if low_edge:
        qs = [(scene.ray_cast(world, (t[0] - 0.8, t[1] - 0.8, t[2]), ang), (t[0] - 0.7, t[1] - 0.9, t[2]))
              for (_, t) in qs]
    params = (5, 1.0, 1.0, 0.6, 20.0)
    P, cost = abi.RtcsmParams(*params), launcher_cost()
    g = ctx.grid_from_array(cells, mx, my, 0.05)
    scans = [ctx.scan(r, ang) for r, _ in qs]
    inits = [i for _, i in qs]
    try:
        ctx.set_option(abi.LGS_OPT_FINE_STAGED, 0)
        gath = [_record(b) for b in ctx.optimize_pose_query_batch(g, P, cost, scans, inits)]
        ctx.set_option(abi.LGS_OPT_FINE_STAGED, 1)
        stag = ctx.optimize_pose_query_batch(g, P, cost, scans, inits)
    finally:
        ctx.set_option(abi.LGS_OPT_FINE_STAGED, 1)
    assert [_record(b) for b in stag] == gath
    for j, ((r, init), b) in enumerate(zip(qs, stag)):
        assert_same(b, oracle_match(cells, mx, my, 0.05, params, r, ang, init), f"q{j}")


def test_wide_seed_same_records_less_coarse_work(ctx, world, small_map):
    """LGS_OPT_SEED_WIDE (the pruning bound seeded from 16 candidate
    superblocks' best members, batches): every record field equal to the
    4-candidate seed's but coarse_blocks / fine_blocks, the device's pruned
    work, which may only shrink in total; and the oracle's answer (a
    config-2-sized window)."""
    cells, mx, my = small_map
    rng = np.random.default_rng(33)
    ang, qs = _queries(world, rng, 12, 541)
    params = (5, 4.0, 4.0, 1.0, 20.0)
    P, cost = abi.RtcsmParams(*params), launcher_cost()
    g = ctx.grid_from_array(cells, mx, my, 0.05)
    scans = [ctx.scan(r, ang) for r, _ in qs]
    inits = [i for _, i in qs]
    try:
        ctx.set_option(abi.LGS_OPT_SEED_WIDE, 0)
        narrow = [_record(b) for b in ctx.optimize_pose_query_batch(g, P, cost, scans, inits)]
        ctx.set_option(abi.LGS_OPT_SEED_WIDE, 16)   # > 4 candidates: the two-launch wide seed runs
        wide = [_record(b) for b in ctx.optimize_pose_query_batch(g, P, cost, scans, inits)]
    finally:
        ctx.set_option(abi.LGS_OPT_SEED_WIDE, 12)   # the library default
    strip = lambda rec: rec[:6] + rec[8:]   # all but coarse_blocks / fine_blocks (the device's work)
    assert [strip(r) for r in wide] == [strip(r) for r in narrow], _diff(wide, narrow)
    for f in (6, 7):
        assert sum(r[f] for r in wide) <= sum(r[f] for r in narrow), ([r[f] for r in wide], [r[f] for r in narrow])
    for j in (0, 5, 11):
        out = ctx.optimize_pose_query_batch(g, P, cost, scans, inits)[j]
        assert_same(out, oracle_match(cells, mx, my, 0.05, params, qs[j][0], ang, inits[j]), f"q{j}")


@pytest.mark.parametrize("wide,theta", [(5, 1.0), (16, 1.0), (12, 3.1)])
def test_wide_seed_candidate_counts_and_large_searches(ctx, world, small_map, wide, theta):
    """The wide seed with its fewest (5) and most (16) candidates, and a
    search with more angle parts than one wave holds (+-3.1 rad: the batch
    falls back to the one-launch seed): records equal the 4-candidate seed's
    but for the device's work counters, which do not grow in total."""
    cells, mx, my = small_map
    rng = np.random.default_rng(51)
    ang, qs = _queries(world, rng, 6, 541)
    params = (5, 2.0, 2.0, theta, 20.0)
    P, cost = abi.RtcsmParams(*params), launcher_cost()
    g = ctx.grid_from_array(cells, mx, my, 0.05)
    scans = [ctx.scan(r, ang) for r, _ in qs]
    inits = [i for _, i in qs]
    try:
        ctx.set_option(abi.LGS_OPT_SEED_WIDE, 0)
        narrow = [_record(b) for b in ctx.optimize_pose_query_batch(g, P, cost, scans, inits)]
        ctx.set_option(abi.LGS_OPT_SEED_WIDE, wide)
        got = [_record(b) for b in ctx.optimize_pose_query_batch(g, P, cost, scans, inits)]
    finally:
        ctx.set_option(abi.LGS_OPT_SEED_WIDE, 12)
    strip = lambda rec: rec[:6] + rec[8:]   # all but coarse_blocks / fine_blocks
    assert [strip(r) for r in got] == [strip(r) for r in narrow], _diff(got, narrow)
    assert sum(r[6] for r in got) <= sum(r[6] for r in narrow)
    if theta > 3.0:   # the fallback: the very same seed, the very same work
        assert got == narrow
    out = ctx.optimize_pose_query_batch(g, P, cost, scans, inits)[2]
    assert_same(out, oracle_match(cells, mx, my, 0.05, params, qs[2][0], ang, inits[2]), "q2")


def test_zero_tiles_follow_map_changes(ctx, world):
    """LGS_OPT_ZERO_TILES: the per-map passes skip the stores of tiles whose
    inputs are all +0 when the set's buffer already holds their +0 outputs.
    One context with it (the default) and one without run the same calls --
    batches whose sets switch between maps with erased regions, a blob and a
    single nonzero cell in otherwise empty tiles, a lone query (its own
    precompute tiling) and batches with fewer and more sets -- and must leave
    the same records and bit-identical phase planes and superblock units."""
    base, mx, my = build_map(world, 600, 0.05, 100, scene.arc_poses(5), n_beams=541)
    a = base.copy()
    a[:, :250] = 0.0                         # erased: whole zero tiles
    b = base.copy()
    b[:200, :] = 0.0
    b[500:560, 20:80] = 0.7                  # a blob where a and base are empty
    c = base.copy()
    c[5, 5] = 0.3                            # one cell in an otherwise empty tile
    c[590, 300] = 0.2
    d = np.zeros_like(base)                  # nothing at all
    d[300:310, 300:310] = 0.9
    maps = {"a": a, "b": b, "c": c, "d": d, "base": base}
    other = abi.Context(0)
    try:
        other.set_option(abi.LGS_OPT_ZERO_TILES, 0)
        P, cost = abi.RtcsmParams(5, 1.0, 1.0, 0.6, 20.0), launcher_cost()
        rng = np.random.default_rng(31)
        ang, qs = _queries(world, rng, 6, 541)
        state = []
        for cx in (ctx, other):
            grids = {k: cx.grid_from_array(v, mx, my, 0.05) for k, v in maps.items()}
            scans = [cx.scan(r, ang) for r, _ in qs]
            state.append((cx, grids, scans))
        inits = [i for _, i in qs]
        calls = [["a", "a", "b", "c"], ["b", "c", "a", "a"], ["c"], ["c", "b", "a", "b"], ["d", "d"],
                 ["a", "c", "b"], ["base", "b", "c", "a", "d", "b"], ["a", "a", "b", "c"]]
        for step, names in enumerate(calls):
            res = []
            for cx, grids, scans in state:
                n = len(names)
                if n == 1:
                    out = [cx.optimize_pose_query(grids[names[0]], P, cost, scans[0], inits[0])]
                else:
                    out = cx.optimize_pose_query_batch([grids[k] for k in names], P, cost, scans[:n], inits[:n])
                recs = [_record(o) for o in out]
                bufs = [(cx.debug_buffer("planes", j), cx.debug_buffer("super", j)) for j in range(n)]
                res.append((recs, bufs))
            (r0, b0), (r1, b1) = res
            assert r0 == r1, (step, _diff(r0, r1))
            for j in range(len(names)):
                for name, u, v in (("planes", b0[j][0], b1[j][0]), ("super", b0[j][1], b1[j][1])):
                    assert u.shape == v.shape and np.array_equal(u.view(np.uint8), v.view(np.uint8)), \
                        (step, j, names[j], name, int(np.argmax(u.view(np.uint8) != v.view(np.uint8))))
    finally:
        other.close()
