"""Loop-closure batch sharding (lgs_amd.loopbatch) on CPU: world sizes 1/2/3 over
gloo, with the oracle as the per-rank matcher, must give byte-identical
records in the reference's candidate order
(C/mapping/loop_detector_real_time_correlative.cpp:38-88)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from lgs_amd import loopbatch, scene

PARAMS = (5, 1.0, 1.0, 0.5, 20.0)                  # LowRes, rangeX, rangeY, rangeTheta, ScanRangeMax
COST = (0.01, 20.0, 0.075, 0.1, 1, 0.05, 1.0)       # launcher-built CostGreedyEndpoint
THR = 0.6                                           # LoopDetectorRealTimeCorrelative.ScoreThreshold (JSON)


def make_problem():
    import oracle_bind as ob
    world = scene.make_world()

    def build(poses, ang):
        m = ob.OMap(0.05, 100, 500, 500)
        for p in poses:
            m.integrate(p, ob.OScan(scene.ray_cast(world, p, ang), ang), ob.BuilderParams(0.01, 20.0, 0.6, 0.45))
        return m.cells(), m.m.min_x, m.m.min_y, 0.05

    return scene.loop_problem(world, build, n_maps=3, nodes_per_map=4, n_beams=121, seed=9, perturb=(0.3, 0.15),
                              arc_scans=6)


def test_shard_bounds_cover_in_order():
    for n in (0, 1, 7, 512, 513):
        for w in (1, 2, 3, 8):
            spans = [loopbatch.shard_bounds(n, w, r) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(spans[r][1] == spans[r + 1][0] for r in range(w - 1))
            sizes = [b - a for a, b in spans]
            assert max(sizes) - min(sizes) <= 1


def test_c_abi_shard_bounds_equal_python():
    """lgs_loop_shard_bounds (the C-ABI's sharding, lgs_coll.hip) == loopbatch.shard_bounds."""
    import ctypes as C

    from lgs_amd import abi
    lib = abi.load()
    lo, hi = C.c_int(), C.c_int()
    for n in (0, 1, 7, 64, 511, 512, 513):
        for w in (1, 2, 3, 4, 7, 8):
            for r in range(w):
                assert lib.lgs_loop_shard_bounds(n, w, r, C.byref(lo), C.byref(hi)) == 0
                assert (lo.value, hi.value) == loopbatch.shard_bounds(n, w, r), (n, w, r)
    assert lib.lgs_loop_shard_bounds(5, 2, 2, C.byref(lo), C.byref(hi)) == 1   # LGS_ERR_INVALID_ARG


def test_sub_queries_rebase():
    C = loopbatch.Candidate
    cands = [C(q, None, None, (0, 0, 0), i) for i, q in enumerate([0, 0, 1, 1, 1, 2])]
    assert loopbatch.sub_queries(cands, 1, 5) == [(0, 0, 1), (1, 1, 3)]
    assert loopbatch.sub_queries(cands, 0, 6) == [(0, 0, 2), (1, 2, 3), (2, 5, 1)]


def _worker(rank, world, port, out):
    import torch.distributed as dist
    from loop_oracle import oracle_detect_fn
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    maps, cands = make_problem()
    rec = loopbatch.run_sharded(cands, oracle_detect_fn(maps, cands, PARAMS, COST, THR), rank, world, dist)
    np.save(os.path.join(out, f"r{rank}.npy"), rec)
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_equals_single(tmp_path, world):
    from loop_oracle import oracle_detect_fn
    maps, cands = make_problem()
    single = loopbatch.run_sharded(cands, oracle_detect_fn(maps, cands, PARAMS, COST, THR))
    assert single.shape == (len(cands), loopbatch.RECORD_BYTES)
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    for r in range(world):
        got = np.load(tmp_path / f"r{r}.npy")
        assert got.tobytes() == single.tobytes()
    res = loopbatch.decode(single)
    found = loopbatch.loop_results(single)
    # order preserved, only found ones, indices as the reference builds them
    assert [r.end_node_index for r in found] == [r.end_node_index for r in res if r.found]
    assert all(r.start_node_index == maps[c.query].node_index for r, c in zip(res, cands))
    assert 0 < len(found) < len(cands)   # both outcomes exercised
