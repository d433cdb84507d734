"""Lean projection (LGS_OPT_LEAN_PROJECT).

k_project does not run: k_beams writes per-beam (range, cos, sin) and
per-angle (cos, sin) tables, and every kernel of the batched pruned chain that
stages a superblock-base, coarse-base or cell row forms it itself with the
projection's own arithmetic (k_super_oct's lean_super_row, lean_cell), guard
records and edge flags included.  Round 5's timing
experiment "nowrite" skipped the same writes WITHOUT the consumers forming
their rows: they gathered through stale plane offsets and the batch faulted
(an illegal memory access).  These tests pin the contract:

* records bit-identical to the materialised rows (lean off), on bench.py's
  own config-2 workload and against the oracle;
* with LGS_OPT_POISON_WS every workspace byte is 0xFF before the batch: a
  consumer still reading an unwritten row would gather through offset -1 and
  change a score; and the rows really are left unwritten (still 0xFF);
* forced guard fix-ups (LGS_OPT_INJECT_INDEX: every guarded cell shifted, in
  k_project AND in lean_cell): the batch's host fix-up reruns materialise
  rows and the records still equal the oracle's.
"""
import numpy as np
import pytest

from conftest import launcher_cost
from lgs_amd import abi
from test_gpu_batch import _diff, _record
from test_gpu_benchcfg import bench_problem  # noqa: F401 (fixture)
from test_gpu_rtcsm import assert_same, oracle_match

pytestmark = pytest.mark.gpu

PARAMS = (5, 4.0, 4.0, 1.0471976, 20.0)   # bench.py config 2


def _batch(ctx, g, P, cost, scans, inits, lean, poison=0, inject=0, geps=1e-9):
    ctx.set_option(abi.LGS_OPT_LEAN_PROJECT, lean)
    ctx.set_option(abi.LGS_OPT_POISON_WS, poison)
    ctx.set_option(abi.LGS_OPT_INJECT_INDEX, inject)
    ctx.set_option(abi.LGS_OPT_GUARD_EPS, geps)
    try:
        return ctx.optimize_pose_query_batch(g, P, cost, scans, inits)
    finally:
        ctx.set_option(abi.LGS_OPT_LEAN_PROJECT, 1)
        ctx.set_option(abi.LGS_OPT_POISON_WS, 0)
        ctx.set_option(abi.LGS_OPT_INJECT_INDEX, 0)
        ctx.set_option(abi.LGS_OPT_GUARD_EPS, 1e-9)


def test_lean_rows_same_records_config2(ctx, bench_problem):
    bm, ang, cells, mx, my, scans, inits, _ = bench_problem
    P, cost = abi.RtcsmParams(*PARAMS), launcher_cost()
    g = ctx.grid_from_array(cells, mx, my, 0.05)
    ds = [ctx.scan(r, ang) for r in scans[:64]]
    full = [_record(b) for b in _batch(ctx, g, P, cost, ds, inits[:64], lean=0)]
    lean_out = _batch(ctx, g, P, cost, ds, inits[:64], lean=1)
    lean = [_record(b) for b in lean_out]
    assert lean == full, _diff(lean, full)
    for j in (0, 31, 63):
        assert_same(lean_out[j], oracle_match(cells, mx, my, 0.05, PARAMS, scans[j], ang, inits[j]), f"q{j}")


def test_lean_rows_poisoned_workspace(ctx, bench_problem):
    """Poisoned workspaces: identical records, and the lean batch left the
    coarse-base and cell rows unwritten (0xFF) -- nothing read them."""
    bm, ang, cells, mx, my, scans, inits, _ = bench_problem
    P, cost = abi.RtcsmParams(*PARAMS), launcher_cost()
    g = ctx.grid_from_array(cells, mx, my, 0.05)
    ds = [ctx.scan(r, ang) for r in scans[64:96]]
    full = [_record(b) for b in _batch(ctx, g, P, cost, ds, inits[64:96], lean=0, poison=1)]
    lean = [_record(b) for b in _batch(ctx, g, P, cost, ds, inits[64:96], lean=1, poison=1)]
    assert lean == full, _diff(lean, full)
    for j in (0, 17):
        idx = ctx.debug_buffer("idx", j)
        assert (idx.view(np.uint8) == 0xFF).all(), j          # cells never written
        cb = ctx.debug_buffer("cbase", j)
        assert (cb.view(np.uint8) == 0xFF).all(), j           # coarse and superblock bases never written


def test_lean_rows_forced_guard_fixups(ctx, bench_problem):
    """LGS_OPT_INJECT_INDEX in a lean batch: every guarded projection is
    shifted on the device (k_project's guard records and lean_cell alike),
    the host re-checks the guards with glibc and reruns the item with
    patched, materialised rows -- records equal the lean-off run's and the
    oracle's, with fix-ups counted."""
    bm, ang, cells, mx, my, scans, inits, _ = bench_problem
    P, cost = abi.RtcsmParams(*PARAMS), launcher_cost()
    g = ctx.grid_from_array(cells, mx, my, 0.05)
    ds = [ctx.scan(r, ang) for r in scans[96:120]]
    # a guard band of 1e-5 cells (default 1e-9): ~20 guarded projections per
    # query, every one shifted and every one fixed up on the host
    full = _batch(ctx, g, P, cost, ds, inits[96:120], lean=0, inject=1, geps=1e-5)
    lean = _batch(ctx, g, P, cost, ds, inits[96:120], lean=1, inject=1, geps=1e-5)
    assert [_record(b) for b in lean] == [_record(b) for b in full], _diff([_record(b) for b in lean],
                                                                         [_record(b) for b in full])
    assert sum(b.fixups for b in lean) == len(ds) and min(b.guard_hits for b in lean) > 0
    plain = [_record(b) for b in _batch(ctx, g, P, cost, ds, inits[96:120], lean=1)]
    strip = lambda r: r[:6]   # noqa: E731 -- the result (a rerun's lone path counts its own blocks)
    assert [strip(_record(b)) for b in lean] == [strip(r) for r in plain]
    for j in (0, 11, 23):
        assert_same(lean[j], oracle_match(cells, mx, my, 0.05, PARAMS, scans[96 + j], ang, inits[96 + j]), f"q{j}")
