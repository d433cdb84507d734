"""The K3 sort (csrc/k_sort.hip): the hand-written stable LSD radix sort that
orders every ray-cast pass's keys by cell (C/mapping/grid_map_builder.cpp:170-186
applies a cell's updates in ray order, so the sort must be stable).  Checked
against numpy's stable argsort on the same bit field, key for key, for empty,
tiny, ragged and multi-million inputs, one- to four-pass bit ranges, and the
clustered, nearly sorted key streams a Bresenham ray-cast emits."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def expected(keys, lo, bits):
    f = (keys >> np.uint32(lo)) & np.uint32((1 << bits) - 1) if bits < 32 else keys
    return keys[np.argsort(f, kind="stable")]


@pytest.mark.parametrize("n,lo,bits", [(0, 1, 20), (1, 1, 20), (63, 1, 8), (1000, 1, 8), (4097, 1, 9),
                                       (100_000, 1, 21), (300_001, 5, 20), (65_536, 0, 32), (5000, 1, 0),
                                       (2_500_000, 1, 22), (3_000_003, 5, 24)])
def test_keysort_random(ctx, n, lo, bits):
    rng = np.random.default_rng(n + 7 * bits)
    keys = rng.integers(0, 2 ** 32, n, dtype=np.uint64).astype(np.uint32)
    got = ctx.debug_keysort(keys, lo, bits)
    assert np.array_equal(got, expected(keys, lo, bits))


def test_keysort_ray_like(ctx):
    """Keys as k_emit writes them: per ray a run of distinct cells along a line,
    many rays through the cells next to the sensor, hit bit in bit 0 -- equal
    cells must keep ray order (the low bits carry the ray index here)."""
    rng = np.random.default_rng(3)
    W = 900
    keys = []
    for s in range(12):
        sx, sy = rng.integers(300, 600, 2)
        for r in range(1081):
            a = 2 * np.pi * r / 1081
            L = int(rng.integers(1, 300))
            t = np.arange(L)
            x = (sx + np.round(t * np.cos(a))).astype(np.int64)
            y = (sy + np.round(t * np.sin(a))).astype(np.int64)
            cell = y * W + x
            k = (cell << 5) | ((s & 15) << 1) | (t == L - 1)
            keys.append(k.astype(np.uint32))
    keys = np.concatenate(keys)
    for lo, bits in ((5, 20), (1, 24)):
        got = ctx.debug_keysort(keys, lo, bits)
        assert np.array_equal(got, expected(keys, lo, bits))


def test_keysort_all_equal_digits(ctx):
    """Every key in one digit bucket (the look-back's worst case: one digit's
    run spans all tiles) and an already sorted / reverse-sorted input."""
    n = 1_500_000
    rng = np.random.default_rng(11)
    same = (np.full(n, 77, dtype=np.uint32) << 1) | rng.integers(0, 2, n).astype(np.uint32)
    assert np.array_equal(ctx.debug_keysort(same, 1, 16), expected(same, 1, 16))
    srt = np.sort(rng.integers(0, 2 ** 22, n).astype(np.uint32))
    assert np.array_equal(ctx.debug_keysort(srt, 0, 22), srt)
    rev = srt[::-1].copy()
    assert np.array_equal(ctx.debug_keysort(rev, 0, 22), expected(rev, 0, 22))


def test_keysort_coop_limit_takes_multipass(ctx):
    """LGS_OPT_COOP_TILES below a sort's tile count: the multi-pass sort runs
    instead of the one-launch k_sort_wide, same keys."""
    from lgs_amd import abi
    rng = np.random.default_rng(5)
    keys = rng.integers(0, 2 ** 32, 100_000, dtype=np.uint64).astype(np.uint32)   # 13 wide tiles
    try:
        for lim in (0, 3, -1):
            ctx.set_option(abi.LGS_OPT_COOP_TILES, lim)
            assert np.array_equal(ctx.debug_keysort(keys, 1, 20), expected(keys, 1, 20)), lim
    finally:
        ctx.set_option(abi.LGS_OPT_COOP_TILES, -1)


def test_keysort_barrier_timeout_fails_loudly(ctx):
    """A grid-barrier wait past LGS_OPT_SORT_BARRIER_US (0 here) ends every
    tile and reports LGS_ERR_INTERNAL instead of spinning; the barrier words
    are reset, so the next sort is right."""
    from lgs_amd import abi
    rng = np.random.default_rng(6)
    keys = rng.integers(0, 2 ** 32, 100_000, dtype=np.uint64).astype(np.uint32)
    try:
        ctx.set_option(abi.LGS_OPT_SORT_BARRIER_US, 0)
        with pytest.raises(abi.LgsError, match="grid barrier timed out"):
            ctx.debug_keysort(keys, 1, 20)
    finally:
        ctx.set_option(abi.LGS_OPT_SORT_BARRIER_US, 50000)
    for _ in range(2):
        assert np.array_equal(ctx.debug_keysort(keys, 1, 20), expected(keys, 1, 20))


def test_keysort_concurrent_contexts(ctx):
    """Four contexts sorting at once from four host threads, each sort close to
    the device's co-residency capacity: together they exceed it, so the
    process-wide reservation sends some to the multi-pass sort -- every result
    right, no barrier time-out."""
    import threading

    from lgs_amd import abi
    ctxs = [abi.Context(0) for _ in range(4)]
    rng = np.random.default_rng(8)
    inputs = [rng.integers(0, 2 ** 32, n, dtype=np.uint64).astype(np.uint32)
              for n in (900_000, 700_000, 1_000_000, 800_000)]
    errs = []

    def run(i):
        try:
            for k in range(6):
                got = ctxs[i].debug_keysort(inputs[i], 1, 20)
                if not np.array_equal(got, expected(inputs[i], 1, 20)):
                    errs.append((i, k, "mismatch"))
        except Exception as e:   # noqa: BLE001 -- reported below
            errs.append((i, repr(e)))

    th = [threading.Thread(target=run, args=(i,)) for i in range(4)]
    try:
        for t in th:
            t.start()
        for t in th:
            t.join()
    finally:
        for c in ctxs:
            c.close()
    assert not errs, errs
