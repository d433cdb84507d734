"""The device build of csrc/glibc_math.hpp against the host's libm, bit for
bit (lgs_debug_libm): glibc's sincos() over every branch of its algorithm and
pow(x, 3.0) over the bicubic kernel's arguments -- what makes the K4 refine
(and every other device recomputation that uses them) the oracle's arithmetic."""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

LIBM = C.CDLL("/lib/x86_64-linux-gnu/libm.so.6")
LIBM.sincos.argtypes = [C.c_double, C.POINTER(C.c_double), C.POINTER(C.c_double)]
LIBM.pow.restype = C.c_double
LIBM.pow.argtypes = [C.c_double, C.c_double]


def host_sincos(x):
    s, c = C.c_double(), C.c_double()
    out = np.empty((len(x), 2))
    for i, v in enumerate(x):
        LIBM.sincos(float(v), C.byref(s), C.byref(c))
        out[i] = (s.value, c.value)
    return out


def test_device_sincos_equals_libm(ctx):
    rng = np.random.default_rng(5)
    xs = np.concatenate([rng.uniform(-lo, lo, 40000) for lo in (2.0 ** -27, 0.13, 0.86, 2.43, 7.0, 1e5)] +
                        [np.array([0.0, -0.0, 0.126, -0.126, 0.85546875, 2.426265, np.pi, -np.pi / 2])])
    dev = ctx.debug_libm(0, xs)
    host = host_sincos(xs)
    assert np.array_equal(dev.view(np.uint64), host.view(np.uint64))


def test_device_pow3_equals_libm(ctx):
    rng = np.random.default_rng(6)
    v = 200 + rng.integers(0, 800, 100000) + np.ldexp(np.floor(np.ldexp(rng.random(100000), 44)), -44)
    f = v - np.floor(v)
    xs = np.concatenate([rng.uniform(0, 2, 100000), 1 + f, f, 1 - f, 2 - f, [0.0, 1.0, 2.0, 0.5]])
    dev = ctx.debug_libm(1, xs)
    host = np.array([LIBM.pow(float(x), 3.0) for x in xs])
    assert np.array_equal(dev.view(np.uint64), host.view(np.uint64))
