"""Pin the device's glibc restatements (csrc/glibc_math.hpp) against this
image's libm.so.6 on the CPU: the same header compiled for the host with
-ffp-contract=off (tests/cpp/libm_pin.cpp), compared bit for bit with libm's
sincos() and pow(x, 3.0) on seeded random inputs over every branch of the
algorithms (|x| < 2^-27, the table range, the pi/2 - x range, Cody-Waite
reduction; the bicubic kernel's pow arguments in [0, 2] including their
fixed-point forms 1 + f, f, 1 - f, 2 - f).  tests/test_gpu_libm.py checks the
device build of the same header against libm.

The constants and tables come from tools/gen_libm_consts.py, which reads them
from the libm whose sha256 it pins and re-derives the mathematical tables;
the GPU box runs the same image, so the reference's transcendental results
there are these.
"""
import ctypes as C
import hashlib
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "tests", "cpp", "build", "liblibm_pin.so")
LIBM = "/lib/x86_64-linux-gnu/libm.so.6"
LIBM_SHA256 = "e5141752c850ea45691513faadc577133fedf77bcbf19473f97e7247561254b2"


@pytest.fixture(scope="module")
def pin():
    assert os.path.exists(LIB), "build first: make -C <repo> all"
    lib = C.CDLL(LIB)
    for f in (lib.pin_sincos, lib.pin_sincos_avx2, lib.pin_pow3):
        f.restype = C.c_long
        f.argtypes = [C.c_uint64, C.c_long, C.c_double, C.c_double, C.c_int, C.POINTER(C.c_double)]
    return lib


def test_libm_is_the_pinned_build():
    with open(LIBM, "rb") as f:
        assert hashlib.sha256(f.read()).hexdigest() == LIBM_SHA256


@pytest.mark.parametrize("lo,hi", [(-2.0 ** -27, 2.0 ** -27), (-0.13, 0.13), (-0.86, 0.86), (-2.43, 2.43),
                                   (-7.0, 7.0), (-40.0, 40.0), (-1.05e8, 1.05e8)])
@pytest.mark.parametrize("mode", [0, 1])
def test_sincos_bit_exact(pin, lo, hi, mode):
    bad = C.c_double()
    n = pin.pin_sincos(11 + mode, 2_000_000, lo, hi, mode, C.byref(bad))
    assert n == 0, f"{n} mismatches, first at x = {bad.value!r}"


@pytest.mark.parametrize("lo,hi", [(-2.0 ** -27, 2.0 ** -27), (-0.13, 0.13), (-0.86, 0.86), (-2.43, 2.43),
                                   (-7.0, 7.0), (-40.0, 40.0), (-1.05e8, 1.05e8), (-2e8, 2e8)])
@pytest.mark.parametrize("mode", [0, 1])
def test_sincos_avx2_bit_exact(pin, lo, hi, mode):
    """The host's four-lane sincos (hit points of every map update) against libm."""
    bad = C.c_double()
    n = pin.pin_sincos_avx2(31 + mode, 2_000_000, lo, hi, mode, C.byref(bad))
    assert n == 0, f"{n} mismatches, first at x = {bad.value!r}"


@pytest.mark.parametrize("lo,hi", [(0.0, 2.0), (0.0, 1e-6), (0.999, 1.001), (1.999, 2.0)])
@pytest.mark.parametrize("mode", [0, 1])
def test_pow3_bit_exact(pin, lo, hi, mode):
    bad = C.c_double()
    n = pin.pin_pow3(21 + mode, 2_000_000, lo, hi, mode, C.byref(bad))
    assert n == 0, f"{n} mismatches, first at x = {bad.value!r}"


def test_special_values(pin):
    lib = C.CDLL(LIB)
    lib.glm_pow3.restype = C.c_double
    lib.glm_pow3.argtypes = [C.c_double]
    libm = C.CDLL(LIBM)
    libm.pow.restype = C.c_double
    libm.pow.argtypes = [C.c_double, C.c_double]
    for x in (0.0, 1.0, 2.0, 0.5, 1.5, 2.0 ** -44, 1 - 2.0 ** -53, 1 + 2.0 ** -52):
        assert lib.glm_pow3(x).hex() == libm.pow(x, 3.0).hex(), x
    lib.glm_sincos.argtypes = [C.c_double, C.POINTER(C.c_double), C.POINTER(C.c_double)]
    libm.sincos.argtypes = [C.c_double, C.POINTER(C.c_double), C.POINTER(C.c_double)]
    s0, c0, s1, c1 = C.c_double(), C.c_double(), C.c_double(), C.c_double()
    for x in (0.0, -0.0, 1e-300, 0.126, -0.126, 0.85546875, 2.426265, 3.141592653589793, -1.5707963267948966,
              1.054e8, 2.0 ** -27, -(2.0 ** -28)):
        libm.sincos(x, C.byref(s0), C.byref(c0))
        lib.glm_sincos(x, C.byref(s1), C.byref(c1))
        assert (s0.value.hex(), c0.value.hex()) == (s1.value.hex(), c1.value.hex()), x
