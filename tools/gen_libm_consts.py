#!/usr/bin/env python3
"""Generate my-lidar-graph-slam_amd/csrc/libm_consts.h: the constants and
tables of this image's glibc libm (Ubuntu GLIBC 2.35-0ubuntu3.11, x86-64)
that the device restatements in csrc/glibc_math.hpp need to reproduce the
reference's transcendental calls bit for bit:

  * sincos()   -- glibc sysdeps/ieee754/dbl-64/s_sincos.c + s_sin.c (IBM
                  Accurate Mathematical Library: table-driven sin/cos around
                  x_i = i/128, Taylor polynomials, Cody-Waite reduction by
                  pi/2).  The reference's ComputeMapGradient / HitPoint pairs
                  of std::sin/std::cos of one argument are fused by GCC -O3
                  into one sincos() call.
  * pow(x, 3.0) -- glibc sysdeps/ieee754/dbl-64/e_pow.c (ARM optimized
                  routines: log_inline with a 128-entry table, exp_inline with
                  a 128-entry 2^(i/128) table); x86-64 dispatches the FMA
                  variant (__pow_fma) on every FMA-capable CPU (the resolver
                  tests CPUID FMA + AVX2), which is what runs on this image
                  and on the GPU box's host.

The values are read from libm.so.6 at the .rodata addresses the machine code
of sincos / __pow_fma references (found by disassembling this exact build;
the sha256 below pins it).  The purely mathematical tables are re-derived
here with 60-digit decimal arithmetic and asserted equal: sin/cos(i/128) as
(nearest double, nearest double of the remainder) and 2^(i/128) as
(scale bits - i<<45, tail).  The polynomial coefficients are minimax
constants of the published algorithms and are taken as they are.

Run: python3 tools/gen_libm_consts.py   (writes the header; needs the libm)
Pinned by tests/test_libm_pin.py (host restatement == libm on random inputs).
"""
import hashlib
import os
import struct
import sys
from decimal import Decimal, getcontext

LIBM = "/lib/x86_64-linux-gnu/libm.so.6"
SHA256 = "e5141752c850ea45691513faadc577133fedf77bcbf19473f97e7247561254b2"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "my-lidar-graph-slam_amd", "csrc", "libm_consts.h")

# .rodata addresses (== file offsets for .rodata in this build)
SINCOS = dict(big=0x9A8A8, sn5=0x9A8B0, neg_sn3=0x9A8B8, cs6=0x9A8C0, neg_cs4=0x9A8C8, cs2=0x8AAB0,
              taylor_max=0x9A878, hp0=0x93048, hp1=0x930B8, hpinv=0x969B8, toint=0x97010,
              mp1=0x9A8D0, mp2=0x9A8D8, pp3=0x9A8E0, pp4=0x9A8E8,
              s5=0x9A880, s4=0x9A888, neg_s3=0x9A890, s2=0x9A898, neg_s1=0x9A8A0)
SINCOSTAB = 0xAEB80          # __sincostab: {sin hi, sin lo, cos hi, cos lo} per x_i = i/128
SINCOSTAB_N = 110            # |x| < 0.85546875 = 109.5/128 -> i <= 109
POW_LOG = 0xB1B20            # __pow_log_data: ln2hi, ln2lo, poly[7], tab[128]{invc, pad, logc, logctail}
EXP_DATA = 0xAF960           # __exp_data: invln2N, shift, negln2hiN, negln2loN, poly[4], exp2..., tab[256] at +0x70
POW_MINUS_ONE = 0x969B0      # the -1.0 of fma(z, invc, -1.0)

getcontext().prec = 60


def d(buf, a):
    return struct.unpack("<d", buf[a:a + 8])[0]


def q(buf, a):
    return struct.unpack("<Q", buf[a:a + 8])[0]


def nearest(x: Decimal) -> float:
    """Round a Decimal to the nearest double (ties to even)."""
    f = float(x)              # correctly rounded by CPython (via repr-exact string)
    return f


def dsin(x: Decimal) -> Decimal:
    s, t, k = Decimal(0), x, 1
    while abs(t) > Decimal(10) ** -58:
        s += t
        t = -t * x * x / ((k + 1) * (k + 2))
        k += 2
    return s


def dcos(x: Decimal) -> Decimal:
    s, t, k = Decimal(0), Decimal(1), 0
    while abs(t) > Decimal(10) ** -58:
        s += t
        t = -t * x * x / ((k + 1) * (k + 2))
        k += 2
    return s


def hexf(v: float) -> str:
    return float.hex(v)


def main() -> int:
    buf = open(LIBM, "rb").read()
    sha = hashlib.sha256(buf).hexdigest()
    if sha != SHA256:
        print(f"libm sha256 {sha} != pinned {SHA256}: addresses are build-specific", file=sys.stderr)
        return 1
    c = {k: d(buf, a) for k, a in SINCOS.items()}
    assert c["big"] == 52776558133248.0 and c["toint"] == 6755399441055744.0 and c["cs2"] == 0.5
    assert c["taylor_max"] == 0.126 and c["hp0"] == 1.5707963267948966
    # sincostab: re-derive sin/cos(i/128) as (hi, lo) and compare bit for bit
    tab = [d(buf, SINCOSTAB + 8 * j) for j in range(4 * SINCOSTAB_N)]
    for i in range(SINCOSTAB_N):
        x = Decimal(i) / 128
        for off, f in ((0, dsin), (2, dcos)):
            v = f(x)
            hi = nearest(v)
            lo = nearest(v - Decimal(hi))
            got_hi, got_lo = tab[4 * i + off], tab[4 * i + off + 1]
            # hi is the nearest double; the table's lo parts carry ~2^-110 of the value
            assert got_hi == hi and abs(Decimal(got_lo) - (v - Decimal(hi))) <= Decimal(2) ** -105, (i, off)
    # pow log data
    ln2hi, ln2lo = d(buf, POW_LOG), d(buf, POW_LOG + 8)
    poly = [d(buf, POW_LOG + 16 + 8 * j) for j in range(7)]
    assert poly[0] == -0.5
    logtab = []
    for i in range(128):
        b = POW_LOG + 0x48 + 32 * i
        logtab.append((d(buf, b), d(buf, b + 16), d(buf, b + 24)))
    # the table's own rule: 1/c = j/N or j/N/2 with j integer, logc = round(2^43 log c) / 2^43
    for invc, logc, logctail in logtab:
        assert (invc * 256).is_integer(), invc
        cc = 1 / Decimal(invc)
        lc = cc.ln()
        assert float(round(lc * 2 ** 43)) / 2 ** 43 == logc, (invc, logc)
        assert abs(logctail - float(lc - Decimal(logc))) <= 2 ** -90, (invc, logctail)
    assert d(buf, POW_MINUS_ONE) == -1.0
    # exp data
    invln2N, shift, negln2hiN, negln2loN = (d(buf, EXP_DATA + 8 * j) for j in range(4))
    epoly = [d(buf, EXP_DATA + 32 + 8 * j) for j in range(4)]
    etab = [q(buf, EXP_DATA + 0x70 + 8 * j) for j in range(256)]
    ln2 = Decimal(2).ln()
    for i in range(128):
        e = (ln2 * i / 128).exp()
        sbits = etab[2 * i + 1] + (i << 45)
        scale = struct.unpack("<d", struct.pack("<Q", sbits))[0]
        assert abs(Decimal(scale) - e) <= Decimal(scale) * Decimal(2) ** -52, i
        tail = struct.unpack("<d", struct.pack("<Q", etab[2 * i]))[0]
        assert abs(Decimal(tail) - (e - Decimal(scale)) / Decimal(scale)) <= Decimal(2) ** -100, i

    L = []
    w = L.append
    w("// GENERATED by tools/gen_libm_consts.py -- do not edit.")
    w(f"// Source: {LIBM} (Ubuntu GLIBC 2.35-0ubuntu3.11), sha256 {SHA256}.")
    w("// Constants and tables of glibc's sincos() (s_sincos.c / s_sin.c, IBM Accurate")
    w("// Mathematical Library) and pow() (e_pow.c, ARM optimized routines; the FMA variant")
    w("// x86-64 dispatches on FMA-capable CPUs).  sin/cos(i/128) and 2^(i/128) are")
    w("// re-derived and checked by the generator; polynomial coefficients are as published.")
    w("#pragma once")
    w("#include <cstdint>")
    w("namespace glm {")
    names = dict(big="kBig", sn5="kSn5", cs6="kCs6", cs2="kCs2", taylor_max="kTaylorMax", hp0="kHp0",
                 hp1="kHp1", hpinv="kHpInv", toint="kToInt", mp1="kMp1", mp2="kMp2", pp3="kPp3", pp4="kPp4",
                 s5="kS5", s4="kS4", s2="kS2")
    for k, n in names.items():
        w(f"constexpr double {n} = {hexf(c[k])};")
    # constants the machine code subtracts (x - (-c) == x + c bit for bit)
    w(f"constexpr double kSn3 = {hexf(-c['neg_sn3'])};")
    w(f"constexpr double kCs4 = {hexf(-c['neg_cs4'])};")
    w(f"constexpr double kS3 = {hexf(-c['neg_s3'])};")
    w(f"constexpr double kS1 = {hexf(-c['neg_s1'])};")
    w(f"constexpr int kSinCosTabN = {SINCOSTAB_N};")
    w("constexpr double kSinCosTab[4 * kSinCosTabN] = {")
    for i in range(SINCOSTAB_N):
        w("    " + ", ".join(hexf(v) for v in tab[4 * i:4 * i + 4]) + ",")
    w("};")
    w(f"constexpr double kPowLn2Hi = {hexf(ln2hi)};")
    w(f"constexpr double kPowLn2Lo = {hexf(ln2lo)};")
    w("constexpr double kPowA[7] = { " + ", ".join(hexf(v) for v in poly) + " };")
    w("// {invc, logc, logctail} per subinterval")
    w("constexpr double kPowLogTab[3 * 128] = {")
    for invc, logc, logctail in logtab:
        w(f"    {hexf(invc)}, {hexf(logc)}, {hexf(logctail)},")
    w("};")
    w(f"constexpr double kExpInvLn2N = {hexf(invln2N)};")
    w(f"constexpr double kExpShift = {hexf(shift)};")
    w(f"constexpr double kExpNegLn2HiN = {hexf(negln2hiN)};")
    w(f"constexpr double kExpNegLn2LoN = {hexf(negln2loN)};")
    w("constexpr double kExpC[4] = { " + ", ".join(hexf(v) for v in epoly) + " };   // C2..C5")
    w("constexpr uint64_t kExpTab[256] = {")
    for i in range(0, 256, 4):
        w("    " + ", ".join(f"0x{v:016x}ull" for v in etab[i:i + 4]) + ",")
    w("};")
    w("}  // namespace glm")
    with open(OUT, "w") as f:
        f.write("\n".join(L) + "\n")
    print(f"wrote {OUT}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
