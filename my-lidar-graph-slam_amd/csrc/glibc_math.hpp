// glibc_math.hpp -- bit-exact restatements of the glibc libm calls the
// reference's hot path makes, for the device (and the host, where
// tests/test_libm_pin.py checks them against this image's libm.so.6).
//
// The reference is built with GCC -O3 on x86-64 (no -march): every
// std::sin/std::cos pair of one argument becomes one sincos() call (DESIGN.md
// §4.2), std::pow(x, 2.0) is folded to x*x, and std::pow(x, 3.0) calls pow(),
// which glibc dispatches to its FMA variant on FMA + AVX2 CPUs.  Restated from
// the published algorithms of glibc 2.35 (constants and tables in
// libm_consts.h, generated from this image's libm by tools/gen_libm_consts.py):
//
//   gl_sincos -- sysdeps/ieee754/dbl-64/s_sincos.c with do_sin / do_cos /
//                reduce_sincos of s_sin.c (generic SSE2 build: no FMA);
//   gl_pow3   -- pow(x, 3.0) for finite x >= 0: e_pow.c's log_inline +
//                exp_inline in the operation order of __pow_fma, the FMA
//                variant's machine code (GCC contracted a*b+c at the places
//                written as fma() below).
//
// Every operation is an IEEE double add/sub/mul/fma (no division, no sqrt),
// so with -ffp-contract=off the device evaluates exactly what libm does.
// Domain: |x| < 105414350 for gl_sincos (glibc's __branred range is not
// restated; gl_sincos_ok tells), finite x >= 0 for gl_pow3.
#pragma once

#include <cmath>
#include <cstdint>
#include <cstring>

#include "libm_consts.h"

#if defined(__HIPCC__)
#define GLM_HD __host__ __device__ __forceinline__
#else
#define GLM_HD static inline
#endif

namespace glm {

GLM_HD uint64_t as_u64(double x) { return __builtin_bit_cast(uint64_t, x); }
GLM_HD double as_f64(uint64_t u) { return __builtin_bit_cast(double, u); }
GLM_HD uint32_t hi32(double x) { return (uint32_t)(as_u64(x) >> 32); }
GLM_HD uint32_t lo32(double x) { return (uint32_t)as_u64(x); }

// s_sin.c TAYLOR_SIN: a - a^3/3! + ... + (1 - a^2) da / 2
GLM_HD double taylor_sin(double xx, double a, double da)
{
    const double poly = ((((kS5 * xx + kS4) * xx + kS3) * xx + kS2) * xx) + kS1;
    const double t = ((poly * a - 0.5 * da) * xx + da);
    return a + t;
}

// s_sin.c do_cos(x, dx): cos(x + dx) by the table entry nearest |x|
GLM_HD double do_cos(double x, double dx)
{
    if (x < 0) dx = -dx;
    const double u = kBig + fabs(x);
    x = fabs(x) - (u - kBig) + dx;
    const double xx = x * x;
    const double s = x + x * xx * (kSn3 + xx * kSn5);
    const double c = xx * (kCs2 + xx * (kCs4 + xx * kCs6));
    const int k = (int)(lo32(u) << 2);
    const double sn = kSinCosTab[k], ssn = kSinCosTab[k + 1], cs = kSinCosTab[k + 2], ccs = kSinCosTab[k + 3];
    const double cor = (ccs - s * ssn - cs * c) - sn * s;
    return cs + cor;
}

// s_sin.c do_sin(x, dx): sin(x + dx)
GLM_HD double do_sin(double x, double dx)
{
    const double xold = x;
    if (fabs(x) < kTaylorMax) return taylor_sin(x * x, x, dx);
    if (x <= 0) dx = -dx;
    const double u = kBig + fabs(x);
    x = fabs(x) - (u - kBig);
    const double xx = x * x;
    const double s = x + (dx + x * xx * (kSn3 + xx * kSn5));
    const double c = x * dx + xx * (kCs2 + xx * (kCs4 + xx * kCs6));
    const int k = (int)(lo32(u) << 2);
    const double sn = kSinCosTab[k], ssn = kSinCosTab[k + 1], cs = kSinCosTab[k + 2], ccs = kSinCosTab[k + 3];
    const double cor = (ssn + s * ccs - sn * c) + cs * s;
    return copysign(sn + cor, xold);
}

// s_sin.c reduce_sincos: x = n pi/2 + (a + da), Cody-Waite with 3 + 1 parts
GLM_HD int reduce_sincos(double x, double& a, double& da)
{
    const double t = (x * kHpInv + kToInt);
    const double xn = t - kToInt;
    const int n = (int)(lo32(t) & 3u);
    const double y = (x - xn * kMp1) - xn * kMp2;
    double t1 = xn * kPp3;
    const double t2 = y - t1;
    double db = (y - t2) - t1;
    t1 = xn * kPp4;
    const double b = t2 - t1;
    db += (t2 - b) - t1;
    a = b;
    da = db;
    return n;
}

GLM_HD bool gl_sincos_ok(double x) { return (hi32(x) & 0x7fffffffu) < 0x419921FBu; }

// s_sincos.c __sincos for |x| < 105414350 (else NaN: __branred not restated)
GLM_HD void gl_sincos(double x, double* sinx, double* cosx)
{
    const uint32_t k = hi32(x) & 0x7fffffffu;
    if (k < 0x400368fdu) {
        if (k < 0x3e400000u) {          // |x| < 2^-27
            *sinx = x;
            *cosx = 1.0;
            return;
        }
        if (k < 0x3feb6000u) {          // |x| < 0.855469
            *sinx = do_sin(x, 0);
            *cosx = do_cos(x, 0);
            return;
        }
        const double y = kHp0 - fabs(x);   // |x| < 2.426265
        const double a = y + kHp1;
        const double da = (y - a) + kHp1;
        *sinx = copysign(do_cos(a, da), x);
        *cosx = do_sin(a, da);
        return;
    }
    if (k < 0x419921FBu) {
        double a, da;
        const int n = reduce_sincos(x, a, da);
        if (n == 1 || n == 2) {
            a = -a;
            da = -da;
        }
        double* s = sinx;
        double* c = cosx;
        if (n & 1) {
            s = cosx;
            c = sinx;
        }
        *s = do_sin(a, da);
        const double cr = do_cos(a, da);
        *c = (n & 2) ? -cr : cr;
        return;
    }
    *sinx = *cosx = __builtin_nan("");
}

// e_pow.c pow(x, 3.0) for finite x >= 0, in __pow_fma's operation order
GLM_HD double gl_pow3(double x)
{
    const uint64_t ix = as_u64(x);
    if (ix == 0) return 0.0;            // pow(+0, 3) = +0 (zeroinfnan path: x * x)
    // log_inline(ix) -> hi + lo
    constexpr uint64_t OFF = 0x3fe6955500000000ull;
    const uint64_t tmp = ix - OFF;
    const int i = (int)((tmp >> 45) % 128);
    const int k = (int)((int64_t)tmp >> 52);
    const uint64_t iz = ix - (tmp & (0xfffull << 52));
    const double z = as_f64(iz);
    const double kd = (double)k;
    const double invc = kPowLogTab[3 * i], logc = kPowLogTab[3 * i + 1], logctail = kPowLogTab[3 * i + 2];
    const double r = fma(z, invc, -1.0);
    const double t1 = fma(kd, kPowLn2Hi, logc);
    const double t2 = t1 + r;
    const double lo1 = fma(kd, kPowLn2Lo, logctail);
    const double lo2 = t1 - t2 + r;
    const double ar = kPowA[0] * r;
    const double ar2 = r * ar;
    const double ar3 = r * ar2;
    const double hi0 = t2 + ar2;
    const double lo3 = fma(ar, r, -ar2);
    const double lo4 = t2 - hi0 + ar2;
    const double pA = fma(r, kPowA[2], kPowA[1]);
    const double pB = fma(r, kPowA[4], kPowA[3]);
    const double pC = fma(r, kPowA[6], kPowA[5]);
    const double p = fma(ar2, fma(pC, ar2, pB), pA);
    const double lo = fma(ar3, p, ((lo1 + lo2) + lo3) + lo4);
    const double lhi = hi0 + lo;
    const double ltail = hi0 - lhi + lo;
    // y * log(x) as ehi + elo
    const double y = 3.0;
    const double ehi = y * lhi;
    const double elo = fma(y, ltail, fma(lhi, y, -ehi));
    // exp_inline(ehi, elo, 0)
    const uint32_t abstop = (uint32_t)(as_u64(ehi) >> 52) & 0x7ffu;
    if (abstop - 0x3c9u >= 0x3fu) {
        // |ehi| < 2^-54: 1 + ehi (larger |ehi| cannot occur for x in a double's range with y = 3)
        return 1.0 + ehi;
    }
    const double kd2 = fma(ehi, kExpInvLn2N, kExpShift);
    const uint64_t ki = as_u64(kd2);
    const double kdd = kd2 - kExpShift;
    double rr = fma(kdd, kExpNegLn2LoN, fma(kdd, kExpNegLn2HiN, ehi));
    rr = rr + elo;
    const uint64_t idx = 2 * (ki % 128);
    const uint64_t top = ki << 45;
    const double tail = as_f64(kExpTab[idx]);
    const uint64_t sbits = kExpTab[idx + 1] + top;
    const double r2 = rr * rr;
    const double q1 = fma(rr, kExpC[1], kExpC[0]);
    const double q2 = fma(rr, kExpC[3], kExpC[2]);
    const double t = fma(q2, r2 * r2, fma(q1, r2, tail + rr));
    const double scale = as_f64(sbits);
    return fma(t, scale, scale);
}

}  // namespace glm
