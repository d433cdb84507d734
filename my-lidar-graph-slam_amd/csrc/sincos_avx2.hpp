// sincos_avx2.hpp -- glibc's sincos() four arguments at a time on the host
// (AVX2, no FMA), bit for bit: the restatement of glibc_math.hpp gl_sincos
// (s_sincos.c / s_sin.c of glibc 2.35, constants from libm_consts.h) with its
// branches evaluated for every lane and blended.  The hit points of a map
// update take one sincos per beam (ComputeBoundingBoxAndScanPoints,
// C/mapping/grid_map_builder.cpp:335-380): ~9 us for 1081 beams through libm,
// on the config-4 step's host path between the match's result and the
// append's first kernel.  Pinned against libm by tests/test_libm_pin.py.
//
// Every operation is an IEEE double add/sub/mul in the order the scalar code
// (and libm) performs it; the file must be compiled without FP contraction
// (-ffp-contract=off), and the target attribute enables AVX2 only (no FMA).
#pragma once

#include <cstdint>
#include <immintrin.h>

#include "libm_consts.h"

namespace glm {
namespace avx2 {

typedef __m256d V;

#define GLM_AVX2 __attribute__((target("avx2"), always_inline)) static inline

GLM_AVX2 V vset(double x) { return _mm256_set1_pd(x); }
GLM_AVX2 V vabs(V x) { return _mm256_andnot_pd(_mm256_set1_pd(-0.0), x); }
// copysign(mag, sgn)
GLM_AVX2 V vcopysign(V mag, V sgn)
{
    const V m = _mm256_set1_pd(-0.0);
    return _mm256_or_pd(_mm256_andnot_pd(m, mag), _mm256_and_pd(m, sgn));
}
GLM_AVX2 V vneg(V x) { return _mm256_xor_pd(x, _mm256_set1_pd(-0.0)); }
// the low / high 32 bits of each lane's bit pattern
GLM_AVX2 __m128i lo32(V x)
{
    const __m256i p = _mm256_permutevar8x32_epi32(_mm256_castpd_si256(x), _mm256_setr_epi32(0, 2, 4, 6, 1, 3, 5, 7));
    return _mm256_castsi256_si128(p);
}
GLM_AVX2 __m128i hi32(V x)
{
    const __m256i p = _mm256_permutevar8x32_epi32(_mm256_castpd_si256(x), _mm256_setr_epi32(1, 3, 5, 7, 0, 2, 4, 6));
    return _mm256_castsi256_si128(p);
}
// a 4 x 32-bit lane mask widened to 4 x 64 bits
GLM_AVX2 V wide(__m128i m) { return _mm256_castsi256_pd(_mm256_cvtepi32_epi64(m)); }
GLM_AVX2 V sel(V m, V a, V b) { return _mm256_blendv_pd(b, a, m); }   // m ? a : b

// TAYLOR_SIN: a + (((poly a - 0.5 da) xx) + da)
GLM_AVX2 V taylor_sin(V xx, V a, V da)
{
    V poly = _mm256_add_pd(_mm256_mul_pd(vset(kS5), xx), vset(kS4));
    poly = _mm256_add_pd(_mm256_mul_pd(poly, xx), vset(kS3));
    poly = _mm256_add_pd(_mm256_mul_pd(poly, xx), vset(kS2));
    poly = _mm256_add_pd(_mm256_mul_pd(poly, xx), vset(kS1));
    const V t = _mm256_add_pd(_mm256_mul_pd(_mm256_sub_pd(_mm256_mul_pd(poly, a), _mm256_mul_pd(vset(0.5), da)), xx), da);
    return _mm256_add_pd(a, t);
}

// the table entry nearest |x|: u = big + |x|, k = 4 * (low word of u); the
// entry's 4 doubles (sn, ssn, cs, ccs) are one 32-byte load per lane,
// transposed (4 x 4) -- gathers are slow on the host's cores.  do_sin and
// do_cos of one argument use the same entry.
struct TabEntry {
    V u, sn, ssn, cs, ccs;
};
GLM_AVX2 TabEntry table(V ax)
{
    TabEntry e;
    e.u = _mm256_add_pd(vset(kBig), ax);
    alignas(16) int k[4];
    _mm_store_si128((__m128i*)k, _mm_slli_epi32(lo32(e.u), 2));
    const V r0 = _mm256_loadu_pd(kSinCosTab + k[0]), r1 = _mm256_loadu_pd(kSinCosTab + k[1]);
    const V r2 = _mm256_loadu_pd(kSinCosTab + k[2]), r3 = _mm256_loadu_pd(kSinCosTab + k[3]);
    const V t0 = _mm256_unpacklo_pd(r0, r1), t1 = _mm256_unpackhi_pd(r0, r1);   // (sn0 sn1 cs0 cs1), (ssn.. ccs..)
    const V t2 = _mm256_unpacklo_pd(r2, r3), t3 = _mm256_unpackhi_pd(r2, r3);
    e.sn = _mm256_permute2f128_pd(t0, t2, 0x20);
    e.cs = _mm256_permute2f128_pd(t0, t2, 0x31);
    e.ssn = _mm256_permute2f128_pd(t1, t3, 0x20);
    e.ccs = _mm256_permute2f128_pd(t1, t3, 0x31);
    return e;
}

// do_cos(x, dx)
GLM_AVX2 V do_cos(V x, V dx, const TabEntry& e)
{
    dx = sel(_mm256_cmp_pd(x, _mm256_setzero_pd(), _CMP_LT_OQ), vneg(dx), dx);
    const V ax = vabs(x);
    const V y = _mm256_add_pd(_mm256_sub_pd(ax, _mm256_sub_pd(e.u, vset(kBig))), dx);
    const V xx = _mm256_mul_pd(y, y);
    const V s = _mm256_add_pd(y, _mm256_mul_pd(_mm256_mul_pd(y, xx),
                                               _mm256_add_pd(vset(kSn3), _mm256_mul_pd(xx, vset(kSn5)))));
    const V c = _mm256_mul_pd(
        xx, _mm256_add_pd(vset(kCs2), _mm256_mul_pd(xx, _mm256_add_pd(vset(kCs4), _mm256_mul_pd(xx, vset(kCs6))))));
    const V cor = _mm256_sub_pd(_mm256_sub_pd(_mm256_sub_pd(e.ccs, _mm256_mul_pd(s, e.ssn)), _mm256_mul_pd(e.cs, c)),
                                _mm256_mul_pd(e.sn, s));
    return _mm256_add_pd(e.cs, cor);
}

// do_sin(x, dx)
GLM_AVX2 V do_sin(V x, V dx, const TabEntry& e)
{
    const V ax = vabs(x);
    const V tay = taylor_sin(_mm256_mul_pd(x, x), x, dx);
    const V dxs = sel(_mm256_cmp_pd(x, _mm256_setzero_pd(), _CMP_LE_OQ), vneg(dx), dx);
    const V y = _mm256_sub_pd(ax, _mm256_sub_pd(e.u, vset(kBig)));
    const V xx = _mm256_mul_pd(y, y);
    const V s = _mm256_add_pd(
        y, _mm256_add_pd(dxs, _mm256_mul_pd(_mm256_mul_pd(y, xx), _mm256_add_pd(vset(kSn3), _mm256_mul_pd(xx, vset(kSn5))))));
    const V c = _mm256_add_pd(
        _mm256_mul_pd(y, dxs),
        _mm256_mul_pd(xx, _mm256_add_pd(vset(kCs2),
                                        _mm256_mul_pd(xx, _mm256_add_pd(vset(kCs4), _mm256_mul_pd(xx, vset(kCs6)))))));
    const V cor = _mm256_add_pd(_mm256_sub_pd(_mm256_add_pd(e.ssn, _mm256_mul_pd(s, e.ccs)), _mm256_mul_pd(e.sn, c)),
                                _mm256_mul_pd(e.cs, s));
    const V tab = vcopysign(_mm256_add_pd(e.sn, cor), x);
    return sel(_mm256_cmp_pd(ax, vset(kTaylorMax), _CMP_LT_OQ), tay, tab);
}

// Four sincos.  Returns a 4-bit mask of the lanes outside the restated
// domain (|x| >= 105414350, NaN, inf): their outputs are left undefined and
// the caller takes libm for them.
__attribute__((target("avx2"))) static inline int sincos4(const double* xp, double* sp, double* cp)
{
    const V x = _mm256_loadu_pd(xp);
    const __m128i k = _mm_and_si128(hi32(x), _mm_set1_epi32(0x7fffffff));
    const __m128i tiny = _mm_cmplt_epi32(k, _mm_set1_epi32(0x3e400000));     // |x| < 2^-27
    const __m128i small = _mm_cmplt_epi32(k, _mm_set1_epi32(0x3feb6000));    // |x| < 0.855469
    const __m128i mid = _mm_cmplt_epi32(k, _mm_set1_epi32(0x400368fd));      // |x| < 2.426265
    const __m128i dom = _mm_cmplt_epi32(k, _mm_set1_epi32(0x419921FB));      // |x| < 105414350
    const V vsmall = wide(small), vmid = wide(mid), vdom = wide(dom);
    // the pi/2 - |x| range
    const V yc = _mm256_sub_pd(vset(kHp0), vabs(x));
    const V ac = _mm256_add_pd(yc, vset(kHp1));
    const V dac = _mm256_add_pd(_mm256_sub_pd(yc, ac), vset(kHp1));
    // Cody-Waite reduction x = n pi/2 + (a + da)
    const V xr = sel(vdom, x, _mm256_setzero_pd());
    const V t = _mm256_add_pd(_mm256_mul_pd(xr, vset(kHpInv)), vset(kToInt));
    const V xn = _mm256_sub_pd(t, vset(kToInt));
    const __m128i n = _mm_and_si128(lo32(t), _mm_set1_epi32(3));
    const V yr = _mm256_sub_pd(_mm256_sub_pd(xr, _mm256_mul_pd(xn, vset(kMp1))), _mm256_mul_pd(xn, vset(kMp2)));
    V t1 = _mm256_mul_pd(xn, vset(kPp3));
    const V t2 = _mm256_sub_pd(yr, t1);
    V db = _mm256_sub_pd(_mm256_sub_pd(yr, t2), t1);
    t1 = _mm256_mul_pd(xn, vset(kPp4));
    const V b = _mm256_sub_pd(t2, t1);
    db = _mm256_add_pd(db, _mm256_sub_pd(_mm256_sub_pd(t2, b), t1));
    // n == 1 or 2: the argument negated
    const V n12 = wide(_mm_or_si128(_mm_cmpeq_epi32(n, _mm_set1_epi32(1)), _mm_cmpeq_epi32(n, _mm_set1_epi32(2))));
    const V ar = sel(n12, vneg(b), b), dar = sel(n12, vneg(db), db);
    // one do_sin / do_cos evaluation per lane on its range's argument
    const V a = sel(vsmall, x, sel(vmid, ac, ar));
    const V da = sel(vsmall, _mm256_setzero_pd(), sel(vmid, dac, dar));
    const TabEntry e = table(vabs(a));
    const V ds = do_sin(a, da, e), dc = do_cos(a, da, e);
    // reduced: sin, cos = (do_sin, +-do_cos) or swapped (n odd); cos-result negated for n & 2
    const V odd = wide(_mm_cmpeq_epi32(_mm_and_si128(n, _mm_set1_epi32(1)), _mm_set1_epi32(1)));
    const V two = wide(_mm_cmpeq_epi32(_mm_and_si128(n, _mm_set1_epi32(2)), _mm_set1_epi32(2)));
    const V dcn = sel(two, vneg(dc), dc);
    const V s_red = sel(odd, dcn, ds), c_red = sel(odd, ds, dcn);
    // pi/2 - |x| range: sin = copysign(do_cos, x), cos = do_sin
    const V s_mid = vcopysign(dc, x), c_mid = ds;
    V s = sel(vsmall, ds, sel(vmid, s_mid, s_red));
    V c = sel(vsmall, dc, sel(vmid, c_mid, c_red));
    const V vtiny = wide(tiny);
    s = sel(vtiny, x, s);
    c = sel(vtiny, vset(1.0), c);
    _mm256_storeu_pd(sp, s);
    _mm256_storeu_pd(cp, c);
    return (~_mm256_movemask_pd(vdom)) & 0xF;
}

#undef GLM_AVX2

}  // namespace avx2
}  // namespace glm
