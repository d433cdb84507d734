// Host harness pinning csrc/glibc_math.hpp (the device's restatement of
// glibc's sincos and pow(x, 3.0)) against this image's libm.so.6: the same
// header compiled for the host with -ffp-contract=off, compared bit for bit
// with the library calls on seeded random inputs (tests/test_libm_pin.py).
#include <cmath>
#include <cstdint>
#include <cstring>
#include <random>

#include "glibc_math.hpp"
#include "sincos_avx2.hpp"

namespace {
uint64_t bits(double x)
{
    uint64_t u;
    std::memcpy(&u, &x, 8);
    return u;
}

// libm's own entry points, called through volatile pointers so that GCC
// cannot constant-fold, fuse or replace them
extern "C" void sincos(double, double*, double*);
void (*volatile libm_sincos)(double, double*, double*) = sincos;
double (*volatile libm_pow)(double, double) = pow;
}  // namespace

extern "C" {

// n inputs: uniform in [lo, hi] (mode 0), or lo + k * 2^-e for a random
// exponent e in [30, 52] (mode 1: the fixed-point hit coordinates of the
// matchers).  Returns the number of mismatching inputs; the first one is
// stored in *bad.
long pin_sincos(uint64_t seed, long n, double lo, double hi, int mode, double* bad)
{
    std::mt19937_64 rng(seed);
    std::uniform_real_distribution<double> U(lo, hi);
    long mism = 0;
    for (long j = 0; j < n; ++j) {
        double x = U(rng);
        if (mode == 1) {
            const int e = 30 + (int)(rng() % 23);
            x = std::ldexp(std::nearbyint(std::ldexp(x, e)), -e);
        }
        double s0, c0, s1, c1;
        libm_sincos(x, &s0, &c0);
        glm::gl_sincos(x, &s1, &c1);
        if (bits(s0) != bits(s1) || bits(c0) != bits(c1)) {
            if (mism == 0 && bad) *bad = x;
            ++mism;
        }
    }
    return mism;
}

// The host's four-lane restatement (sincos_avx2.hpp, host_simd.cpp
// sincos_batch) on the same inputs, four at a time; lanes it reports outside
// its domain must be exactly those gl_sincos_ok rejects.
long pin_sincos_avx2(uint64_t seed, long n, double lo, double hi, int mode, double* bad)
{
    std::mt19937_64 rng(seed);
    std::uniform_real_distribution<double> U(lo, hi);
    long mism = 0;
    for (long j = 0; j + 4 <= n; j += 4) {
        double x[4], s1[4], c1[4];
        for (int l = 0; l < 4; ++l) {
            x[l] = U(rng);
            if (mode == 1) {
                const int e = 30 + (int)(rng() % 23);
                x[l] = std::ldexp(std::nearbyint(std::ldexp(x[l], e)), -e);
            }
        }
        const int out = glm::avx2::sincos4(x, s1, c1);
        for (int l = 0; l < 4; ++l) {
            double s0, c0;
            libm_sincos(x[l], &s0, &c0);
            const bool dom = glm::gl_sincos_ok(x[l]);
            const bool ok = (out >> l & 1) ? !dom : (dom && bits(s0) == bits(s1[l]) && bits(c0) == bits(c1[l]));
            if (!ok) {
                if (mism == 0 && bad) *bad = x[l];
                ++mism;
            }
        }
    }
    return mism;
}

// pow(x, 3.0) for the bicubic kernel's arguments |t| in [0, 2]: mode 0
// uniform in [lo, hi]; mode 1 the differences 1 + f, f, 1 - f, 2 - f of a
// fractional part f = k * 2^-e (e in [36, 52]) as ComputeSmoothedValue forms them.
long pin_pow3(uint64_t seed, long n, double lo, double hi, int mode, double* bad)
{
    std::mt19937_64 rng(seed);
    std::uniform_real_distribution<double> U(lo, hi);
    long mism = 0;
    for (long j = 0; j < n; ++j) {
        double x = U(rng);
        if (mode == 1) {
            const int e = 36 + (int)(rng() % 17);
            const double base = (double)(200 + rng() % 800);
            const double v = base + std::ldexp((double)(rng() >> (64 - e)), -e);
            const double fl = std::floor(v);
            const double cand[4] = { 1.0 + v - fl, v - fl, fl + 1.0 - v, fl + 2.0 - v };
            x = std::fabs(cand[rng() & 3]);
        }
        const double a = libm_pow(x, 3.0), b = glm::gl_pow3(x);
        if (bits(a) != bits(b)) {
            if (mism == 0 && bad) *bad = x;
            ++mism;
        }
    }
    return mism;
}

void glm_sincos(double x, double* s, double* c) { glm::gl_sincos(x, s, c); }
double glm_pow3(double x) { return glm::gl_pow3(x); }
}
