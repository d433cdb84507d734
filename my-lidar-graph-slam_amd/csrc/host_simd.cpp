// host_simd.cpp -- vectorised host helpers of the map path.
//
// WorldCoordinateToGridCellIndex (C/mapping/grid_map_builder.cpp via
// H/grid_map/grid_map.hpp:779-790) is floor((x - min) / res) per coordinate:
// a config-4 step converts ~1000 hit points for the latest map and again for
// the local map (the shift check, k_raycast.hip latest_step), ~4000 fp64
// divisions that took ~10 us scalar.  The AVX2 path multiplies by 1 / res
// four lanes at a time and divides only the lanes whose product is within a
// guard band of a cell edge, where the two could floor differently.
#include <cmath>
#include <immintrin.h>

#include "sincos_avx2.hpp"

namespace lgs {
namespace {
// floor(a / res) through a * (1 / res): the product is within 3 * 2^-53
// relative of the quotient (< 4e-10 for |a / res| < 2^20 cells), and so is
// the correctly rounded division, so unless the product lies within kGuard of
// an integer both floors agree; such lanes take the division itself
constexpr double kGuard = 1e-6;

inline int cell_div(double v, double mn, double res) { return (int)std::floor((v - mn) / res); }

__attribute__((target("avx2"))) void cells_avx2(const double* xy, long long n2, double mx, double my, double res,
                                                int* out)
{
    const __m256d mn = _mm256_setr_pd(mx, my, mx, my), inv = _mm256_set1_pd(1.0 / res);
    const __m256d lo = _mm256_set1_pd(kGuard), hi = _mm256_set1_pd(1.0 - kGuard);
    const __m256d lim = _mm256_set1_pd(1048576.0);
    long long j = 0;
    for (; j + 4 <= n2; j += 4) {
        const __m256d q = _mm256_mul_pd(_mm256_sub_pd(_mm256_loadu_pd(xy + j), mn), inv);
        const __m256d f = _mm256_floor_pd(q);
        const __m256d d = _mm256_sub_pd(q, f);
        const __m256d ok = _mm256_and_pd(_mm256_and_pd(_mm256_cmp_pd(d, lo, _CMP_GT_OQ), _mm256_cmp_pd(d, hi, _CMP_LT_OQ)),
                                         _mm256_cmp_pd(_mm256_andnot_pd(_mm256_set1_pd(-0.0), q), lim, _CMP_LT_OQ));
        if (_mm256_movemask_pd(ok) == 0xF) {
            _mm_storeu_si128((__m128i*)(out + j), _mm256_cvttpd_epi32(f));
        } else {
            for (long long k = j; k < j + 4; ++k) out[k] = cell_div(xy[k], (k & 1) ? my : mx, res);
        }
    }
    for (; j < n2; ++j) out[j] = cell_div(xy[j], (j & 1) ? my : mx, res);
}
}  // namespace

// out[2k], out[2k+1] = the cell of point (xy[2k], xy[2k+1]) in a map with
// origin (mx, my) and cell size res: floor((x - mx) / res) exactly
void cells_of_points(const double* xy, long long n2, double mx, double my, double res, int* out)
{
    static const bool avx2 = __builtin_cpu_supports("avx2");
    if (avx2) {
        cells_avx2(xy, n2, mx, my, res, out);
        return;
    }
    for (long long j = 0; j < n2; ++j) out[j] = cell_div(xy[j], (j & 1) ? my : mx, res);
}

// s[j], c[j] = glibc sincos(x[j]) bit for bit: four at a time through the
// AVX2 restatement (sincos_avx2.hpp), libm for lanes outside its domain and
// the tail
void sincos_batch(const double* x, long long n, double* s, double* c)
{
    static const bool avx2 = __builtin_cpu_supports("avx2");
    long long j = 0;
    if (avx2) {
        for (; j + 4 <= n; j += 4) {
            const int bad = glm::avx2::sincos4(x + j, s + j, c + j);
            if (bad)
                for (int l = 0; l < 4; ++l)
                    if (bad >> l & 1) ::sincos(x[j + l], s + j + l, c + j + l);
        }
    }
    for (; j < n; ++j) ::sincos(x[j], s + j, c + j);
}
}  // namespace lgs
