// The guarded multiply-by-1/res cell conversion (csrc/host_simd.cpp) against
// floor((x - min) / res) itself: random points, points on cell edges and one
// ulp either side of them, three cell sizes.  Exit status 1 on any mismatch.
#include <cmath>
#include <cstdio>
#include <random>
#include <vector>
namespace lgs { void cells_of_points(const double* xy, long long n2, double mx, double my, double res, int* out); }
int main() {
    std::mt19937_64 g(5); std::uniform_real_distribution<double> u(-30, 30);
    long long bad = 0, n = 0;
    const double res[3] = {0.05, 0.1, 0.025};
    for (int r = 0; r < 3; ++r) for (int it = 0; it < 2000; ++it) {
        std::vector<double> xy(2048);
        double mx = std::floor(u(g)) * res[r] + 0.0, my = -17.35;
        for (size_t i = 0; i < xy.size(); ++i) {
            double v = u(g);
            if (i % 3 == 0) v = mx + std::round((v - mx) / res[r]) * res[r];          // on cell edges
            if (i % 7 == 0) v = std::nextafter(v, i % 2 ? 1e9 : -1e9);
            xy[i] = v;
        }
        std::vector<int> c(xy.size());
        lgs::cells_of_points(xy.data(), xy.size(), mx, my, res[r], c.data());
        for (size_t j = 0; j < xy.size(); ++j) { ++n; if (c[j] != (int)std::floor((xy[j] - (j & 1 ? my : mx)) / res[r])) ++bad; }
    }
    printf("checked %lld, mismatches %lld\n", n, bad);
    return bad ? 1 : 0;
}
