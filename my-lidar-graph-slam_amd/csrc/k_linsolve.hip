// k_linsolve.hip -- K4: Gauss-Newton scan matcher (ScanMatcherLinearSolver) on MI355X.
//
// Restates ScanMatcherLinearSolver::OptimizePose / OptimizeStep
// (C/mapping/scan_matcher_linear_solver.cpp:38-148) with CostSquareError
// (C/mapping/cost_function_square_error.cpp: Cost :21-58, ComputeCovariance
// :112-135, ComputeMapGradient :172-229, ComputeSmoothedValue :276-346).
//
// One workgroup runs one whole refine (all iterations) without returning to
// the host: per iteration every thread takes beams i = tid, tid + 512, ...,
// evaluates the bicubic smoothed value and its central-difference map
// gradient (5 x 16 gathers per beam, all independent), and accumulates
// b = sum res*g and H = sum g*g^T in registers; wave64 shuffle butterflies
// plus one LDS pass reduce the 9 sums; lane 0 solves the regularised 3x3
// system with the column-pivoting Householder QR Eigen's colPivHouseholderQr
// uses (restated, Eigen is not vendored), updates the pose, and the cost at
// the new pose is reduced the same way for the convergence test.  A batch
// launches one workgroup per scan.
//
// Numerics: the reference's own result moves by up to ~1e-5
// under a 1-ulp change of its input pose (ComputeSmoothedValue truncates
// coordinates that sit on integers +- rounding), so parity with the oracle is
// judged within the north-star tolerance, not bitwise.  Device sin/cos/pow
// follow ocml; pow(x, 2.0) is the exact x*x GCC folds it to, pow(x, 3.0) is
// the correctly rounded cube (glibc's pow agrees with it in 99.9% of inputs).
#include "lgs_internal.hpp"

#include <cfloat>
#include <climits>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

using namespace lgs;

namespace {

constexpr int kLsThreads = 512;

struct LsPlan {
    double min_x, min_y, res;
    int W, H, N;
    int max_iter;
    double conv;
    double step_min, step_max;    // OptimizeStep's beam filter (open interval)
    double cost_min, cost_max;    // CostSquareError's beam filter
    double reg_t, reg_r;
};

struct LsRecord {
    double pose[3];     // best sensor pose
    double cost;
    double grad[3];     // CostSquareError::ComputeGradient at the best pose
    int iterations;
    int pad;
};

// x86-64 cvttsd2si semantics of static_cast<int>(double) (the reference's
// host): out-of-range and NaN give INT_MIN; the GPU conversion would saturate.
__device__ __forceinline__ int host_trunc(double x)
{
    return (x > -2147483649.0 && x < 2147483648.0) ? (int)x : INT_MIN;
}

// pow(a, 3.0), correctly rounded: a^3 = c + ce + pe*a exactly up to 2^-106 relative
__device__ __forceinline__ double cube(double a)
{
    const double p = a * a;
    const double pe = fma(a, a, -p);
    const double c = p * a;
    const double ce = fma(p, a, -c);
    return c + (ce + pe * a);
}

// bicubic kernel h(t) (:281-295); pow(at, 2.0) is at*at after GCC folding
__device__ __forceinline__ double bicubic_h(double t)
{
    const double at = fabs(t);
    if (at <= 1.0) {
        const double at3 = cube(at);
        const double at2 = at * at;
        return (at3 - 2.0 * at2 + 1.0);
    } else if (at <= 2.0) {
        const double at3 = cube(at);
        const double at2 = at * at;
        return (-at3 + 5.0 * at2 - 8.0 * at + 4.0);
    }
    return 0.0;
}

// One axis of ComputeSmoothedValue (:276-346) for coordinate v: the four
// sample indices clamp(static_cast<int>(v_i), 0, n-1) of f (:298-310,
// truncation) and the four kernel weights h(v_1..v_4).  The x axis of
// (fx, fy +- d) and the y axis of (fx +- d, fy) are the axes of (fx, fy): the
// reference's "+ 0.0" / "- 0.0" leave every derived quantity unchanged
// (v + 0.0 differs from v only for v = -0.0, which yields the same floor
// differences, indices and weights), so five smoothed values share six axes.
struct Axis {
    int idx[4];
    double w[4];
};

__device__ __forceinline__ int clampi(int v, int lo, int hi) { return v < lo ? lo : (hi < v ? hi : v); }

__device__ __forceinline__ Axis make_axis(double v, int n)
{
    const double fl = floor(v);
    const double v1 = 1.0 + v - fl;
    const double v2 = v - fl;
    const double v3 = fl + 1.0 - v;
    const double v4 = fl + 2.0 - v;
    Axis a;
    a.idx[0] = clampi(host_trunc(v - v1), 0, n - 1);
    a.idx[1] = clampi(host_trunc(v - v2), 0, n - 1);
    a.idx[2] = clampi(host_trunc(v + v3), 0, n - 1);
    a.idx[3] = clampi(host_trunc(v + v4), 0, n - 1);
    a.w[0] = bicubic_h(v1);
    a.w[1] = bicubic_h(v2);
    a.w[2] = bicubic_h(v3);
    a.w[3] = bicubic_h(v4);
    return a;
}

// vecX^T * M * vecY with M(i, j) = f(xs_i, ys_j), evaluated as
// r_j = sum_i vx_i M_ij, then sum_j r_j vy_j (the oracle's order; Eigen's
// own order is not pinned), clamped to [0, 1] (:345)
__device__ __forceinline__ double smoothed(const double* __restrict__ g, int W, const Axis& ax,
                                           const Axis& ay)
{
    double m[4][4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const double* row = g + (size_t)ay.idx[j] * W;
#pragma unroll
        for (int i = 0; i < 4; ++i) m[j][i] = row[ax.idx[i]];
    }
    double s = 0.0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        double acc = ax.w[0] * m[j][0];
#pragma unroll
        for (int i = 1; i < 4; ++i) acc = acc + ax.w[i] * m[j][i];
        s = (j == 0) ? acc * ay.w[0] : s + acc * ay.w[j];
    }
    return s < 0.0 ? 0.0 : (1.0 < s ? 1.0 : s);
}

// Per beam at one sensor pose: residual e = 1 - S(hit point) and the map
// gradient w.r.t. the pose (ComputeMapGradient :172-229: central differences
// of +-0.05 cells, / (0.1 res), dtheta = -r sin gx + r cos gy).
constexpr double kDeltaIdx = 0.1;             // ComputeMapGradient's +- 0.05 cells
constexpr double kHalfDelta = kDeltaIdx / 2.0;

// hit point of a beam in (fractional) cell coordinates
__device__ __forceinline__ void beam_cell(const LsPlan& p, const double pose[3], double r, double a, double& sn,
                                          double& cs, double& fx, double& fy)
{
    sincos(pose[2] + a, &sn, &cs);
    const double hx = pose[0] + r * cs;
    const double hy = pose[1] + r * sn;
    fx = (hx - p.min_x) / p.res;
    fy = (hy - p.min_y) / p.res;
}

// residual and pose gradient from the five smoothed values
__device__ __forceinline__ void beam_finish(const LsPlan& p, double r, double sn, double cs, double s0, double sxp,
                                            double sxm, double syp, double sym, double& e, double gv[3])
{
    const double deltaDist = p.res * kDeltaIdx;
    const double gx = (sxp - sxm) / deltaDist;
    const double gy = (syp - sym) / deltaDist;
    e = 1.0 - s0;
    gv[0] = gx;
    gv[1] = gy;
    gv[2] = -r * sn * gx + r * cs * gy;
}

__device__ __forceinline__ void beam_terms(const LsPlan& p, const double* __restrict__ g,
                                           const double pose[3], double r, double a, double& e,
                                           double gv[3])
{
    double sn, cs, fx, fy;
    beam_cell(p, pose, r, a, sn, cs, fx, fy);
    const double d = kHalfDelta;
    const Axis x0 = make_axis(fx, p.W), xp = make_axis(fx + d, p.W), xm = make_axis(fx - d, p.W);
    const Axis y0 = make_axis(fy, p.H), yp = make_axis(fy + d, p.H), ym = make_axis(fy - d, p.H);
    const double s0 = smoothed(g, p.W, x0, y0);
    const double sxp = smoothed(g, p.W, xp, y0);
    const double sxm = smoothed(g, p.W, xm, y0);
    const double syp = smoothed(g, p.W, x0, yp);
    const double sym = smoothed(g, p.W, x0, ym);
    beam_finish(p, r, sn, cs, s0, sxp, sxm, syp, sym, e, gv);
}

// sum over the workgroup of NV values per thread (wave64 butterfly + LDS);
// every thread gets the totals
template <int NV>
__device__ void wg_sum(double (&v)[NV], double* red)
{
#pragma unroll
    for (int k = 0; k < NV; ++k)
        for (int off = 32; off > 0; off >>= 1) v[k] += __shfl_xor(v[k], off, 64);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    constexpr int nw = kLsThreads / 64;
    __syncthreads();
    if (lane == 0)
#pragma unroll
        for (int k = 0; k < NV; ++k) red[k * nw + wid] = v[k];
    __syncthreads();
#pragma unroll
    for (int k = 0; k < NV; ++k) {
        double s = red[k * nw];
        for (int w = 1; w < nw; ++w) s += red[k * nw + w];
        v[k] = s;
    }
}

// Eigen ColPivHouseholderQR<Matrix3d>::compute + solve (published algorithm,
// Eigen >= 3.3), one thread.  Every loop is unrolled and every data-dependent
// index (pivot column, permutation) is resolved with compile-time-indexed
// selects, so the 3x3 problem lives in registers (no scratch).
template <class T>
__device__ __forceinline__ void cswap(bool c, T& a, T& b)
{
    const T ta = a, tb = b;
    a = c ? tb : ta;
    b = c ? ta : tb;
}

__device__ void solve3_colpiv_qr(const double Hin[9], const double bin[3], double xout[3])
{
    constexpr int N = 3;
    double A[N][N];
#pragma unroll
    for (int i = 0; i < N; ++i)
#pragma unroll
        for (int j = 0; j < N; ++j) A[i][j] = Hin[3 * i + j];
    double hc[N], normU[N], normD[N];
    int transp[N];
    const double eps = DBL_EPSILON;
#pragma unroll
    for (int k = 0; k < N; ++k) {
        double s = 0.0;
#pragma unroll
        for (int i = 0; i < N; ++i) s += A[i][k] * A[i][k];
        normD[k] = sqrt(s);
        normU[k] = normD[k];
    }
    double maxn = normU[0];
#pragma unroll
    for (int k = 1; k < N; ++k)
        if (normU[k] > maxn) maxn = normU[k];
    const double thrHelper = (maxn * eps) * (maxn * eps) / (double)N;
    const double downdateThr = sqrt(eps);
    int nonzero = N;
#pragma unroll
    for (int k = 0; k < N; ++k) {
        int big = k;
        double bigv = normU[k];
#pragma unroll
        for (int j = k + 1; j < N; ++j)
            if (normU[j] > bigv) {
                bigv = normU[j];
                big = j;
            }
        if (nonzero == N && bigv * bigv < thrHelper * (double)(N - k)) nonzero = k;
        transp[k] = big;
#pragma unroll
        for (int j = k + 1; j < N; ++j) {
            const bool sw = (j == big);
#pragma unroll
            for (int i = 0; i < N; ++i) cswap(sw, A[i][k], A[i][j]);
            cswap(sw, normU[k], normU[j]);
            cswap(sw, normD[k], normD[j]);
        }
        double tailSq = 0.0;
#pragma unroll
        for (int i = k + 1; i < N; ++i) tailSq += A[i][k] * A[i][k];
        const double c0 = A[k][k];
        double tau, beta;
        if (tailSq <= DBL_MIN) {
            tau = 0.0;
            beta = c0;
#pragma unroll
            for (int i = k + 1; i < N; ++i) A[i][k] = 0.0;
        } else {
            beta = sqrt(c0 * c0 + tailSq);
            if (c0 >= 0.0) beta = -beta;
#pragma unroll
            for (int i = k + 1; i < N; ++i) A[i][k] = A[i][k] / (c0 - beta);
            tau = (beta - c0) / beta;
        }
        hc[k] = tau;
        A[k][k] = beta;
        if (tau != 0.0) {
#pragma unroll
            for (int j = k + 1; j < N; ++j) {
                double tmp = 0.0;
#pragma unroll
                for (int i = k + 1; i < N; ++i) tmp += A[i][k] * A[i][j];
                tmp += A[k][j];
                A[k][j] -= tau * tmp;
#pragma unroll
                for (int i = k + 1; i < N; ++i) A[i][j] -= (tau * A[i][k]) * tmp;
            }
        }
#pragma unroll
        for (int j = k + 1; j < N; ++j) {
            if (normU[j] != 0.0) {
                double temp = fabs(A[k][j]) / normU[j];
                temp = (1.0 + temp) * (1.0 - temp);
                temp = temp < 0.0 ? 0.0 : temp;
                const double q = normU[j] / normD[j];
                if (temp * (q * q) <= downdateThr) {
                    double s = 0.0;
#pragma unroll
                    for (int i = k + 1; i < N; ++i) s += A[i][j] * A[i][j];
                    normD[j] = sqrt(s);
                    normU[j] = normD[j];
                } else {
                    normU[j] *= sqrt(temp);
                }
            }
        }
    }
    // permutation: perm = transpositions applied in order
    int perm[N] = { 0, 1, 2 };
#pragma unroll
    for (int k = 0; k < N; ++k)
#pragma unroll
        for (int j = k + 1; j < N; ++j) cswap(transp[k] == j, perm[k], perm[j]);
    if (nonzero == 0) {
        xout[0] = xout[1] = xout[2] = 0.0;
        return;
    }
    double c[N] = { bin[0], bin[1], bin[2] };
#pragma unroll
    for (int k = 0; k < N; ++k) {
        if (k >= nonzero) break;
        if (k == N - 1) {
            c[k] *= 1.0 - hc[k];
            continue;
        }
        if (hc[k] == 0.0) continue;
        double tmp = 0.0;
#pragma unroll
        for (int i = k + 1; i < N; ++i) tmp += A[i][k] * c[i];
        tmp += c[k];
        c[k] -= hc[k] * tmp;
#pragma unroll
        for (int i = k + 1; i < N; ++i) c[i] -= (hc[k] * A[i][k]) * tmp;
    }
#pragma unroll
    for (int i = N - 1; i >= 0; --i) {
        if (i < nonzero && c[i] != 0.0) {
            c[i] /= A[i][i];
#pragma unroll
            for (int j = 0; j < i; ++j) c[j] -= c[i] * A[j][i];
        }
    }
#pragma unroll
    for (int i = 0; i < N; ++i)
        if (i >= nonzero) c[i] = 0.0;
#pragma unroll
    for (int m = 0; m < N; ++m) {
        double v = 0.0;
#pragma unroll
        for (int i = 0; i < N; ++i) v = (perm[i] == m) ? c[i] : v;
        xout[m] = v;
    }
}

struct LsScanRef {
    const double* ranges;
    const double* angles;
    double min_range, max_range;   // ScanData min/max range (filters take the max/min with usable)
    double pose0[3];               // Compound(initialPose, relPose), glibc on the host
    int n;
    int pad;
};

// One pass over the beams at one sensor pose accumulates everything any
// phase of the loop needs at that pose:
//   [0..8]   OptimizeStep's b = sum e*g, H = sum g*g^T (upper triangle)
//            over beams in (step_min, step_max) (:100-132);
//   [9]      CostSquareError::Cost = sum e^2 over beams in (cost_min, cost_max);
//   [10..12] ComputeGradient's sum 2*e*(-g) over the same beams (:61-109).
// The reference's loop (step; cost at the new pose; convergence test) then
// needs one pass per iteration plus the first (:48-69).
constexpr int kAcc = 13;

__device__ __forceinline__ void pass(const LsPlan& p, const double* __restrict__ grid, const LsScanRef& sc,
                                     const double pose[3], double smin, double smax, double cmin,
                                     double cmax, double (&acc)[kAcc])
{
#pragma unroll
    for (int k = 0; k < kAcc; ++k) acc[k] = 0.0;
    for (int i = threadIdx.x; i < sc.n; i += kLsThreads) {
        const double r = sc.ranges[i];
        const bool in_step = !(r >= smax || r <= smin);
        const bool in_cost = !(r >= cmax || r <= cmin);
        if (!in_step && !in_cost) continue;
        double e, gv[3];
        beam_terms(p, grid, pose, r, sc.angles[i], e, gv);
        if (in_step) {
            acc[0] += e * gv[0];
            acc[1] += e * gv[1];
            acc[2] += e * gv[2];
            acc[3] += gv[0] * gv[0];
            acc[4] += gv[0] * gv[1];
            acc[5] += gv[0] * gv[2];
            acc[6] += gv[1] * gv[1];
            acc[7] += gv[1] * gv[2];
            acc[8] += gv[2] * gv[2];
        }
        if (in_cost) {
            acc[9] += e * e;   // pow(1.0 - S, 2.0): GCC folds it to the exact product
            acc[10] += 2.0 * e * (-gv[0]);
            acc[11] += 2.0 * e * (-gv[1]);
            acc[12] += 2.0 * e * (-gv[2]);
        }
    }
}

// The 13 sums of one beam (zeros for a beam outside both filters)
__device__ __forceinline__ void beam_acc(bool in_step, bool in_cost, double e, const double gv[3],
                                         double (&t)[kAcc])
{
#pragma unroll
    for (int k = 0; k < kAcc; ++k) t[k] = 0.0;
    if (in_step) {
        t[0] = e * gv[0];
        t[1] = e * gv[1];
        t[2] = e * gv[2];
        t[3] = gv[0] * gv[0];
        t[4] = gv[0] * gv[1];
        t[5] = gv[0] * gv[2];
        t[6] = gv[1] * gv[1];
        t[7] = gv[1] * gv[2];
        t[8] = gv[2] * gv[2];
    }
    if (in_cost) {
        t[9] = e * e;   // pow(1.0 - S, 2.0): GCC folds it to the exact product
        t[10] = 2.0 * e * (-gv[0]);
        t[11] = 2.0 * e * (-gv[1]);
        t[12] = 2.0 * e * (-gv[2]);
    }
}

__device__ __forceinline__ void wave_total(double (&t)[kAcc])
{
#pragma unroll
    for (int k = 0; k < kAcc; ++k)
        for (int off = 32; off > 0; off >>= 1) t[k] += __shfl_xor(t[k], off, 64);
}

// Summation order of a refine's sums (every kernel below uses it, so a lone
// refine, split or not, is bit-identical to the same refine in a batch):
// beams in groups of 64 (group g = beams 64 g .. 64 g + 63), each group summed
// by the wave64 xor butterfly (every lane ends with the same bits), the group
// totals then added in group order.
constexpr int kGroup = 64;
constexpr int kMaxGroups = 512;      // 32768 beams

// One pass of the batch kernel at `pose`: group g evaluated by wave g % 8,
// group totals through LDS, every thread returns the 13 totals.  Ends with a
// barrier, so `red` may be rewritten by the next pass.
__device__ __forceinline__ void group_pass(const LsPlan& p, const double* __restrict__ grid, const LsScanRef& sc,
                                           const double pose[3], double smin, double smax, double cmin,
                                           double cmax, double* red, double (&acc)[kAcc])
{
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int G = (sc.n + kGroup - 1) / kGroup;
    for (int g = wid; g < G; g += kLsThreads / 64) {
        const int i = g * kGroup + lane;
        bool in_step = false, in_cost = false;
        double e = 0.0, gv[3] = { 0.0, 0.0, 0.0 };
        if (i < sc.n) {
            const double r = sc.ranges[i];
            in_step = !(r >= smax || r <= smin);
            in_cost = !(r >= cmax || r <= cmin);
            if (in_step || in_cost) beam_terms(p, grid, pose, r, sc.angles[i], e, gv);
        }
        double t[kAcc];
        beam_acc(in_step, in_cost, e, gv, t);
        wave_total(t);
        if (lane < kAcc) {
            double v = t[0];
#pragma unroll
            for (int k = 1; k < kAcc; ++k) v = (lane == k) ? t[k] : v;
            red[g * kAcc + lane] = v;
        }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kAcc; ++k) {
        double v = red[k];
        for (int g = 1; g < G; ++g) v = v + red[g * kAcc + k];
        acc[k] = v;
    }
    __syncthreads();
}

// One workgroup per scan: the whole OptimizePose loop (:48-69) + covariance.
__global__ __launch_bounds__(kLsThreads) void k_linsolve(LsPlan p, const double* __restrict__ grid,
                                                         const LsScanRef* __restrict__ scans,
                                                         LsRecord* __restrict__ out,
                                                         double* __restrict__ traj)
{
    __shared__ double red[kMaxGroups * kAcc];
    __shared__ double spose[3];
    const LsScanRef sc = scans[blockIdx.x];
    const double smin = fmax(p.step_min, sc.min_range), smax = fmin(p.step_max, sc.max_range);
    const double cmin = fmax(p.cost_min, sc.min_range), cmax = fmin(p.cost_max, sc.max_range);
    double pose[3] = { sc.pose0[0], sc.pose0[1], sc.pose0[2] };
    double prevCost = DBL_MAX, cost = DBL_MAX;
    double acc[kAcc];
    group_pass(p, grid, sc, pose, smin, smax, cmin, cmax, red, acc);
    int it = 0;
    for (;;) {
        // OptimizeStep (:88-148): regularised normal equations, col-piv QR, pose += delta
        if (threadIdx.x == 0) {
            const double H[9] = { acc[3] + p.reg_t, acc[4], acc[5],
                                  acc[4], acc[6] + p.reg_t, acc[7],
                                  acc[5], acc[7], acc[8] + p.reg_r };
            const double b[3] = { acc[0], acc[1], acc[2] };
            double d[3];
            solve3_colpiv_qr(H, b, d);
            spose[0] = pose[0] + d[0];
            spose[1] = pose[1] + d[1];
            spose[2] = pose[2] + d[2];
        }
        __syncthreads();
        pose[0] = spose[0];
        pose[1] = spose[1];
        pose[2] = spose[2];
        // cost at the new pose (and the next step's sums, and the covariance
        // gradient should the loop stop here)
        group_pass(p, grid, sc, pose, smin, smax, cmin, cmax, red, acc);
        cost = acc[9];
        if (traj && threadIdx.x == 0) {
            double* tr = traj + ((size_t)blockIdx.x * max(1, p.max_iter) + it) * 4;
            tr[0] = pose[0];
            tr[1] = pose[1];
            tr[2] = pose[2];
            tr[3] = cost;
        }
        if (++it >= p.max_iter || fabs(prevCost - cost) < p.conv) break;
        prevCost = cost;
    }
    if (threadIdx.x == 0) {
        LsRecord rec;
        rec.pose[0] = pose[0];
        rec.pose[1] = pose[1];
        rec.pose[2] = pose[2];
        rec.cost = cost;
        rec.grad[0] = acc[10];
        rec.grad[1] = acc[11];
        rec.grad[2] = acc[12];
        rec.iterations = it;
        rec.pad = 0;
        out[blockIdx.x] = rec;
    }
}

// --------------------------------------------------------------------------
// Split refine (a lone OptimizePose, the frontend's case).  One workgroup of
// 8 waves per group of 64 beams (17 workgroups on 17 CUs for 1081 beams; with
// more than kSplitMaxWG groups a workgroup takes groups wg, wg + nwg, ...).
// The waves share the work of a beam (lane = beam): waves 0-5 compute the
// hit cell and one bicubic axis each (x0, y0, xp, xm, yp, ym; through LDS),
// waves 0-4 one smoothed value each, then waves 0-3 finish the beam (the same
// bits in each), and each sums a quarter of the 13 group sums with the
// butterfly and publishes them -- the same functions on the same inputs as
// beam_terms, so the bits are the batch kernel's.  Measured per pass on
// config 3 (LGS_LS_TRACE): hit cell + axes 1.45 us, smoothed values 1.1 us,
// finish + sums + publish 1.5 -> (8 waves) less, hand-off 1.5-3.5 us after
// the last publisher, 3x3 col-piv QR 1.65 us.
// Per pass every group total is published as 26 write-through 8-byte granules
// {tag = pass + 1, 32 bits of a double} (cdna_hip_programming.md,
// publish/consume recipe R2: the data is the flag, agent-scope relaxed
// atomics, no fence); wave 0 of every workgroup sweeps all G x 26 granules
// until every tag matches, adds the totals in group order and runs the 3x3
// solve itself, so every workgroup holds the identical pose and takes the
// identical stopping decision (no broadcast, no second hand-off per pass).
// Granules are double-buffered by pass parity: a workgroup publishes pass
// p + 2 only after every workgroup has published p + 1, i.e. finished reading
// pass p.  Spins are bounded (~0.2 s of s_memrealtime): on time-out the
// timeout word is set, every workgroup leaves, and the host reports an error.
// --------------------------------------------------------------------------
constexpr int kSplitThreads = 512;
constexpr int kSplitMaxWG = 64;
constexpr int kSplitMaxGroups = 128;     // larger scans use one workgroup (k_linsolve)
constexpr int kGran = 2 * kAcc;          // granules per group and pass
typedef __attribute__((address_space(1))) unsigned long long gu64;
typedef __attribute__((address_space(1))) unsigned gu32;

struct SplitLds {
    Axis ax[6][kGroup];                  // x0, y0, xp, xm, yp, ym
    double sv[5][kGroup];                // S(x0,y0), S(xp,y0), S(xm,y0), S(x0,yp), S(x0,ym)
    double sc[2][kGroup];                // sin, cos of the beam angle
    double br[kSplitMaxGroups / kSplitMaxWG][kGroup];   // the workgroup's ranges and angles, loaded once
    double ba[kSplitMaxGroups / kSplitMaxWG][kGroup];
    unsigned gran[kSplitMaxGroups * kGran];
    double tot[kAcc];
    double pose[3];
    int stop;
};

// wave 0: wait for every group's granules of this pass, then the totals in
// group order (every lane)
__device__ __forceinline__ bool consume(gu64* __restrict__ slot, gu32* __restrict__ tmo, int G, unsigned epoch,
                                        unsigned* __restrict__ lds, double (&acc)[kAcc])
{
    const int lane = threadIdx.x;
    const int total = G * kGran;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    for (unsigned polls = 1;; ++polls) {
        // every load of a sweep chunk in flight before the first is waited on
        // (a strided loop waits on each load in turn: 7 round trips per poll)
        bool ok = true;
        for (int base = 0; base < total; base += 64 * 8) {
            unsigned long long x[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int q = base + u * 64 + lane;
                x[u] = (q < total) ? __hip_atomic_load(slot + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                   : ((unsigned long long)epoch << 32);
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int q = base + u * 64 + lane;
                if (q < total) lds[q] = (unsigned)x[u];
                ok &= (unsigned)(x[u] >> 32) == epoch;
            }
        }
        if (__all(ok)) break;
        // the timeout word is one more round trip: looked at every 256 polls only
        if ((polls & 255u) == 0u) {
            if (__hip_atomic_load(tmo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) return false;
            if (__builtin_amdgcn_s_memrealtime() - t0 > 20000000ull) {   // 100 MHz clock: 0.2 s
                if (lane == 0) __hip_atomic_store(tmo, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                return false;
            }
        }
    }
    __builtin_amdgcn_wave_barrier();
    double sk = 0.0;
    if (lane < kAcc)
        for (int g = 0; g < G; ++g) {
            const unsigned lo = lds[g * kGran + 2 * lane], hi = lds[g * kGran + 2 * lane + 1];
            const double v = __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
            sk = (g == 0) ? v : sk + v;
        }
#pragma unroll
    for (int k = 0; k < kAcc; ++k) acc[k] = __shfl(sk, k, 64);
    return true;
}

// the workgroup's groups of one pass; wave 0 publishes each group's totals
// diagnostics (env LGS_LS_TRACE=1): workgroup 0 stamps s_memrealtime at the
// phase boundaries of every pass
__device__ __forceinline__ void stamp(unsigned long long* tr, int k)
{
    if (tr && blockIdx.x == 0 && threadIdx.x == 0) tr[k] = __builtin_amdgcn_s_memrealtime();
}

// wave w of the 4 finishing waves: sums kSumLo[w] .. kSumLo[w + 1] - 1
__device__ __forceinline__ int sum_lo(int w) { return (w * kAcc + 3) / 4; }   // 0, 4, 7, 10, 13

__device__ __forceinline__ void split_pass(const LsPlan& p, const double* __restrict__ grid, const LsScanRef& sc,
                                           const double pose[3], double smin, double smax, double cmin, double cmax,
                                           int G, gu64* __restrict__ slot, unsigned epoch, SplitLds& L,
                                           unsigned long long* tr, unsigned long long* tr2)
{
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    for (int g = blockIdx.x, k = 0; g < G; g += gridDim.x, ++k) {
        const int i = g * kGroup + lane;
        bool in_step = false, in_cost = false;
        double r = 0.0, sn = 0.0, cs = 0.0, fx = 0.0, fy = 0.0;
        if (i < sc.n) {
            r = L.br[k][lane];
            in_step = !(r >= smax || r <= smin);
            in_cost = !(r >= cmax || r <= cmin);
        }
        const bool act = in_step || in_cost;
        // phase A: the hit cell (every wave), one axis per wave 0..5
        if (act && wid < 6) {
            beam_cell(p, pose, r, L.ba[k][lane], sn, cs, fx, fy);
            const double d = kHalfDelta;
            const bool isx = !(wid & 1);
            const double v = (wid < 2) ? (isx ? fx : fy) : (wid < 4) ? (fx + ((wid == 2) ? d : -d))
                                                                     : (fy + ((wid == 4) ? d : -d));
            // ax order: x0, y0, xp, xm, yp, ym
            L.ax[wid][lane] = make_axis(v, (wid == 0 || wid == 2 || wid == 3) ? p.W : p.H);
            if (wid == 0) {
                L.sc[0][lane] = sn;
                L.sc[1][lane] = cs;
            }
        }
        __syncthreads();
        stamp(tr, 1);
        // phase B: one smoothed value per wave 0..4
        if (act && wid < 5) {
            const int xa = (wid == 1) ? 2 : (wid == 2) ? 3 : 0;
            const int ya = (wid == 3) ? 4 : (wid == 4) ? 5 : 1;
            L.sv[wid][lane] = smoothed(grid, p.W, L.ax[xa][lane], L.ax[ya][lane]);
        }
        __syncthreads();
        stamp(tr, 2);
        // phase C: waves 0..3 finish the beam (identical bits in each), sum
        // their share of the 13 sums over the group and publish it
        if (wid < 4) {
            double e = 0.0, gv[3] = { 0.0, 0.0, 0.0 };
            if (act)
                beam_finish(p, r, L.sc[0][lane], L.sc[1][lane], L.sv[0][lane], L.sv[1][lane], L.sv[2][lane],
                            L.sv[3][lane], L.sv[4][lane], e, gv);
            double t[kAcc];
            beam_acc(in_step, in_cost, e, gv, t);
            const int lo = sum_lo(wid), hi = sum_lo(wid + 1);
#pragma unroll
            for (int k = 0; k < kAcc; ++k)
                if (k >= lo && k < hi)
                    for (int off = 32; off > 0; off >>= 1) t[k] += __shfl_xor(t[k], off, 64);
            // lane j < 2 (hi - lo) publishes half j & 1 of sum lo + (j >> 1)
            if (lane == 0)
#pragma unroll
                for (int k = 0; k < kAcc; ++k)
                    if (k >= lo && k < hi) L.tot[k] = t[k];
            __builtin_amdgcn_wave_barrier();
            const int nk = 2 * (hi - lo);
            if (lane < nk) {
                const double mine = L.tot[lo + (lane >> 1)];
                const unsigned long long bits = (unsigned long long)__double_as_longlong(mine);
                const unsigned half = (lane & 1) ? (unsigned)(bits >> 32) : (unsigned)bits;
                __hip_atomic_store(slot + (size_t)g * kGran + 2 * lo + lane, ((unsigned long long)epoch << 32) | half,
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            stamp(tr, 3);
            if (tr2 && threadIdx.x == 0) tr2[blockIdx.x] = __builtin_amdgcn_s_memrealtime();
        }
        __syncthreads();   // LDS axes / values free for the next group
    }
}

__global__ __launch_bounds__(kSplitThreads) void k_linsolve_split(LsPlan p, const double* __restrict__ grid,
                                                                  LsScanRef sc, LsRecord* __restrict__ out,
                                                                  double* __restrict__ traj,
                                                                  gu64* __restrict__ gran, gu32* __restrict__ tmo,
                                                                  unsigned long long* __restrict__ trace)
{
    __shared__ SplitLds L;
    const int wid = threadIdx.x >> 6;
    const double smin = fmax(p.step_min, sc.min_range), smax = fmin(p.step_max, sc.max_range);
    const double cmin = fmax(p.cost_min, sc.min_range), cmax = fmin(p.cost_max, sc.max_range);
    const int G = (sc.n + kGroup - 1) / kGroup;
    double pose[3] = { sc.pose0[0], sc.pose0[1], sc.pose0[2] };
    // the workgroup's beams stay in LDS for every pass
    for (int g = blockIdx.x, k = 0; g < G; g += gridDim.x, ++k)
        if (threadIdx.x < kGroup && g * kGroup + (int)threadIdx.x < sc.n) {
            L.br[k][threadIdx.x] = sc.ranges[g * kGroup + threadIdx.x];
            L.ba[k][threadIdx.x] = sc.angles[g * kGroup + threadIdx.x];
        }
    __syncthreads();
    double acc[kAcc];
    int pass_idx = 0;
    double prevCost = DBL_MAX, cost = DBL_MAX;
    int it = 0;
    for (;;) {
        gu64* slot = gran + (size_t)(pass_idx & 1) * kSplitMaxGroups * kGran;
        const unsigned epoch = (unsigned)pass_idx + 1u;
        unsigned long long* tr = trace ? trace + (size_t)min(pass_idx, 127) * 8 : nullptr;
        unsigned long long* tr2 = trace ? trace + 128 * 8 + (size_t)min(pass_idx, 127) * 64 : nullptr;
        stamp(tr, 0);
        split_pass(p, grid, sc, pose, smin, smax, cmin, cmax, G, slot, epoch, L, tr, tr2);
        if (wid == 0) {
            int stop = 0;
            const bool ok = consume(slot, tmo, G, epoch, L.gran, acc);
            stamp(tr, 4);
            if (!ok) {
                stop = 2;
            } else {
                if (pass_idx > 0) {
                    cost = acc[9];
                    if (traj && blockIdx.x == 0 && threadIdx.x == 0) {
                        double* tr = traj + (size_t)it * 4;
                        tr[0] = pose[0];
                        tr[1] = pose[1];
                        tr[2] = pose[2];
                        tr[3] = cost;
                    }
                    if (++it >= p.max_iter || fabs(prevCost - cost) < p.conv) stop = 1;
                    prevCost = cost;
                }
                if (!stop) {
                    // OptimizeStep (:88-148), solved by every lane of wave 0 of every workgroup
                    const double H[9] = { acc[3] + p.reg_t, acc[4], acc[5],
                                          acc[4], acc[6] + p.reg_t, acc[7],
                                          acc[5], acc[7], acc[8] + p.reg_r };
                    const double b[3] = { acc[0], acc[1], acc[2] };
                    double d[3];
                    solve3_colpiv_qr(H, b, d);
                    pose[0] = pose[0] + d[0];
                    pose[1] = pose[1] + d[1];
                    pose[2] = pose[2] + d[2];
                }
            }
            stamp(tr, 5);
            if (threadIdx.x == 0) {
                L.pose[0] = pose[0];
                L.pose[1] = pose[1];
                L.pose[2] = pose[2];
                L.stop = stop;
            }
        }
        __syncthreads();
        const int stop = L.stop;
        pose[0] = L.pose[0];
        pose[1] = L.pose[1];
        pose[2] = L.pose[2];
        __syncthreads();
        if (stop == 2) return;
        if (stop) break;
        ++pass_idx;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        LsRecord rec;
        rec.pose[0] = pose[0];
        rec.pose[1] = pose[1];
        rec.pose[2] = pose[2];
        rec.cost = cost;
        rec.grad[0] = acc[10];
        rec.grad[1] = acc[11];
        rec.grad[2] = acc[12];
        rec.iterations = it;
        rec.pad = 0;
        out[0] = rec;
    }
}

// CostSquareError::Cost and ComputeGradient sums at one pose (diagnostics):
// out[0] = cost, out[1..3] = sum 2 e (-grad)
__global__ __launch_bounds__(kLsThreads) void k_sq_cost(LsPlan p, const double* __restrict__ grid,
                                                        LsScanRef sc, double* __restrict__ out)
{
    __shared__ double red[kAcc * (kLsThreads / 64)];
    const double cmin = fmax(p.cost_min, sc.min_range), cmax = fmin(p.cost_max, sc.max_range);
    double acc[kAcc];
    // step filter empty: only the cost-side sums are accumulated
    pass(p, grid, sc, sc.pose0, 0.0, 0.0, cmin, cmax, acc);
    wg_sum(acc, red);
    if (threadIdx.x == 0) {
        out[0] = acc[9];
        out[1] = acc[10];
        out[2] = acc[11];
        out[3] = acc[12];
    }
}

LsPlan make_ls_plan(const lgs_grid* g, const lgs_linsolve_params* prm)
{
    LsPlan p{};
    p.min_x = g->min_x;
    p.min_y = g->min_y;
    p.res = g->res;
    p.W = g->w;
    p.H = g->h;
    p.max_iter = prm->num_iterations_max;
    p.conv = prm->convergence_threshold;
    p.step_min = prm->usable_range_min;
    p.step_max = prm->usable_range_max;
    p.cost_min = prm->cost_usable_range_min;
    p.cost_max = prm->cost_usable_range_max;
    p.reg_t = prm->translation_regularizer;
    p.reg_r = prm->rotation_regularizer;
    return p;
}

LsScanRef scan_ref(const lgs_scan* s, lgs_pose2d initial)
{
    LsScanRef r{};
    r.ranges = s->d_ranges;
    r.angles = s->d_angles;
    r.min_range = s->min_range;
    r.max_range = s->max_range;
    const lgs_pose2d sp = compound(initial, s->rel);
    r.pose0[0] = sp.x;
    r.pose0[1] = sp.y;
    r.pose0[2] = sp.theta;
    r.n = s->n;
    return r;
}

void check_grid(const lgs_grid* g)
{
    LGS_REQUIRE(g && g->d && g->w >= 1 && g->h >= 1, "grid must be non-empty");
}

void run_linsolve(lgs_ctx* ctx, const lgs_grid* grid, const lgs_linsolve_params* prm,
                  const lgs_scan* const* scans, const lgs_pose2d* init, int n,
                  lgs_linsolve_summary* out, double* traj)
{
    check_grid(grid);
    LGS_REQUIRE(prm, "null params");
    LGS_HIP_CHECK(hipSetDevice(ctx->device));
    const LsPlan p = make_ls_plan(grid, prm);
    const int iters = std::max(1, p.max_iter);
    std::vector<LsScanRef> refs(n);
    for (int j = 0; j < n; ++j) {
        LGS_REQUIRE(scans[j] && scans[j]->n >= 1, "empty scan");
        LGS_REQUIRE(scans[j]->n <= kMaxGroups * kGroup, "scan has more than 32768 beams");
        refs[j] = scan_ref(scans[j], init[j]);
    }
    // pinned staging: [refs | records | trajectory]
    const size_t b_refs = sizeof(LsScanRef) * n, b_rec = sizeof(LsRecord) * n;
    const size_t b_traj = traj ? sizeof(double) * 4 * (size_t)iters * n : 0;
    char* h = (char*)ctx->ensure_pinned(b_refs + b_rec + b_traj + 16);   // + the split refine's timeout word
    std::memcpy(h, refs.data(), b_refs);
    char* d = (char*)ctx->ensure(S_LIN0, b_refs + b_rec + b_traj);
    LGS_HIP_CHECK(hipMemcpyAsync(d, h, b_refs, hipMemcpyHostToDevice, ctx->stream));
    const int groups = (refs[0].n + kGroup - 1) / kGroup;
    const bool split = n == 1 && ctx->linsolve_split && groups <= kSplitMaxGroups;
    const int split_wg = std::min(groups, kSplitMaxWG);
    constexpr size_t b_gran = sizeof(unsigned long long) * 2 * kSplitMaxGroups * kGran;   // multiple of 16
    char* hs = split ? (char*)ctx->ensure(S_LIN2, b_gran + 16) : nullptr;
    if (split)   // granule tags and the timeout word zeroed every call (one block from the start)
        LGS_HIP_CHECK(hipMemsetAsync(hs, 0, b_gran + 16, ctx->stream));
    // diagnostics: LGS_LS_TRACE=1 prints the split refine's phase stamps
    static const bool trace_on = getenv("LGS_LS_TRACE") != nullptr;
    unsigned long long* trace_dev = nullptr;
    if (split && trace_on) {
        trace_dev = (unsigned long long*)ctx->ensure(S_LIN3, 128 * 72 * sizeof(unsigned long long));
        LGS_HIP_CHECK(hipMemsetAsync(trace_dev, 0, 128 * 72 * sizeof(unsigned long long), ctx->stream));
    }
    const int tok = ctx->timing_begin(K_LINSOLVE, 0.0);
    if (split)
        hipLaunchKernelGGL(k_linsolve_split, dim3(split_wg), dim3(kSplitThreads), 0, ctx->stream, p, grid->d, refs[0],
                           (LsRecord*)(d + b_refs), traj ? (double*)(d + b_refs + b_rec) : nullptr, (gu64*)hs,
                           (gu32*)(hs + b_gran), trace_dev);
    else
        hipLaunchKernelGGL(k_linsolve, dim3(n), dim3(kLsThreads), 0, ctx->stream, p, grid->d,
                           (const LsScanRef*)d, (LsRecord*)(d + b_refs),
                           traj ? (double*)(d + b_refs + b_rec) : nullptr);
    ctx->timing_end(tok);
    LGS_HIP_CHECK(hipGetLastError());
    LGS_HIP_CHECK(hipMemcpyAsync(h + b_refs, d + b_refs, b_rec + b_traj, hipMemcpyDeviceToHost,
                                 ctx->stream));
    unsigned* htmo = (unsigned*)(h + b_refs + b_rec + b_traj);
    if (split) LGS_HIP_CHECK(hipMemcpyAsync(htmo, hs + b_gran, sizeof(unsigned), hipMemcpyDeviceToHost, ctx->stream));
    ctx->sync();
    if (ctx->profile) ctx->harvest();
    if (split && *htmo != 0u) throw Error(LGS_ERR_INTERNAL, "split refine: in-launch hand-off timed out");
    if (trace_dev) {
        std::vector<unsigned long long> t(128 * 72);
        LGS_HIP_CHECK(hipMemcpy(t.data(), trace_dev, t.size() * sizeof(t[0]), hipMemcpyDeviceToHost));
        for (int q = 0; q < 128 && t[q * 8]; ++q) {
            fprintf(stderr, "LSTRACE pass %d:", q);
            for (int k = 1; k < 6; ++k)
                fprintf(stderr, " %.2f", t[q * 8 + k] ? 0.01 * (double)(t[q * 8 + k] - t[q * 8]) : -1.0);
            if (q + 1 < 128 && t[(q + 1) * 8]) fprintf(stderr, " | next %.2f", 0.01 * (double)(t[(q + 1) * 8] - t[q * 8]));
            fprintf(stderr, " | pub");
            for (int w = 0; w < split_wg; ++w) {
                const unsigned long long v = t[128 * 8 + q * 64 + w];
                fprintf(stderr, " %.2f", v ? 0.01 * ((double)v - (double)t[q * 8]) : -1.0);
            }
            fprintf(stderr, "\n");
        }
    }
    const LsRecord* rec = (const LsRecord*)(h + b_refs);
    for (int j = 0; j < n; ++j) {
        lgs_linsolve_summary& o = out[j];
        std::memset(&o, 0, sizeof(o));
        const LsRecord& r = rec[j];
        o.pose_found = 1;
        o.iterations = r.iterations;
        o.cost = r.cost;
        o.normalized_cost = r.cost / (double)scans[j]->n;
        o.initial_pose = init[j];
        o.sensor_pose = { refs[j].pose0[0], refs[j].pose0[1], refs[j].pose0[2] };
        o.best_sensor_pose = { r.pose[0], r.pose[1], r.pose[2] };
        o.estimated_pose = move_backward(o.best_sensor_pose, scans[j]->rel);
        for (int a = 0; a < 3; ++a)
            for (int b = 0; b < 3; ++b) o.covariance[3 * a + b] = r.grad[a] * r.grad[b];
        o.covariance[0] += 0.01;
        o.covariance[4] += 0.01;
        o.covariance[8] += 0.01;
    }
    if (traj) {
        const double* t = (const double*)(h + b_refs + b_rec);
        std::memcpy(traj, t, sizeof(double) * 4 * (size_t)out[0].iterations);
    }
}

}  // namespace

extern "C" int lgs_linsolve_optimize_pose(lgs_ctx* ctx, const lgs_grid* grid,
                                          const lgs_linsolve_params* params, const lgs_scan* scan,
                                          lgs_pose2d initial, lgs_linsolve_summary* out,
                                          double* trajectory)
{
    if (!ctx || !grid || !params || !scan || !out) return LGS_ERR_INVALID_ARG;
    return guarded(ctx, [&] { run_linsolve(ctx, grid, params, &scan, &initial, 1, out, trajectory); });
}

extern "C" int lgs_linsolve_optimize_pose_batch(lgs_ctx* ctx, const lgs_grid* grid,
                                                const lgs_linsolve_params* params,
                                                const lgs_scan* const* scans,
                                                const lgs_pose2d* initial, int n,
                                                lgs_linsolve_summary* out)
{
    if (!ctx || !grid || !params || !scans || !initial || !out || n < 0) return LGS_ERR_INVALID_ARG;
    if (n == 0) return LGS_OK;
    return guarded(ctx, [&] { run_linsolve(ctx, grid, params, scans, initial, n, out, nullptr); });
}

extern "C" int lgs_cost_square_error(lgs_ctx* ctx, const lgs_grid* grid, double umin, double umax,
                                     const lgs_scan* scan, lgs_pose2d sensor_pose, double* out_cost,
                                     double* out_cov)
{
    if (!ctx || !grid || !scan || !out_cost) return LGS_ERR_INVALID_ARG;
    return guarded(ctx, [&] {
        check_grid(grid);
        LGS_HIP_CHECK(hipSetDevice(ctx->device));
        lgs_linsolve_params prm{};
        prm.cost_usable_range_min = umin;
        prm.cost_usable_range_max = umax;
        const LsPlan p = make_ls_plan(grid, &prm);
        LsScanRef r = scan_ref(scan, { 0, 0, 0 });
        r.pose0[0] = sensor_pose.x;
        r.pose0[1] = sensor_pose.y;
        r.pose0[2] = sensor_pose.theta;
        double* d = (double*)ctx->ensure(S_LIN1, 4 * sizeof(double));
        double* h = (double*)ctx->ensure_pinned(4 * sizeof(double));
        hipLaunchKernelGGL(k_sq_cost, dim3(1), dim3(kLsThreads), 0, ctx->stream, p, grid->d, r, d);
        LGS_HIP_CHECK(hipGetLastError());
        LGS_HIP_CHECK(hipMemcpyAsync(h, d, 4 * sizeof(double), hipMemcpyDeviceToHost, ctx->stream));
        ctx->sync();
        *out_cost = h[0];
        if (out_cov) {
            for (int a = 0; a < 3; ++a)
                for (int b = 0; b < 3; ++b) out_cov[3 * a + b] = h[1 + a] * h[1 + b];
            out_cov[0] += 0.01;
            out_cov[4] += 0.01;
            out_cov[8] += 0.01;
        }
    });
}
