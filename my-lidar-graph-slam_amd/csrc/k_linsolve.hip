// k_linsolve.hip -- K4: Gauss-Newton scan matcher (ScanMatcherLinearSolver) on MI355X.
//
// Restates ScanMatcherLinearSolver::OptimizePose / OptimizeStep
// (C/mapping/scan_matcher_linear_solver.cpp:38-148) with CostSquareError
// (C/mapping/cost_function_square_error.cpp: Cost :21-58, ComputeCovariance
// :112-135, ComputeMapGradient :172-229, ComputeSmoothedValue :276-346).
//
// One workgroup runs one whole refine (all iterations) without returning to
// the host; a batch launches one workgroup per scan.  Per pass every thread
// evaluates beams of the current chunk (the bicubic smoothed value and its
// central-difference map gradient: 5 x 16 independent gathers per beam) and
// writes the beam's 13 terms to LDS; lanes 0..12 of wave 0 then add the
// terms in beam order, one lane per sum -- the reference's own sequential
// fp64 sums (scan_matcher_linear_solver.cpp:105-133,
// cost_function_square_error.cpp:21-58, :61-109).  Lane 0 solves the
// regularised 3x3 system with the column-pivoting Householder QR Eigen's
// colPivHouseholderQr uses (restated, Eigen is not vendored) and updates the
// pose; the same pass at the new pose gives the cost for the convergence
// test and the next step's sums.
//
// Numerics: sin/cos of a beam are glibc's sincos() and
// pow(x, 3.0) is glibc's pow(), both restated bit-exactly (glibc_math.hpp,
// pinned against this image's libm by tests/test_libm_pin.py); pow(x, 2.0) is
// the exact x*x GCC folds it to; every sum runs in beam order.  The device
// therefore performs the oracle's arithmetic operation for operation, and its
// trajectory is the oracle's bit for bit.
#include "lgs_internal.hpp"
#include "glibc_math.hpp"

#include <cfloat>
#include <climits>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

using namespace lgs;

namespace {

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

// bicubic kernel h(t) (:281-295): pow(at, 3.0) is glibc's pow (restated bit-exactly),
// pow(at, 2.0) is at*at after GCC folding
__device__ __forceinline__ double bicubic_h(double t)
{
    const double at = fabs(t);
    if (at <= 1.0) {
        const double at3 = glm::gl_pow3(at);
        const double at2 = at * at;
        return (at3 - 2.0 * at2 + 1.0);
    } else if (at <= 2.0) {
        const double at3 = glm::gl_pow3(at);
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
    glm::gl_sincos(pose[2] + a, &sn, &cs);   // GCC fuses the reference's cos/sin pair into sincos()
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
// needs one pass per iteration plus the first (:48-69).  A beam outside a
// filter contributes +0.0 to that filter's sums, which leaves a sum that
// started at +0.0 unchanged bit for bit (it is never -0.0).
constexpr int kAcc = 13;

// The 13 terms of one beam (zeros for a beam outside both filters)
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

// Workgroup shape: kLsThreads threads evaluate up to kChunk beams per chunk
// (a 1081-beam scan is one chunk), their terms staged in LDS rows of
// kTermStride doubles (16-byte aligned rows; the 13 summing lanes read
// distinct banks).
constexpr int kLsThreads = 512;
constexpr int kChunk = 1280;
constexpr int kTermStride = kChunk + 2;

struct alignas(16) LsLds {
    double terms[kAcc][kTermStride];
    double pose[3];
};

// s + row[0] + row[1] + ... + row[m-1], strictly in that order (LDS row,
// 16-byte aligned).  Software-pipelined with two register buffers of 8
// terms: one buffer's loads are in flight while the other's are added, so
// the chain waits on the adds only.
constexpr int kSeqBuf = 4;   // double2 per buffer: a 64-beam group is 4 buffer pairs, 8 loads in flight

__device__ __forceinline__ double add_buf(double s, const double2 (&a)[kSeqBuf])
{
#pragma unroll
    for (int q = 0; q < kSeqBuf; ++q) {
        s = s + a[q].x;
        s = s + a[q].y;
    }
    return s;
}

__device__ __forceinline__ void load_buf(double2 (&a)[kSeqBuf], const double* __restrict__ p)
{
#pragma unroll
    for (int q = 0; q < kSeqBuf; ++q) a[q] = *(const double2*)(p + 2 * q);
}

__device__ __forceinline__ double seq_add(double s, const double* __restrict__ row, int m)
{
    constexpr int B = 2 * kSeqBuf;   // terms per buffer
    int j = 0;
    if (m >= 2 * B) {
        double2 a[kSeqBuf], b[kSeqBuf];
        load_buf(a, row);
        load_buf(b, row + B);
        for (j = 2 * B; j + 2 * B <= m; j += 2 * B) {
            // the scheduling barriers keep each buffer's loads issued a whole
            // buffer of adds before its first use
            __builtin_amdgcn_sched_barrier(0);
            s = add_buf(s, a);
            __builtin_amdgcn_sched_barrier(0);
            load_buf(a, row + j);
            __builtin_amdgcn_sched_barrier(0);
            s = add_buf(s, b);
            __builtin_amdgcn_sched_barrier(0);
            load_buf(b, row + j + B);
        }
        __builtin_amdgcn_sched_barrier(0);
        s = add_buf(s, a);
        s = add_buf(s, b);
    }
    for (; j < m; ++j) s = s + row[j];
    return s;
}

// One pass at `pose`: lane k < 13 of wave 0 returns sum k in beam order
// (other threads return 0).  Ends with a barrier, so the LDS rows may be
// rewritten by the next pass.
__device__ __forceinline__ double seq_pass(const LsPlan& p, const double* __restrict__ grid, const LsScanRef& sc,
                                           const double pose[3], double smin, double smax, double cmin,
                                           double cmax, LsLds& L)
{
    double s = 0.0;
    for (int c0 = 0; c0 < sc.n; c0 += kChunk) {
        const int m = min(kChunk, sc.n - c0);
        for (int j = threadIdx.x; j < m; j += kLsThreads) {
            const double r = sc.ranges[c0 + j];
            const bool in_step = !(r >= smax || r <= smin);
            const bool in_cost = !(r >= cmax || r <= cmin);
            double e = 0.0, gv[3] = { 0.0, 0.0, 0.0 };
            if (in_step || in_cost) beam_terms(p, grid, pose, r, sc.angles[c0 + j], e, gv);
            double t[kAcc];
            beam_acc(in_step, in_cost, e, gv, t);
#pragma unroll
            for (int k = 0; k < kAcc; ++k) L.terms[k][j] = t[k];
        }
        __syncthreads();
        if (threadIdx.x < kAcc) s = seq_add(s, L.terms[threadIdx.x], m);
        __syncthreads();
    }
    return s;
}

// the 13 sums from lanes 0..12 of wave 0 into every lane of wave 0
__device__ __forceinline__ void gather_sums(double s, double (&acc)[kAcc])
{
#pragma unroll
    for (int k = 0; k < kAcc; ++k) acc[k] = __shfl(s, k, 64);
}

// One workgroup per scan: the whole OptimizePose loop (:48-69) + covariance.
__global__ __launch_bounds__(kLsThreads) void k_linsolve(LsPlan p, const double* __restrict__ grid,
                                                         const LsScanRef* __restrict__ scans,
                                                         LsRecord* __restrict__ out,
                                                         double* __restrict__ traj)
{
    __shared__ LsLds L;
    const LsScanRef sc = scans[blockIdx.x];
    const double smin = fmax(p.step_min, sc.min_range), smax = fmin(p.step_max, sc.max_range);
    const double cmin = fmax(p.cost_min, sc.min_range), cmax = fmin(p.cost_max, sc.max_range);
    double pose[3] = { sc.pose0[0], sc.pose0[1], sc.pose0[2] };
    double prevCost = DBL_MAX, cost = DBL_MAX;
    double acc[kAcc];
    gather_sums(seq_pass(p, grid, sc, pose, smin, smax, cmin, cmax, L), acc);   // wave 0 only is meaningful
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
            L.pose[0] = pose[0] + d[0];
            L.pose[1] = pose[1] + d[1];
            L.pose[2] = pose[2] + d[2];
        }
        __syncthreads();
        pose[0] = L.pose[0];
        pose[1] = L.pose[1];
        pose[2] = L.pose[2];
        // cost at the new pose (and the next step's sums, and the covariance
        // gradient should the loop stop here); every thread needs the cost
        // for the stopping rule: through LDS
        gather_sums(seq_pass(p, grid, sc, pose, smin, smax, cmin, cmax, L), acc);
        if (threadIdx.x == 0) L.pose[0] = acc[9];
        __syncthreads();
        cost = L.pose[0];
        __syncthreads();
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
// Split refine (a lone OptimizePose, the frontend's case): one workgroup of 8
// waves per group of 64 beams (17 workgroups on 17 CUs for 1081 beams), all
// passes in one launch.  The waves share the work of a beam (lane = beam):
// waves 0-5 compute the hit point and one bicubic axis each (x0, y0, xp, xm,
// yp, ym; 4 glibc pow() per axis) into LDS, waves 0-4 one smoothed value
// each, wave 0 finishes the beam -- the functions of beam_terms on the same
// inputs, so the bits are the batch kernel's.  Every workgroup publishes its
// beams' 13 terms (write-through stores, one flag per group;
// cdna_hip_programming.md Guideline 16, recipe R1), then EVERY workgroup
// waits for all groups, stages all terms into LDS and adds them in beam order
// (13 lanes of wave 0, group by group as the other 7 waves stage the groups
// into LDS in beam order) and solves the 3x3 system itself: every workgroup
// holds the identical pose and takes the identical stopping decision, no
// broadcast.  Terms and flags are double-buffered by pass parity: a
// workgroup publishes pass p + 2 only after every group has published p + 1,
// i.e. finished reading pass p.
// Residency: the host launches it only when the device can hold all its
// workgroups at once (occupancy query); spins are bounded (~0.2 s of
// s_memrealtime) and on time-out every workgroup leaves and the host reruns
// the refine with k_linsolve (one workgroup), which computes the same bits.
// --------------------------------------------------------------------------
constexpr int kGroup = 64;
constexpr int kSplitThreads = 512;
constexpr int kSplitMaxGroups = kChunk / kGroup;          // 20 groups: 1280 beams
typedef __attribute__((address_space(1))) unsigned long long gu64;
typedef __attribute__((address_space(1))) unsigned gu32;

struct alignas(16) SplitLds {
    double terms[kAcc][kTermStride];   // all groups' terms of one pass, beam order per row
    struct {
        Axis ax[6][kGroup];            // x0, y0, xp, xm, yp, ym
        double sv[5][kGroup];          // S(x0,y0), S(xp,y0), S(xm,y0), S(x0,yp), S(x0,ym)
        double sc[2][kGroup];          // sin, cos of the beam angle
    } b;
    double pose[3];
    unsigned ready[kSplitMaxGroups];   // group staged in `terms` for pass epoch
    int stop;
    int abort;
};

// seq_add over a row whose 64-beam groups are staged by other waves: each
// group is added once its LDS flag shows (an acquire, so its loads stay
// behind it); a full group is one fully unrolled block of 32 16-byte loads and
// 64 adds, so the compiler pipelines the loads against the add chain without
// loop-carried copies.  Returns 0 early if another wave set *abort.
//
// LGS_SEQ_PIPE (r06, default): the operands in a ring of four 8-term
// register chunks (half a group).  Each chunk is reloaded with the next half
// group's terms as soon as its adds are issued, so the LDS loads run half a
// group ahead of the chain instead of every group's loads (and flag) waiting
// in front of its adds.  The next group's flag is read between a group's two
// halves: LDS operations of a wave complete in order, so waiting for the flag
// costs only the wait for the second half's loads, which its adds need next
// anyway; the loads of the next group are issued after the flag read that
// saw it staged (in-order LDS, the staging wave's release), hence see its
// rows.  No load sits under a branch (a conditional reload made the compiler
// copy every chunk and drain the loads at each half), and an empty volatile
// asm on s after each half keeps its adds ahead of the next flag wait.  The last group is
// added in full: lanes past n publish +0.0 terms (beam_acc of an unused beam)
// and s + 0.0 == s bit for bit here (s starts at +0.0 and a sum is -0.0 only
// if both addends are).
#ifndef LGS_SEQ_PIPE
#define LGS_SEQ_PIPE 1
#endif
constexpr int kPipeC = 4;   // double2 per chunk: 8 terms, 4 chunks per half group
__device__ __forceinline__ void pipe_load(double2 (&v)[kPipeC], const double* __restrict__ p)
{
#pragma unroll
    for (int q = 0; q < kPipeC; ++q) v[q] = *(const double2*)(p + 2 * q);
}
__device__ __forceinline__ double pipe_add(double s, const double2 (&v)[kPipeC])
{
#pragma unroll
    for (int q = 0; q < kPipeC; ++q) {
        s = s + v[q].x;
        s = s + v[q].y;
    }
    return s;
}
__device__ __forceinline__ double seq_add_staged(const double* __restrict__ row, int m, const unsigned* ready,
                                                 const int* abort, unsigned epoch)
{
#if LGS_SEQ_PIPE
    static_assert(8 * 2 * kPipeC == kGroup, "four chunks per half group");
    const int G = (m + kGroup - 1) / kGroup;
    auto wait_staged = [&](int gg) {
        while (__hip_atomic_load(&ready[gg], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) != epoch)
            if (__hip_atomic_load(abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) return false;
        return true;
    };
    double2 v0[kPipeC], v1[kPipeC], v2[kPipeC], v3[kPipeC];
    if (!wait_staged(0)) return 0.0;
    pipe_load(v0, row);
    pipe_load(v1, row + 8);
    pipe_load(v2, row + 16);
    pipe_load(v3, row + 24);
    double s = 0.0;
    for (int gg = 0; gg < G; ++gg) {
        const double* h1 = row + gg * kGroup + 32;
        __builtin_amdgcn_sched_barrier(0);
        s = pipe_add(s, v0);
        pipe_load(v0, h1);
        __builtin_amdgcn_sched_barrier(0);
        s = pipe_add(s, v1);
        pipe_load(v1, h1 + 8);
        __builtin_amdgcn_sched_barrier(0);
        s = pipe_add(s, v2);
        pipe_load(v2, h1 + 16);
        __builtin_amdgcn_sched_barrier(0);
        s = pipe_add(s, v3);
        pipe_load(v3, h1 + 24);
        // the first half's adds before the flag wait (the compiler would
        // otherwise sink them past the spin loop: they have no side effects)
        asm volatile("" : "+v"(s)::"memory");
        const bool more = gg + 1 < G;
        if (more && !wait_staged(gg + 1)) return 0.0;
        const double* n0 = more ? row + (gg + 1) * kGroup : row;   // (past the last group: a harmless reload)
        __builtin_amdgcn_sched_barrier(0);
        s = pipe_add(s, v0);
        pipe_load(v0, n0);
        __builtin_amdgcn_sched_barrier(0);
        s = pipe_add(s, v1);
        pipe_load(v1, n0 + 8);
        __builtin_amdgcn_sched_barrier(0);
        s = pipe_add(s, v2);
        pipe_load(v2, n0 + 16);
        __builtin_amdgcn_sched_barrier(0);
        s = pipe_add(s, v3);
        pipe_load(v3, n0 + 24);
        asm volatile("" : "+v"(s)::"memory");
    }
    return s;
#else
    double s = 0.0;
    for (int gg = 0; gg * kGroup < m; ++gg) {
        while (__hip_atomic_load(&ready[gg], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) != epoch)
            if (__hip_atomic_load(abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) return 0.0;
        const double* r = row + gg * kGroup;
        const int cnt = min(kGroup, m - gg * kGroup);
        if (cnt == kGroup) {
            double2 v[kGroup / 2];
#pragma unroll
            for (int q = 0; q < kGroup / 2; ++q) v[q] = *(const double2*)(r + 2 * q);
#pragma unroll
            for (int q = 0; q < kGroup / 2; ++q) {
                s = s + v[q].x;
                s = s + v[q].y;
            }
        } else {
            s = seq_add(s, r, cnt);
        }
    }
    return s;
#endif
}

__device__ __forceinline__ bool spin_expired(unsigned long long t0, unsigned long long limit)
{
    return __builtin_amdgcn_s_memrealtime() - t0 > limit;
}

__global__ __launch_bounds__(kSplitThreads) void k_linsolve_split(LsPlan p, const double* __restrict__ grid,
                                                                  LsScanRef sc, LsRecord* __restrict__ out,
                                                                  double* __restrict__ traj, gu64* __restrict__ tbuf,
                                                                  gu32* __restrict__ flags, gu32* __restrict__ tmo,
                                                                  unsigned long long spin_limit,
                                                                  unsigned long long* __restrict__ trace)
{
    __shared__ SplitLds L;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const double smin = fmax(p.step_min, sc.min_range), smax = fmin(p.step_max, sc.max_range);
    const double cmin = fmax(p.cost_min, sc.min_range), cmax = fmin(p.cost_max, sc.max_range);
    const int G = (sc.n + kGroup - 1) / kGroup;
    const int g = blockIdx.x;                      // this workgroup's group (gridDim.x == G)
    const int i = g * kGroup + lane;
    // the workgroup's beam (lane) stays in registers for every pass
    double r = 0.0, ang = 0.0;
    bool in_step = false, in_cost = false;
    if (i < sc.n) {
        r = sc.ranges[i];
        ang = sc.angles[i];
        in_step = !(r >= smax || r <= smin);
        in_cost = !(r >= cmax || r <= cmin);
    }
    const bool act = in_step || in_cost;
    if (spin_limit == 0ull) {                      // diagnostics: the host's time-out fallback
        if (threadIdx.x == 0) __hip_atomic_store(tmo, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return;
    }
    if (threadIdx.x < kSplitMaxGroups) L.ready[threadIdx.x] = 0u;
    if (threadIdx.x == 0) L.abort = 0;
    __syncthreads();
    double pose[3] = { sc.pose0[0], sc.pose0[1], sc.pose0[2] };
    double acc[kAcc];
    double prevCost = DBL_MAX, cost = DBL_MAX;
    int it = 0;
    for (int pass = 0;; ++pass) {
        const unsigned epoch = (unsigned)pass + 1u;
        gu64* tb = tbuf + (size_t)(pass & 1) * kSplitMaxGroups * kAcc * kGroup;
        gu32* fl = flags + (pass & 1) * kSplitMaxGroups;
        unsigned long long* tr = (trace && blockIdx.x == 0 && threadIdx.x == 0) ? trace + (size_t)min(pass, 127) * 32
                                                                                : nullptr;
        unsigned long long* trs = (trace && blockIdx.x == 0 && lane == 0) ? trace + (size_t)min(pass, 127) * 32 + 8
                                                                          : nullptr;
        if (tr) tr[0] = __builtin_amdgcn_s_memrealtime();
        unsigned long long* twg = (trace && threadIdx.x == 0) ? trace + 128 * 32 + (size_t)min(pass, 127) * 64 + 3 * g
                                                              : nullptr;
        if (twg) twg[0] = __builtin_amdgcn_s_memrealtime();
        // phase A: the hit point (every wave), one axis per wave 0..5
        if (act && wid < 6) {
            double sn, cs, fx, fy;
            beam_cell(p, pose, r, ang, sn, cs, fx, fy);
            const double d = kHalfDelta;
            const bool isx = !(wid & 1);
            const double v = (wid < 2) ? (isx ? fx : fy) : (wid < 4) ? (fx + ((wid == 2) ? d : -d))
                                                                     : (fy + ((wid == 4) ? d : -d));
            L.b.ax[wid][lane] = make_axis(v, (wid == 0 || wid == 2 || wid == 3) ? p.W : p.H);
            if (wid == 0) {
                L.b.sc[0][lane] = sn;
                L.b.sc[1][lane] = cs;
            }
        }
        __syncthreads();
        if (tr) tr[1] = __builtin_amdgcn_s_memrealtime();
        // phase B: one smoothed value per wave 0..4
        if (act && wid < 5) {
            const int xa = (wid == 1) ? 2 : (wid == 2) ? 3 : 0;
            const int ya = (wid == 3) ? 4 : (wid == 4) ? 5 : 1;
            L.b.sv[wid][lane] = smoothed(grid, p.W, L.b.ax[xa][lane], L.b.ax[ya][lane]);
        }
        __syncthreads();
        if (tr) tr[2] = __builtin_amdgcn_s_memrealtime();
        // phase C: wave 0 finishes the beam and publishes its 13 terms
        // write-through (sc1) with the group's flag (recipe R1)
        if (wid == 0) {
            double e = 0.0, gv[3] = { 0.0, 0.0, 0.0 };
            if (act)
                beam_finish(p, r, L.b.sc[0][lane], L.b.sc[1][lane], L.b.sv[0][lane], L.b.sv[1][lane],
                            L.b.sv[2][lane], L.b.sv[3][lane], L.b.sv[4][lane], e, gv);
            double t[kAcc];
            beam_acc(in_step, in_cost, e, gv, t);
#pragma unroll
            for (int k = 0; k < kAcc; ++k)
                __hip_atomic_store(tb + ((size_t)g * kAcc + k) * kGroup + lane,
                                   (unsigned long long)__double_as_longlong(t[k]), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            if (lane == 0) __hip_atomic_store(fl + g, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (tr) tr[3] = __builtin_amdgcn_s_memrealtime();
            if (twg) twg[1] = __builtin_amdgcn_s_memrealtime();
            // the 13 sums in beam order, group by group as the staging waves
            // deliver them (LDS flag per group)
            const double sk = (lane < kAcc) ? seq_add_staged(L.terms[lane], sc.n, L.ready, &L.abort, epoch) : 0.0;
            gather_sums(sk, acc);
            if (tr) tr[4] = __builtin_amdgcn_s_memrealtime();
            if (twg) twg[2] = __builtin_amdgcn_s_memrealtime();
        } else {
            // staging waves 1..7: group gg (gg = wid - 1, wid + 6, ...) once its
            // flag shows this pass: its 13 rows with sc1 loads (every load of
            // the handed-off terms is agent-scope, so no acquire fence;
            // Guideline 16), into the LDS rows in beam order, then the group's
            // LDS flag
            const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
            for (int gg = wid - 1; gg < G; gg += kSplitThreads / 64 - 1) {
                bool ok = true;
                for (unsigned polls = 1;; ++polls) {
                    if (__hip_atomic_load(fl + gg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == epoch) break;
                    if ((polls & 255u) == 0u &&
                        (__hip_atomic_load(tmo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u ||
                         spin_expired(t0, spin_limit))) {
                        if (lane == 0) {
                            __hip_atomic_store(tmo, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                            __hip_atomic_store(&L.abort, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                        }
                        ok = false;
                        break;
                    }
                }
                if (!ok) break;
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                unsigned long long v[kAcc];
#pragma unroll
                for (int k = 0; k < kAcc; ++k)
                    v[k] = __hip_atomic_load(tb + ((size_t)gg * kAcc + k) * kGroup + lane, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
                for (int k = 0; k < kAcc; ++k) L.terms[k][gg * kGroup + lane] = __longlong_as_double((long long)v[k]);
                // LDS ops of a wave complete in order: the rows land before the flag
                if (lane == 0) __hip_atomic_store(&L.ready[gg], epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                if (trs) trs[gg] = __builtin_amdgcn_s_memrealtime();
            }
        }
        __syncthreads();
        if (L.abort) return;
        if (wid == 0) {
            int stop = 0;
            if (pass > 0) {
                cost = acc[9];
                if (traj && g == 0 && lane == 0) {
                    double* tr = traj + (size_t)it * 4;
                    tr[0] = pose[0];
                    tr[1] = pose[1];
                    tr[2] = pose[2];
                    tr[3] = cost;
                }
                if (++it >= p.max_iter || fabs(prevCost - cost) < p.conv) stop = 1;
                prevCost = cost;
            }
            if (!stop && lane == 0) {
                // OptimizeStep (:88-148), solved by lane 0 of every workgroup
                const double H[9] = { acc[3] + p.reg_t, acc[4], acc[5],
                                      acc[4], acc[6] + p.reg_t, acc[7],
                                      acc[5], acc[7], acc[8] + p.reg_r };
                const double b[3] = { acc[0], acc[1], acc[2] };
                double dd[3];
                solve3_colpiv_qr(H, b, dd);
                L.pose[0] = pose[0] + dd[0];
                L.pose[1] = pose[1] + dd[1];
                L.pose[2] = pose[2] + dd[2];
            }
            if (lane == 0) L.stop = stop;
            if (tr) tr[7] = __builtin_amdgcn_s_memrealtime();
        }
        __syncthreads();
        const int stop = L.stop;
        if (stop) break;
        pose[0] = L.pose[0];
        pose[1] = L.pose[1];
        pose[2] = L.pose[2];
        __syncthreads();
    }
    if (g == 0 && threadIdx.x == 0) {
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
    __shared__ LsLds L;
    const double cmin = fmax(p.cost_min, sc.min_range), cmax = fmin(p.cost_max, sc.max_range);
    double acc[kAcc];
    // step filter empty: only the cost-side sums are accumulated
    gather_sums(seq_pass(p, grid, sc, sc.pose0, 0.0, 0.0, cmin, cmax, L), acc);
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
    grid_acquire(ctx, grid);
    check_grid(grid);
    LGS_REQUIRE(prm, "null params");
    LGS_HIP_CHECK(hipSetDevice(ctx->device));
    const LsPlan p = make_ls_plan(grid, prm);
    const int iters = std::max(1, p.max_iter);
    std::vector<LsScanRef> refs(n);
    for (int j = 0; j < n; ++j) LGS_REQUIRE(scans[j] && scans[j]->n >= 1, "empty scan");
    scans_to_device(ctx, scans, n);
    for (int j = 0; j < n; ++j) {
        refs[j] = scan_ref(scans[j], init[j]);
    }
    // pinned staging: [refs | records | trajectory]
    const size_t b_refs = sizeof(LsScanRef) * n, b_rec = sizeof(LsRecord) * n;
    const size_t b_traj = traj ? sizeof(double) * 4 * (size_t)iters * n : 0;
    char* h = (char*)ctx->ensure_pinned(b_refs + b_rec + b_traj + 16);   // + the split refine's timeout word
    std::memcpy(h, refs.data(), b_refs);
    char* d = (char*)ctx->ensure(S_LIN0, b_refs + b_rec + b_traj);
    LGS_HIP_CHECK(hipMemcpyAsync(d, h, b_refs, hipMemcpyHostToDevice, ctx->stream));
    // a lone refine of at most kSplitMaxGroups groups runs split over one
    // workgroup per group when the device can hold all of them at once
    const int groups = (refs[0].n + kGroup - 1) / kGroup;
    bool split = n == 1 && ctx->linsolve_split && groups <= kSplitMaxGroups && groups > 1;
    if (split) {
        // workgroups the device holds at once, per device (filled once under a lock)
        static std::mutex mu;
        static int cap[64] = {};
        int c = 0;
        if (ctx->device >= 0 && ctx->device < 64) {
            std::lock_guard<std::mutex> g(mu);
            if (!cap[ctx->device]) {
                int cus = 0, per_cu = 0;
                LGS_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, ctx->device));
                LGS_HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_linsolve_split, kSplitThreads, 0));
                cap[ctx->device] = std::max(1, per_cu * cus);
            }
            c = cap[ctx->device];
        }
        split = c >= groups;
    }
    // split hand-off state: [flags (2 x kSplitMaxGroups) | timeout word | pad] then the terms
    constexpr size_t b_flags = 16 * ((sizeof(unsigned) * (2 * kSplitMaxGroups + 1) + 15) / 16);
    constexpr size_t b_terms = sizeof(double) * 2 * kSplitMaxGroups * kAcc * kGroup;
    char* hs = split ? (char*)ctx->ensure(S_LIN2, b_flags + b_terms) : nullptr;
    unsigned* htmo = (unsigned*)(h + b_refs + b_rec + b_traj);
    // diagnostics: LGS_LS_TRACE=1 prints the split refine's per-pass phase
    // stamps of workgroup 0 (us after the pass start: axes, smoothed values,
    // published, summed (-1), (-1), solved | next pass)
    static const bool trace_on = getenv("LGS_LS_TRACE") != nullptr;
    unsigned long long* trace_dev = nullptr;
    if (split && trace_on) {
        trace_dev = (unsigned long long*)ctx->ensure(S_LIN3, 128 * 96 * sizeof(unsigned long long));
        LGS_HIP_CHECK(hipMemsetAsync(trace_dev, 0, 128 * 96 * sizeof(unsigned long long), ctx->stream));
    }
    *htmo = 0u;
    const auto launch_one_wg = [&] {
        hipLaunchKernelGGL(k_linsolve, dim3(n), dim3(kLsThreads), 0, ctx->stream, p, grid->d, (const LsScanRef*)d,
                           (LsRecord*)(d + b_refs), traj ? (double*)(d + b_refs + b_rec) : nullptr);
    };
    const int tok = ctx->timing_begin(K_LINSOLVE, 0.0);
    if (split) {
        LGS_HIP_CHECK(hipMemsetAsync(hs, 0, b_flags, ctx->stream));   // flags + timeout word, every call
        hipLaunchKernelGGL(k_linsolve_split, dim3(groups), dim3(kSplitThreads), 0, ctx->stream, p, grid->d, refs[0],
                           (LsRecord*)(d + b_refs), traj ? (double*)(d + b_refs + b_rec) : nullptr,
                           (gu64*)(hs + b_flags), (gu32*)hs, (gu32*)(hs + sizeof(unsigned) * 2 * kSplitMaxGroups),
                           (unsigned long long)ctx->handoff_spin_us * 100ull,    // s_memrealtime: 100 MHz
                           trace_dev);
    } else {
        launch_one_wg();
    }
    ctx->timing_end(tok);
    LGS_HIP_CHECK(hipGetLastError());
    if (split)
        LGS_HIP_CHECK(hipMemcpyAsync(htmo, hs + sizeof(unsigned) * 2 * kSplitMaxGroups, sizeof(unsigned),
                                     hipMemcpyDeviceToHost, ctx->stream));
    LGS_HIP_CHECK(hipMemcpyAsync(h + b_refs, d + b_refs, b_rec + b_traj, hipMemcpyDeviceToHost,
                                 ctx->stream));
    ctx->sync();
    if (split && *htmo != 0u) {
        // the split refine's workgroups were not all resident (time-out): the
        // one-workgroup kernel computes the same bits
        ++ctx->handoff_fallbacks;
        launch_one_wg();
        LGS_HIP_CHECK(hipGetLastError());
        LGS_HIP_CHECK(hipMemcpyAsync(h + b_refs, d + b_refs, b_rec + b_traj, hipMemcpyDeviceToHost,
                                     ctx->stream));
        ctx->sync();
    }
    if (ctx->profile) ctx->harvest();
    if (trace_dev) {
        std::vector<unsigned long long> t(128 * 96);
        LGS_HIP_CHECK(hipMemcpy(t.data(), trace_dev, t.size() * sizeof(t[0]), hipMemcpyDeviceToHost));
        for (int q = 0; q < 128 && t[q * 32]; ++q) {
            const unsigned long long* u = &t[q * 32];
            fprintf(stderr, "LSTRACE pass %d:", q);
            for (int k = 1; k < 8; ++k) fprintf(stderr, " %.2f", u[k] ? 0.01 * (double)(u[k] - u[0]) : -1.0);
            if (q + 1 < 128 && t[(q + 1) * 32]) fprintf(stderr, " | next %.2f", 0.01 * (double)(t[(q + 1) * 32] - u[0]));
            fprintf(stderr, " | staged");
            for (int k = 8; k < 28 && u[k]; ++k) fprintf(stderr, " %.2f", 0.01 * (double)(u[k] - u[0]));
            fprintf(stderr, "\n");
            fprintf(stderr, "LSWG pass %d (start publish summed per workgroup, us after wg 0's start):", q);
            const unsigned long long* w = &t[128 * 32 + q * 64];
            for (int k = 0; k < groups; ++k)
                fprintf(stderr, " [%d %.2f %.2f %.2f]", k, 0.01 * ((double)w[3 * k] - (double)u[0]),
                        0.01 * ((double)w[3 * k + 1] - (double)u[0]), 0.01 * ((double)w[3 * k + 2] - (double)u[0]));
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
        grid_acquire(ctx, grid);
        lgs_linsolve_params prm{};
        prm.cost_usable_range_min = umin;
        prm.cost_usable_range_max = umax;
        const LsPlan p = make_ls_plan(grid, &prm);
        scan_to_device(ctx, scan);
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

namespace {
__global__ void k_debug_libm(int op, const double* __restrict__ x, int n, double* __restrict__ out)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    if (op == 0) {
        double s, c;
        glm::gl_sincos(x[i], &s, &c);
        out[2 * i] = s;
        out[2 * i + 1] = c;
    } else {
        out[i] = glm::gl_pow3(x[i]);
    }
}
}  // namespace

extern "C" int lgs_debug_libm(lgs_ctx* ctx, int op, const double* x, int n, double* out)
{
    if (!ctx || !x || !out || n < 0 || (op != 0 && op != 1)) return LGS_ERR_INVALID_ARG;
    if (n == 0) return LGS_OK;
    return guarded(ctx, [&] {
        LGS_HIP_CHECK(hipSetDevice(ctx->device));
        const size_t bin = sizeof(double) * n, bout = bin * (op == 0 ? 2 : 1);
        char* d = (char*)ctx->ensure(S_LIN1, bin + bout);
        LGS_HIP_CHECK(hipMemcpyAsync(d, x, bin, hipMemcpyHostToDevice, ctx->stream));
        hipLaunchKernelGGL(k_debug_libm, dim3((n + 255) / 256), dim3(256), 0, ctx->stream, op, (const double*)d, n,
                           (double*)(d + bin));
        LGS_HIP_CHECK(hipGetLastError());
        LGS_HIP_CHECK(hipMemcpyAsync(out, d + bin, bout, hipMemcpyDeviceToHost, ctx->stream));
        ctx->sync();
    });
}
