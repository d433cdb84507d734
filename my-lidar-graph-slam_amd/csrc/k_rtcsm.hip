// k_rtcsm.hip -- K1: exhaustive correlative scan matcher on MI355X.
//
// Restates ScanMatcherRealTimeCorrelative::OptimizePose
// (C/mapping/scan_matcher_real_time_correlative.cpp:50-145) with a search order
// built for the GPU and a result proven identical to the reference's
// sequential, pruned loop (DESIGN.md §K1 "exact pruning"):
//
//   k_project   ComputeScanIndices (:178-203) for every search angle at once;
//               fp64 with -ffp-contract=off; projections within guard_eps of a
//               cell boundary are reported and re-checked on the host with glibc.
//   k_coarse    ComputeScore (:207-224) on the coarse map for every coarse
//               block (t, xc, yc): one lane per block, beams walked in order so
//               each score is the reference's sequential fp64 sum.  Also flags
//               "unsafe" blocks where the coarse score may not bound the fine
//               scores (coarse reads left/below the map return 0 while fine
//               reads can land inside).
//   k_seed      lower bound L = fine max of the best safe coarse block.
//   k_select    blocks that can influence the reference's result:
//               (c > thr) && (unsafe || c >= L)  -> ordered list (hipcub).
//   k_fine      EvaluateHighResolutionMap (:227-256) for listed blocks: block
//               max and its first position in the reference's (x, y) order.
//   k_replay    the reference's acceptance rule `c > s && f > s` replayed in
//               block order over the list; detects the one case the pruning
//               proof does not cover (unsafe block with c < L <= f) and asks
//               the host for an exact dense rerun.
//   k_cost_*    CostGreedyEndpoint::Cost at the best pose and its six
//               central-difference neighbours (C/mapping/cost_function_greedy_endpoint.cpp:32-171).
#include "lgs_internal.hpp"

#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cfloat>
#include <cstring>

using namespace lgs;

namespace lgs {
void launch_precompute(lgs_ctx* ctx, const lgs_grid* in, int win, double* out);
}

namespace {

constexpr int kCoarseBlock = 256;

__device__ __forceinline__ bool near_boundary(double q, double eps)
{
    const double f = q - floor(q);
    const double e = eps + fabs(q) * 1e-13;
    return f < e || f > 1.0 - e;
}

// --------------------------------------------------------------------------
// k_project: idx[t][v] = WorldCoordinateToGridCellIndex(HitPoint(pose_t, beam))
// --------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_project(RtcsmPlan pl, const double* __restrict__ ranges,
                                                 const double* __restrict__ angles,
                                                 const int* __restrict__ vidx,
                                                 int2* __restrict__ idx, RtcsmRecord* rec,
                                                 int guard_cap, double guard_eps, int inject)
{
    const int v = blockIdx.x * blockDim.x + threadIdx.x;
    const int tt = blockIdx.y;
    if (v >= pl.Nv) return;
    const int i = vidx[v];
    const double r = ranges[i];
    const double a = angles[i];
    const int t = tt - pl.win_t;
    // currentSensorPose.mTheta = sensorPose.mTheta + stepTheta * t (:90-91)
    const double th = pl.st + pl.step_t * (double)t;
    // HitPoint: cos(sensorPose.mTheta + scanAngle) (H/sensor/sensor_data.hpp:168-172)
    const double c = cos(th + a);
    const double s = sin(th + a);
    const double hx = pl.sx + r * c;
    const double hy = pl.sy + r * s;
    const double qx = (hx - pl.min_x) / pl.res;
    const double qy = (hy - pl.min_y) / pl.res;
    int ix = (int)floor(qx);
    int iy = (int)floor(qy);
    if (near_boundary(qx, guard_eps) || near_boundary(qy, guard_eps)) {
        const int slot = atomicAdd(&rec->guard_count, 1);
        if (slot < guard_cap) {
            GuardRec g;
            g.t = tt;
            g.v = v;
            g.ix = ix + inject;
            g.iy = iy;
            rec->guard[slot] = g;
        }
        ix += inject;
    }
    idx[(size_t)tt * pl.Nv + v] = make_int2(ix, iy);
}

__global__ void k_patch(RtcsmPlan pl, int2* __restrict__ idx, const int4* __restrict__ patches,
                        int n)
{
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    const int4 p = patches[k];
    idx[(size_t)p.x * pl.Nv + p.y] = make_int2(p.z, p.w);
}

__global__ void k_cost_patch(int4* __restrict__ cidx, const int4* __restrict__ pairs, int n)
{
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    cidx[pairs[2 * k].x] = pairs[2 * k + 1];
}

// --------------------------------------------------------------------------
// wave/block argmax helpers: max value, ties -> smallest key
// --------------------------------------------------------------------------
__device__ __forceinline__ bool better(double a, long long ka, double b, long long kb)
{
    return (a > b) || (a == b && ka < kb);
}

__device__ void block_argmax(double& v, long long& k, double* sv, long long* sk)
{
    // wave64 butterfly
    for (int off = 32; off > 0; off >>= 1) {
        const double ov = __shfl_xor(v, off, 64);
        const long long ok = __shfl_xor(k, off, 64);
        if (better(ov, ok, v, k)) {
            v = ov;
            k = ok;
        }
    }
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int nw = (blockDim.x + 63) >> 6;
    __syncthreads();
    if (lane == 0) {
        sv[wid] = v;
        sk[wid] = k;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < nw; ++w)
            if (better(sv[w], sk[w], v, k)) {
                v = sv[w];
                k = sk[w];
            }
        sv[0] = v;
        sk[0] = k;
    }
    __syncthreads();
    v = sv[0];
    k = sk[0];
}

// --------------------------------------------------------------------------
// k_coarse: one lane per coarse block (t, jx, jy); lanes of a wave share t
// and sweep jx fastest, so the gathered cells of one beam are 5 cells apart.
// --------------------------------------------------------------------------
__global__ __launch_bounds__(kCoarseBlock) void k_coarse(
    RtcsmPlan pl, const double* __restrict__ cgrid, const int2* __restrict__ idx,
    double* __restrict__ cscore, uint8_t* __restrict__ cflag, double* __restrict__ part_c,
    long long* __restrict__ part_k)
{
    __shared__ double sv[kCoarseBlock / 64];
    __shared__ long long sk[kCoarseBlock / 64];
    const int tt = blockIdx.y;
    const int p = blockIdx.x * kCoarseBlock + threadIdx.x;
    const bool active = p < pl.P;
    const int jx = active ? p % pl.ncx : 0;
    const int jy = active ? p / pl.ncx : 0;
    const int xc = -pl.win_x + jx * pl.low_res;
    const int yc = -pl.win_y + jy * pl.low_res;
    const int W = pl.W, H = pl.H;
    const int lo = -(pl.low_res - 1);
    const int xmin = -pl.win_x, ymin = -pl.win_y;
    const int2* __restrict__ id = idx + (size_t)tt * pl.Nv;

    double sum = 0.0;
    bool unsafe = false;
#pragma unroll 8
    for (int v = 0; v < pl.Nv; ++v) {
        const int2 q = id[v];
        const int x = q.x + xc;
        const int y = q.y + yc;
        const bool inb = ((unsigned)x < (unsigned)W) & ((unsigned)y < (unsigned)H);
        const size_t off = inb ? (size_t)y * (size_t)W + (size_t)x : 0;
        const double val = cgrid[off];
        sum += inb ? val : 0.0;
        if (q.x + xmin < 0 || q.y + ymin < 0)  // wave-uniform pre-check
            unsafe |= (x >= lo) & (x < W) & (y >= lo) & (y < H) & ((x < 0) | (y < 0));
    }
    const long long k = (long long)tt * pl.P + (long long)jx * pl.ncy + jy;
    if (active) {
        cscore[k] = sum;
        cflag[k] = unsafe ? 1 : 0;
    }
    double bv = (active && !unsafe) ? sum : -1.0;
    long long bk = (active && !unsafe) ? k : LLONG_MAX;
    block_argmax(bv, bk, sv, sk);
    if (threadIdx.x == 0) {
        const int part = blockIdx.y * gridDim.x + blockIdx.x;
        part_c[part] = bv;
        part_k[part] = bk;
    }
}

// Fine scores of one block for lanes q in [0, lr*lr): lane q -> (xo = q % lr,
// yo = q / lr); reference order index o = xo*lr + yo (x outer, y inner, :239-240).
__device__ __forceinline__ double fine_score(const RtcsmPlan& pl, const double* __restrict__ grid,
                                             const int2* __restrict__ id, int xf, int yf)
{
    const int W = pl.W, H = pl.H;
    double sum = 0.0;
#pragma unroll 8
    for (int v = 0; v < pl.Nv; ++v) {
        const int2 q = id[v];
        const int x = q.x + xf;
        const int y = q.y + yf;
        const bool inb = ((unsigned)x < (unsigned)W) & ((unsigned)y < (unsigned)H);
        const size_t off = inb ? (size_t)y * (size_t)W + (size_t)x : 0;
        const double val = grid[off];
        sum += inb ? val : 0.0;
    }
    return sum;
}

__device__ void eval_block(const RtcsmPlan& pl, const double* __restrict__ grid,
                           const int2* __restrict__ idx, long long k, double* sv,
                           long long* sk, double& f, int& pos)
{
    const int tt = (int)(k / pl.P);
    const int rem = (int)(k % pl.P);
    const int jx = rem / pl.ncy, jy = rem % pl.ncy;
    const int xc = -pl.win_x + jx * pl.low_res;
    const int yc = -pl.win_y + jy * pl.low_res;
    const int lr = pl.low_res;
    const int2* __restrict__ id = idx + (size_t)tt * pl.Nv;
    double bv = -1.0;
    long long bo = LLONG_MAX;
    for (int q = threadIdx.x; q < lr * lr; q += blockDim.x) {
        const int xo = q % lr, yo = q / lr;
        const double s = fine_score(pl, grid, id, xc + xo, yc + yo);
        const long long o = (long long)xo * lr + yo;
        if (better(s, o, bv, bo)) {
            bv = s;
            bo = o;
        }
    }
    block_argmax(bv, bo, sv, sk);
    f = bv;
    pos = (int)bo;
}

// k_seed: best safe coarse block -> its fine max is a lower bound of the
// final score (every safe block's fine max is <= the reference's final score).
__global__ __launch_bounds__(256) void k_seed(RtcsmPlan pl, const double* __restrict__ grid,
                                              const int2* __restrict__ idx,
                                              const double* __restrict__ part_c,
                                              const long long* __restrict__ part_k, int nparts,
                                              double* __restrict__ Lout, int force_dense)
{
    __shared__ double sv[4];
    __shared__ long long sk[4];
    double bv = -1.0;
    long long bk = LLONG_MAX;
    for (int i = threadIdx.x; i < nparts; i += blockDim.x)
        if (better(part_c[i], part_k[i], bv, bk)) {
            bv = part_c[i];
            bk = part_k[i];
        }
    block_argmax(bv, bk, sv, sk);
    if (force_dense) {
        if (threadIdx.x == 0) *Lout = -INFINITY;
        return;
    }
    if (bk == LLONG_MAX || !(bv > pl.thr)) {
        // no safe block can ever be accepted
        if (threadIdx.x == 0) *Lout = INFINITY;
        return;
    }
    double f;
    int pos;
    eval_block(pl, grid, idx, bk, sv, sk, f, pos);
    if (threadIdx.x == 0) *Lout = f;
}

__global__ void k_select(RtcsmPlan pl, const double* __restrict__ cscore,
                         const uint8_t* __restrict__ cflag, const double* __restrict__ Lp,
                         uint8_t* __restrict__ sel)
{
    const long long k = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= pl.K) return;
    const double L = *Lp;
    const double c = cscore[k];
    sel[k] = (c > pl.thr) && (cflag[k] || c >= L) ? 1 : 0;
}

__global__ __launch_bounds__(64) void k_fine(RtcsmPlan pl, const double* __restrict__ grid,
                                             const int2* __restrict__ idx,
                                             const int* __restrict__ list,
                                             const int* __restrict__ count,
                                             double* __restrict__ fval, int* __restrict__ fpos)
{
    __shared__ double sv[1];
    __shared__ long long sk[1];
    const int n = *count;
    for (int b = blockIdx.x; b < n; b += gridDim.x) {
        double f;
        int pos;
        eval_block(pl, grid, idx, list[b], sv, sk, f, pos);
        if (threadIdx.x == 0) {
            fval[b] = f;
            fpos[b] = pos;
        }
        __syncthreads();
    }
}

// k_replay: the reference's sequential acceptance over the ordered list
// (:98-114 with the strict update of :246), then the 7 cost poses.
__global__ void k_replay(RtcsmPlan pl, const double* __restrict__ cscore,
                         const uint8_t* __restrict__ cflag, const int* __restrict__ list,
                         const int* __restrict__ count, const double* __restrict__ fval,
                         const int* __restrict__ fpos, const double* __restrict__ Lp,
                         RtcsmRecord* rec, double* __restrict__ poses7)
{
    if (threadIdx.x != 0) return;
    const int n = *count;
    const double L = *Lp;
    double s = pl.thr;
    int bx = -pl.win_x, by = -pl.win_y, bt = -pl.win_t;
    int status = 0;
    for (int b = 0; b < n; ++b) {
        const long long k = list[b];
        const double c = cscore[k];
        const double f = fval[b];
        if (cflag[k] && c < L && f >= L) status |= REC_DANGEROUS;
        if (c > s && f > s) {
            s = f;
            const int tt = (int)(k / pl.P);
            const int rem = (int)(k % pl.P);
            const int jx = rem / pl.ncy, jy = rem % pl.ncy;
            const int o = fpos[b];
            bx = -pl.win_x + jx * pl.low_res + o / pl.low_res;
            by = -pl.win_y + jy * pl.low_res + o % pl.low_res;
            bt = tt - pl.win_t;
        }
    }
    rec->status = status;
    rec->found = s > pl.thr;
    rec->n_eval = n;
    rec->best[0] = bx;
    rec->best[1] = by;
    rec->best[2] = bt;
    rec->score_max = s;
    rec->L = L;
    // bestSensorPose (:122-125) and the central-difference poses of
    // CostGreedyEndpoint::ComputeGradient (C/mapping/cost_function_greedy_endpoint.cpp:119-136)
    const double x = pl.sx + bx * pl.step_x;
    const double y = pl.sy + by * pl.step_y;
    const double th = pl.st + bt * pl.step_t;
    const double dl = pl.res, da = 1e-2;
    const double P7[7][3] = {
        { x, y, th },
        { x + dl, y + 0.0, th + 0.0 }, { x - dl, y - 0.0, th - 0.0 },
        { x + 0.0, y + dl, th + 0.0 }, { x - 0.0, y - dl, th - 0.0 },
        { x + 0.0, y + 0.0, th + da }, { x - 0.0, y - 0.0, th - da },
    };
    for (int i = 0; i < 7; ++i)
        for (int j = 0; j < 3; ++j) poses7[3 * i + j] = P7[i][j];
}

// --------------------------------------------------------------------------
// greedy-endpoint cost: cell indices per (pose, beam), then per-pose terms
// summed sequentially in beam order (the reference's `costValue -= exp(..)`).
// --------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_cost_idx(CostPlan cp, const double* __restrict__ ranges,
                                                  const double* __restrict__ angles,
                                                  const double* __restrict__ poses,
                                                  int4* __restrict__ cidx, RtcsmRecord* rec,
                                                  int guard_cap, double guard_eps, int inject)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const int pi = blockIdx.y;
    if (i >= cp.N) return;
    const double r = ranges[i];
    int4 out = make_int4(INT_MIN, 0, 0, 0);
    if (!(r >= cp.max_range || r <= cp.min_range)) {
        const double px = poses[3 * pi], py = poses[3 * pi + 1], pt = poses[3 * pi + 2];
        const double c = cos(pt + angles[i]);
        const double s = sin(pt + angles[i]);
        const double q[4] = {
            (px + r * c - cp.min_x) / cp.res,
            (py + r * s - cp.min_y) / cp.res,
            (px + (r - cp.hit_and_missed_dist) * c - cp.min_x) / cp.res,
            (py + (r - cp.hit_and_missed_dist) * s - cp.min_y) / cp.res,
        };
        int cell[4];
        for (int j = 0; j < 4; ++j) {
            cell[j] = (int)floor(q[j]);
            if (near_boundary(q[j], guard_eps)) {
                cell[j] += inject;
                const int slot = atomicAdd(&rec->cost_guard_count, 1);
                if (slot < guard_cap) {
                    CostGuardRec g;
                    g.pose_which = pi * 4 + j;
                    g.beam = i;
                    g.ix = cell[j];
                    g.iy = 0;
                    rec->cost_guard[slot] = g;
                }
            }
        }
        out = make_int4(cell[0], cell[1], cell[2], cell[3]);
    }
    cidx[(size_t)pi * cp.N + i] = out;
}

__device__ __forceinline__ double gval(const CostPlan& cp, const double* __restrict__ g, int x,
                                       int y)
{
    const bool inb = ((unsigned)x < (unsigned)cp.W) & ((unsigned)y < (unsigned)cp.H);
    return inb ? g[(size_t)y * cp.W + x] : 0.0;
}

__global__ __launch_bounds__(256) void k_cost_eval(CostPlan cp, const double* __restrict__ grid,
                                                   const int4* __restrict__ cidx,
                                                   double* __restrict__ terms,
                                                   double* __restrict__ costs_out)
{
    const int pi = blockIdx.x;
    const int4* __restrict__ ci = cidx + (size_t)pi * cp.N;
    double* __restrict__ tm = terms + (size_t)pi * cp.N;
    const int K = cp.kernel_size;
    const double lim = (K + 1) * cp.res;
    const double minSq0 = lim * lim + lim * lim;
    for (int i = threadIdx.x; i < cp.N; i += blockDim.x) {
        const int4 c = ci[i];
        if (c.x == INT_MIN) continue;
        double minSq = minSq0;
        for (int ky = -K; ky <= K; ++ky)
            for (int kx = -K; kx <= K; ++kx) {
                const double hv = gval(cp, grid, c.x + kx, c.y + ky);
                const double mv = gval(cp, grid, c.z + kx, c.w + ky);
                if (hv == 0.0 || mv == 0.0) continue;
                if (hv < cp.occupancy_threshold || mv > cp.occupancy_threshold) continue;
                const double dX = kx * cp.res;
                const double dY = ky * cp.res;
                const double sq = dX * dX + dY * dY;
                minSq = (minSq < sq) ? minSq : sq;
            }
        tm[i] = exp(-0.5 * minSq / cp.variance);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        double cost = 0.0;
        for (int i = 0; i < cp.N; ++i)
            if (ci[i].x != INT_MIN) cost -= tm[i];
        cost *= cp.scaling_factor;
        costs_out[pi] = cost;
    }
}

// --------------------------------------------------------------------------
// dense diagnostics: every fine score of the window
// --------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_fine_dense(RtcsmPlan pl, const double* __restrict__ grid,
                                                    const int2* __restrict__ idx, int nfx,
                                                    int nfy, double* __restrict__ out)
{
    const int tt = blockIdx.y;
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= nfx * nfy) return;
    const int fx = p % nfx, fy = p / nfx;
    const double s = fine_score(pl, grid, idx + (size_t)tt * pl.Nv, -pl.win_x + fx, -pl.win_y + fy);
    out[((size_t)tt * nfx + fx) * nfy + fy] = s;
}

// --------------------------------------------------------------------------
// host orchestration
// --------------------------------------------------------------------------
RtcsmPlan make_plan(const lgs_grid* grid, const lgs_rtcsm_params* p, const lgs_scan* scan,
                    lgs_pose2d initial, double nthr, int nv)
{
    RtcsmPlan pl{};
    // :58-59
    const lgs_pose2d sp = compound(initial, scan->rel);
    pl.sx = sp.x;
    pl.sy = sp.y;
    pl.st = sp.theta;
    // ComputeSearchStep (:156-175)
    const double maxRange = std::min(scan->max_elem, p->scan_range_max);
    const double theta = grid->res / maxRange;
    pl.step_x = grid->res;
    pl.step_y = grid->res;
    pl.step_t = std::acos(1.0 - 0.5 * theta * theta);
    // :69-74
    pl.win_x = (int)std::ceil(0.5 * p->range_x / pl.step_x);
    pl.win_y = (int)std::ceil(0.5 * p->range_y / pl.step_y);
    pl.win_t = (int)std::ceil(0.5 * p->range_theta / pl.step_t);
    // :77-78
    pl.thr = nthr * (double)scan->n;
    pl.min_x = grid->min_x;
    pl.min_y = grid->min_y;
    pl.res = grid->res;
    pl.W = grid->w;
    pl.H = grid->h;
    pl.low_res = p->low_resolution;
    pl.T = 2 * pl.win_t + 1;
    pl.ncx = (2 * pl.win_x) / pl.low_res + 1;
    pl.ncy = (2 * pl.win_y) / pl.low_res + 1;
    pl.P = pl.ncx * pl.ncy;
    pl.K = (long long)pl.T * pl.P;
    pl.Nv = nv;
    pl.N = scan->n;
    return pl;
}

CostPlan make_cost_plan(const lgs_grid* grid, const lgs_cost_ge_params* c, const lgs_scan* s)
{
    CostPlan cp{};
    cp.min_range = std::max(c->usable_range_min, s->min_range);
    cp.max_range = std::min(c->usable_range_max, s->max_range);
    cp.hit_and_missed_dist = c->hit_and_missed_dist;
    cp.occupancy_threshold = c->occupancy_threshold;
    cp.variance = c->standard_deviation * c->standard_deviation;
    cp.scaling_factor = c->scaling_factor;
    cp.min_x = grid->min_x;
    cp.min_y = grid->min_y;
    cp.res = grid->res;
    cp.W = grid->w;
    cp.H = grid->h;
    cp.kernel_size = c->kernel_size;
    cp.N = s->n;
    return cp;
}

struct Workspace {
    int2* idx;
    double* cscore;
    uint8_t* cflag;
    uint8_t* sel;
    int* list;
    double* fval;
    int* fpos;
    double* part_c;
    long long* part_k;
    int* count;  // [0] = list count
    double* Lp;
    double* poses7;
    int4* cidx;
    double* terms;
    void* cub_temp;
    size_t cub_bytes;
    int nparts;
};

Workspace ensure_workspace(lgs_ctx* ctx, const RtcsmPlan& pl, int N)
{
    Workspace w{};
    const int tiles = (pl.P + kCoarseBlock - 1) / kCoarseBlock;
    w.nparts = tiles * pl.T;
    const size_t K = (size_t)pl.K;
    w.idx = (int2*)ctx->ensure(S_IDX, sizeof(int2) * (size_t)pl.T * std::max(pl.Nv, 1));
    w.cscore = (double*)ctx->ensure(S_CSCORE, sizeof(double) * K);
    w.cflag = (uint8_t*)ctx->ensure(S_CFLAG, K);
    w.sel = (uint8_t*)ctx->ensure(S_SEL, K);
    w.list = (int*)ctx->ensure(S_LIST, sizeof(int) * K);
    w.fval = (double*)ctx->ensure(S_FVAL, sizeof(double) * K);
    w.fpos = (int*)ctx->ensure(S_FPOS, sizeof(int) * K);
    w.part_c = (double*)ctx->ensure(S_PART_C, sizeof(double) * (size_t)w.nparts);
    w.part_k = (long long*)ctx->ensure(S_PART_K, sizeof(long long) * (size_t)w.nparts);
    char* cnt = (char*)ctx->ensure(S_COUNT, 64);
    w.count = (int*)cnt;
    w.Lp = (double*)(cnt + 16);
    w.poses7 = (double*)ctx->ensure(S_POSES7, sizeof(double) * 21);
    w.cidx = (int4*)ctx->ensure(S_COST_IDX, sizeof(int4) * 7 * (size_t)N);
    w.terms = (double*)ctx->ensure(S_COST_TERM, sizeof(double) * 7 * (size_t)N);
    size_t bytes = 0;
    LGS_HIP_CHECK(hipcub::DeviceSelect::Flagged(nullptr, bytes, hipcub::CountingInputIterator<int>(0),
                                                w.sel, w.list, w.count, (int)K, ctx->stream));
    w.cub_temp = ctx->ensure(S_CUB_TEMP, bytes);
    w.cub_bytes = bytes;
    return w;
}

struct ScanOptions {
    bool dense = false;
    const std::vector<int4>* patches = nullptr;    // projection patches (t, v, ix, iy)
    const std::vector<int2>* host_idx = nullptr;   // full host projection [T*Nv]
    const std::vector<int4>* cost_patches = nullptr;
};

// Enqueue the whole device pipeline of one match on ctx->stream.
void enqueue_match(lgs_ctx* ctx, const lgs_grid* grid, const lgs_grid* coarse,
                   const lgs_cost_ge_params* cost, lgs_scan* scan, const RtcsmPlan& pl,
                   const int* d_vidx, RtcsmRecord* d_rec, const ScanOptions& opt)
{
    Workspace w = ensure_workspace(ctx, pl, scan->n);
    hipStream_t st = ctx->stream;
    LGS_HIP_CHECK(hipMemsetAsync(d_rec, 0, sizeof(RtcsmRecord), st));
    const int inject = ctx->inject_index ? 1 : 0;
    if (pl.Nv > 0) {
        if (opt.host_idx) {
            LGS_HIP_CHECK(hipMemcpyAsync(w.idx, opt.host_idx->data(), sizeof(int2) * opt.host_idx->size(),
                                         hipMemcpyHostToDevice, st));
        } else {
            dim3 g((pl.Nv + 255) / 256, pl.T);
            {
                const int tok_ = ctx->timing_begin(K_PROJECT, 16.0 * (double)pl.T * pl.Nv);
                hipLaunchKernelGGL(k_project, g, dim3(256), 0, st, pl, scan->d_ranges, scan->d_angles,
                                   d_vidx, w.idx, d_rec, ctx->guard_cap, ctx->guard_eps, inject);
                ctx->timing_end(tok_);
            }
            LGS_HIP_CHECK(hipGetLastError());
            if (opt.patches && !opt.patches->empty()) {
                int4* dp = (int4*)ctx->ensure(S_PATCH, sizeof(int4) * opt.patches->size());
                LGS_HIP_CHECK(hipMemcpyAsync(dp, opt.patches->data(), sizeof(int4) * opt.patches->size(),
                                             hipMemcpyHostToDevice, st));
                const int np = (int)opt.patches->size();
                hipLaunchKernelGGL(k_patch, dim3((np + 255) / 256), dim3(256), 0, st, pl, w.idx, dp, np);
                LGS_HIP_CHECK(hipGetLastError());
            }
        }
    }
    {
        dim3 g((pl.P + kCoarseBlock - 1) / kCoarseBlock, pl.T);
        {
            const int tok_ = ctx->timing_begin(K_COARSE, 8.0 * (double)pl.K * pl.Nv);
            hipLaunchKernelGGL(k_coarse, g, dim3(kCoarseBlock), 0, st, pl, coarse->d, w.idx, w.cscore,
                               w.cflag, w.part_c, w.part_k);
            ctx->timing_end(tok_);
        }
        LGS_HIP_CHECK(hipGetLastError());
    }
    {
        const int tok_ = ctx->timing_begin(K_SEED, 8.0 * pl.low_res * pl.low_res * (double)pl.Nv);
        hipLaunchKernelGGL(k_seed, dim3(1), dim3(256), 0, st, pl, grid->d, w.idx, w.part_c, w.part_k,
                           w.nparts, w.Lp, (opt.dense || ctx->force_dense) ? 1 : 0);
        ctx->timing_end(tok_);
    }
    LGS_HIP_CHECK(hipGetLastError());
    {
        const int tok_ = ctx->timing_begin(K_SELECT, 10.0 * (double)pl.K);
        hipLaunchKernelGGL(k_select, dim3((unsigned)((pl.K + 255) / 256)), dim3(256), 0, st, pl, w.cscore,
                           w.cflag, w.Lp, w.sel);
        ctx->timing_end(tok_);
    }
    LGS_HIP_CHECK(hipGetLastError());
    size_t bytes = w.cub_bytes;
    LGS_HIP_CHECK(hipcub::DeviceSelect::Flagged(w.cub_temp, bytes, hipcub::CountingInputIterator<int>(0),
                                                w.sel, w.list, w.count, (int)pl.K, st));
    {
        const int tok_ = ctx->timing_begin(K_FINE, 0.0);
        hipLaunchKernelGGL(k_fine, dim3(2048), dim3(64), 0, st, pl, grid->d, w.idx, w.list, w.count,
                           w.fval, w.fpos);
        ctx->timing_end(tok_);
    }
    LGS_HIP_CHECK(hipGetLastError());
    {
        const int tok_ = ctx->timing_begin(K_REPLAY, 0.0);
        hipLaunchKernelGGL(k_replay, dim3(1), dim3(64), 0, st, pl, w.cscore, w.cflag, w.list, w.count,
                           w.fval, w.fpos, w.Lp, d_rec, w.poses7);
        ctx->timing_end(tok_);
    }
    LGS_HIP_CHECK(hipGetLastError());
    // cost + covariance terms at the 7 poses
    CostPlan cp = make_cost_plan(grid, cost, scan);
    {
        dim3 g((scan->n + 255) / 256, 7);
        hipLaunchKernelGGL(k_cost_idx, g, dim3(256), 0, st, cp, scan->d_ranges, scan->d_angles,
                           w.poses7, w.cidx, d_rec, ctx->guard_cap, ctx->guard_eps, inject);
        LGS_HIP_CHECK(hipGetLastError());
        if (opt.cost_patches && !opt.cost_patches->empty()) {
            // (key, cells) pairs: cidx[key.x] = cells, computed on the host with glibc
            const int np = (int)(opt.cost_patches->size() / 2);
            int4* dp = (int4*)ctx->ensure(S_PATCH, sizeof(int4) * opt.cost_patches->size());
            LGS_HIP_CHECK(hipMemcpyAsync(dp, opt.cost_patches->data(),
                                         sizeof(int4) * opt.cost_patches->size(),
                                         hipMemcpyHostToDevice, st));
            hipLaunchKernelGGL(k_cost_patch, dim3((np + 255) / 256), dim3(256), 0, st, w.cidx, dp, np);
            LGS_HIP_CHECK(hipGetLastError());
        }
        {
            const int tok_ = ctx->timing_begin(K_COST, 8.0 * 7.0 * 2.0 * (2 * cost->kernel_size + 1) * (2 * cost->kernel_size + 1) * (double)scan->n);
            hipLaunchKernelGGL(k_cost_eval, dim3(7), dim3(256), 0, st, cp, grid->d, w.cidx, w.terms,
                               d_rec->costs);
            ctx->timing_end(tok_);
        }
        LGS_HIP_CHECK(hipGetLastError());
    }
}

// glibc recomputation of one projected index (host side of the guard).
void host_project(const RtcsmPlan& pl, const lgs_scan* scan, int vbeam, int tt, int& ix, int& iy)
{
    const double r = scan->h_ranges[vbeam];
    const double a = scan->h_angles[vbeam];
    const double th = pl.st + pl.step_t * (double)(tt - pl.win_t);
    const double c = std::cos(th + a);
    const double s = std::sin(th + a);
    const double hx = pl.sx + r * c;
    const double hy = pl.sy + r * s;
    ix = (int)std::floor((hx - pl.min_x) / pl.res);
    iy = (int)std::floor((hy - pl.min_y) / pl.res);
}

void host_cost_cells(const CostPlan& cp, const lgs_scan* scan, const double pose[3], int beam,
                     int cells[4])
{
    const double r = scan->h_ranges[beam];
    const double c = std::cos(pose[2] + scan->h_angles[beam]);
    const double s = std::sin(pose[2] + scan->h_angles[beam]);
    const double hx = pose[0] + r * c;
    const double hy = pose[1] + r * s;
    const double mx = pose[0] + (r - cp.hit_and_missed_dist) * c;
    const double my = pose[1] + (r - cp.hit_and_missed_dist) * s;
    cells[0] = (int)std::floor((hx - cp.min_x) / cp.res);
    cells[1] = (int)std::floor((hy - cp.min_y) / cp.res);
    cells[2] = (int)std::floor((mx - cp.min_x) / cp.res);
    cells[3] = (int)std::floor((my - cp.min_y) / cp.res);
}

// Host-side seven poses (identical arithmetic to k_replay).
void host_poses7(const RtcsmPlan& pl, const int best[3], double P7[7][3])
{
    const double x = pl.sx + best[0] * pl.step_x;
    const double y = pl.sy + best[1] * pl.step_y;
    const double th = pl.st + best[2] * pl.step_t;
    const double dl = pl.res, da = 1e-2;
    const double v[7][3] = {
        { x, y, th },
        { x + dl, y + 0.0, th + 0.0 }, { x - dl, y - 0.0, th - 0.0 },
        { x + 0.0, y + dl, th + 0.0 }, { x - 0.0, y - dl, th - 0.0 },
        { x + 0.0, y + 0.0, th + da }, { x - 0.0, y - 0.0, th - da },
    };
    std::memcpy(P7, v, sizeof(v));
}

// Verify guarded projections against glibc; returns true if the match must be
// re-run (and fills the options for the rerun).
bool check_projection_guards(lgs_ctx* ctx, const RtcsmPlan& pl, const lgs_scan* scan,
                             const RtcsmRecord& rec, std::vector<int4>& patches,
                             std::vector<int2>& host_idx, bool& use_host_idx)
{
    use_host_idx = false;
    patches.clear();
    if (rec.guard_count == 0) return false;
    if (rec.guard_count > ctx->guard_cap) {
        // too many to inspect: full host projection (exact, slow path)
        host_idx.resize((size_t)pl.T * pl.Nv);
        for (int tt = 0; tt < pl.T; ++tt)
            for (int v = 0; v < pl.Nv; ++v) {
                int ix, iy;
                host_project(pl, scan, scan->h_vidx[v], tt, ix, iy);
                host_idx[(size_t)tt * pl.Nv + v] = make_int2(ix, iy);
            }
        use_host_idx = true;
        return true;
    }
    for (int k = 0; k < rec.guard_count; ++k) {
        const GuardRec& g = rec.guard[k];
        int ix, iy;
        host_project(pl, scan, scan->h_vidx[g.v], g.t, ix, iy);
        if (ix != g.ix || iy != g.iy) patches.push_back(make_int4(g.t, g.v, ix, iy));
    }
    return !patches.empty();
}

bool check_cost_guards(lgs_ctx* ctx, const RtcsmPlan& pl, const CostPlan& cp,
                       const lgs_scan* scan, const RtcsmRecord& rec, std::vector<int4>& cpatch,
                       bool& full)
{
    cpatch.clear();
    full = false;
    if (rec.cost_guard_count == 0) return false;
    double P7[7][3];
    host_poses7(pl, rec.best, P7);
    if (rec.cost_guard_count > ctx->guard_cap) {
        full = true;
        return true;
    }
    bool bad = false;
    std::vector<std::pair<int, int>> seen;
    for (int k = 0; k < rec.cost_guard_count; ++k) {
        const CostGuardRec& g = rec.cost_guard[k];
        const int pi = g.pose_which / 4, which = g.pose_which % 4;
        int cells[4];
        host_cost_cells(cp, scan, P7[pi], g.beam, cells);
        if (cells[which] != g.ix) bad = true;
        seen.push_back({ pi, g.beam });
    }
    if (!bad) return false;
    std::sort(seen.begin(), seen.end());
    seen.erase(std::unique(seen.begin(), seen.end()), seen.end());
    for (auto& pb : seen) {
        int cells[4];
        host_cost_cells(cp, scan, P7[pb.first], pb.second, cells);
        cpatch.push_back(make_int4(pb.first * cp.N + pb.second, 0, 0, 0));
        cpatch.push_back(make_int4(cells[0], cells[1], cells[2], cells[3]));
    }
    return true;
}

void finish_summary(const RtcsmPlan& pl, const lgs_scan* scan, lgs_pose2d initial,
                    const RtcsmRecord& rec, lgs_rtcsm_summary* out)
{
    std::memset(out, 0, sizeof(*out));
    out->pose_found = rec.found;
    out->initial_pose = initial;
    out->score_max = rec.score_max;
    out->score_threshold = pl.thr;
    for (int i = 0; i < 3; ++i) out->best_win[i] = rec.best[i];
    out->win[0] = pl.win_x;
    out->win[1] = pl.win_y;
    out->win[2] = pl.win_t;
    out->steps[0] = pl.step_x;
    out->steps[1] = pl.step_y;
    out->steps[2] = pl.step_t;
    // :122-125
    const lgs_pose2d best{ pl.sx + rec.best[0] * pl.step_x, pl.sy + rec.best[1] * pl.step_y,
                           pl.st + rec.best[2] * pl.step_t };
    out->best_sensor_pose = best;
    // :128-135
    out->normalized_cost = rec.costs[0] / (double)scan->n;
    out->estimated_pose = move_backward(best, scan->rel);
    // ComputeGradient / ComputeCovariance (C/mapping/cost_function_greedy_endpoint.cpp:131-170)
    const double dl = pl.res, da = 1e-2;
    const double g[3] = { 0.5 * (rec.costs[1] - rec.costs[2]) / dl,
                          0.5 * (rec.costs[3] - rec.costs[4]) / dl,
                          0.5 * (rec.costs[5] - rec.costs[6]) / da };
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) out->covariance[3 * i + j] = g[i] * g[j];
    out->covariance[0] += 0.01;
    out->covariance[4] += 0.01;
    out->covariance[8] += 0.01;
    out->coarse_blocks = pl.K;
    out->fine_blocks = rec.n_eval;
}

void check_args(const lgs_grid* grid, const lgs_grid* coarse, const lgs_rtcsm_params* p,
                const lgs_cost_ge_params* c, const lgs_scan* s)
{
    LGS_REQUIRE(grid && coarse && p && c && s, "null argument");
    LGS_REQUIRE(grid->w == coarse->w && grid->h == coarse->h && grid->min_x == coarse->min_x &&
                    grid->min_y == coarse->min_y && grid->res == coarse->res,
                "coarse map must have the fine map's geometry (CreateSameSizeMap)");
    LGS_REQUIRE(p->low_resolution >= 1 && p->low_resolution <= 32, "low_resolution must be in [1, 32]");
    LGS_REQUIRE(p->range_x >= 0 && p->range_y >= 0 && p->range_theta >= 0, "negative search range");
    LGS_REQUIRE(s->n >= 1, "empty scan");
    LGS_REQUIRE(c->kernel_size >= 0, "negative kernel size");
}

// Run n matches against one grid with one host synchronisation in the common
// case; guarded projections / dangerous blocks trigger exact per-scan reruns.
void run_batch(lgs_ctx* ctx, const lgs_grid* grid, const lgs_grid* coarse,
               const lgs_rtcsm_params* params, const lgs_cost_ge_params* cost,
               lgs_scan* const* scans, const lgs_pose2d* init, int n, double nthr,
               lgs_rtcsm_summary* out)
{
    LGS_HIP_CHECK(hipSetDevice(ctx->device));
    std::vector<RtcsmPlan> plans(n);
    std::vector<const int*> vidx(n);
    for (int j = 0; j < n; ++j) {
        check_args(grid, coarse, params, cost, scans[j]);
        int nv = 0;
        vidx[j] = scan_valid_indices(ctx, scans[j], params->scan_range_max, &nv);
        plans[j] = make_plan(grid, params, scans[j], init[j], nthr, nv);
        LGS_REQUIRE(plans[j].K < (1LL << 31), "search window too large");
    }
    RtcsmRecord* d_rec = (RtcsmRecord*)ctx->ensure(S_RECORDS, sizeof(RtcsmRecord) * (size_t)n);
    RtcsmRecord* h_rec = (RtcsmRecord*)ctx->ensure_pinned(sizeof(RtcsmRecord) * (size_t)n);
    ScanOptions none;
    for (int j = 0; j < n; ++j)
        enqueue_match(ctx, grid, coarse, cost, scans[j], plans[j], vidx[j], d_rec + j, none);
    LGS_HIP_CHECK(hipMemcpyAsync(h_rec, d_rec, sizeof(RtcsmRecord) * (size_t)n,
                                 hipMemcpyDeviceToHost, ctx->stream));
    LGS_HIP_CHECK(hipStreamSynchronize(ctx->stream));
    if (ctx->profile) ctx->harvest();

    for (int j = 0; j < n; ++j) {
        RtcsmRecord rec = h_rec[j];
        int guard_hits = rec.guard_count + rec.cost_guard_count;
        int fixups = 0, slow = 0;
        // exactness loop: at most a few reruns
        ScanOptions opt;
        std::vector<int4> patches, cpatch;
        std::vector<int2> hidx;
        for (int iter = 0; iter < 4; ++iter) {
            bool use_hidx = false, full_cost = false;
            bool rerun = false;
            if (!opt.host_idx && !opt.patches &&
                check_projection_guards(ctx, plans[j], scans[j], rec, patches, hidx, use_hidx)) {
                if (use_hidx) opt.host_idx = &hidx;
                else opt.patches = &patches;
                rerun = true;
                fixups = 1;
            }
            if (rec.status & REC_DANGEROUS && !opt.dense) {
                opt.dense = true;
                rerun = true;
                slow = 1;
            }
            if (!rerun && !opt.cost_patches) {
                CostPlan cp = make_cost_plan(grid, cost, scans[j]);
                if (check_cost_guards(ctx, plans[j], cp, scans[j], rec, cpatch, full_cost)) {
                    if (full_cost) {
                        // rebuild every cost cell on the host
                        double P7[7][3];
                        host_poses7(plans[j], rec.best, P7);
                        cpatch.clear();
                        for (int pi = 0; pi < 7; ++pi)
                            for (int b = 0; b < cp.N; ++b) {
                                const double r = scans[j]->h_ranges[b];
                                if (r >= cp.max_range || r <= cp.min_range) continue;
                                int cells[4];
                                host_cost_cells(cp, scans[j], P7[pi], b, cells);
                                cpatch.push_back(make_int4(pi * cp.N + b, 0, 0, 0));
                                cpatch.push_back(make_int4(cells[0], cells[1], cells[2], cells[3]));
                            }
                    }
                    opt.cost_patches = &cpatch;
                    rerun = true;
                    fixups = 1;
                }
            }
            if (!rerun) break;
            enqueue_match(ctx, grid, coarse, cost, scans[j], plans[j], vidx[j], d_rec + j, opt);
            LGS_HIP_CHECK(hipMemcpyAsync(&h_rec[j], d_rec + j, sizeof(RtcsmRecord),
                                         hipMemcpyDeviceToHost, ctx->stream));
            LGS_HIP_CHECK(hipStreamSynchronize(ctx->stream));
            rec = h_rec[j];
            if (opt.patches || opt.host_idx) rec.guard_count = 0;  // already exact
        }
        finish_summary(plans[j], scans[j], init[j], rec, &out[j]);
        out[j].guard_hits = guard_hits;
        out[j].fixups = fixups;
        out[j].slow_path = slow;
    }
}

}  // namespace

extern "C" int lgs_rtcsm_optimize_pose(lgs_ctx* ctx, const lgs_grid* grid, const lgs_grid* coarse,
                                       const lgs_rtcsm_params* params,
                                       const lgs_cost_ge_params* cost, const lgs_scan* scan,
                                       lgs_pose2d initial, double nthr, lgs_rtcsm_summary* out)
{
    if (!ctx || !out) return LGS_ERR_INVALID_ARG;
    return guarded(ctx, [&] {
        lgs_scan* s = const_cast<lgs_scan*>(scan);
        run_batch(ctx, grid, coarse, params, cost, &s, &initial, 1, nthr, out);
    });
}

extern "C" int lgs_rtcsm_optimize_pose_batch(lgs_ctx* ctx, const lgs_grid* grid,
                                             const lgs_grid* coarse, const lgs_rtcsm_params* params,
                                             const lgs_cost_ge_params* cost,
                                             const lgs_scan* const* scans,
                                             const lgs_pose2d* initial, int n, double nthr,
                                             lgs_rtcsm_summary* out)
{
    if (!ctx || !out || !scans || !initial || n < 0) return LGS_ERR_INVALID_ARG;
    if (n == 0) return LGS_OK;
    return guarded(ctx, [&] {
        run_batch(ctx, grid, coarse, params, cost, const_cast<lgs_scan* const*>(scans), initial, n,
                  nthr, out);
    });
}

extern "C" int lgs_rtcsm_optimize_pose_query(lgs_ctx* ctx, const lgs_grid* grid,
                                             const lgs_rtcsm_params* params,
                                             const lgs_cost_ge_params* cost,
                                             const lgs_scan* scan, lgs_pose2d initial,
                                             lgs_rtcsm_summary* out)
{
    if (!ctx || !grid || !params || !out) return LGS_ERR_INVALID_ARG;
    return guarded(ctx, [&] {
        LGS_REQUIRE(params->low_resolution >= 1, "low_resolution must be >= 1");
        // ComputeCoarserMap (:148-153) into a context-owned coarse grid
        lgs_grid* cg = ctx->coarse_scratch;
        if (!cg) {
            cg = new lgs_grid();
            cg->ctx = ctx;
            cg->owned = false;
            ctx->coarse_scratch = cg;
        }
        cg->d = (double*)ctx->ensure(S_COARSE_GRID, sizeof(double) * std::max<size_t>(1, (size_t)grid->w * grid->h));
        cg->w = grid->w;
        cg->h = grid->h;
        cg->min_x = grid->min_x;
        cg->min_y = grid->min_y;
        cg->res = grid->res;
        launch_precompute(ctx, grid, params->low_resolution, cg->d);
        lgs_scan* s = const_cast<lgs_scan*>(scan);
        run_batch(ctx, grid, cg, params, cost, &s, &initial, 1, DBL_MIN, out);
    });
}

extern "C" int lgs_rtcsm_dense_scores(lgs_ctx* ctx, const lgs_grid* grid, const lgs_grid* coarse,
                                      const lgs_rtcsm_params* params, const lgs_scan* scan,
                                      lgs_pose2d initial, double* coarse_scores,
                                      double* fine_scores, int* dims)
{
    if (!ctx || !grid || !coarse || !params || !scan) return LGS_ERR_INVALID_ARG;
    return guarded(ctx, [&] {
        LGS_HIP_CHECK(hipSetDevice(ctx->device));
        lgs_scan* s = const_cast<lgs_scan*>(scan);
        int nv = 0;
        const int* vidx = scan_valid_indices(ctx, s, params->scan_range_max, &nv);
        RtcsmPlan pl = make_plan(grid, params, s, initial, DBL_MIN, nv);
        const int nfx = pl.ncx * pl.low_res, nfy = pl.ncy * pl.low_res;
        if (dims) {
            dims[0] = pl.win_x; dims[1] = pl.win_y; dims[2] = pl.win_t;
            dims[3] = pl.ncx; dims[4] = pl.ncy; dims[5] = nfx; dims[6] = nfy;
        }
        if (!coarse_scores && !fine_scores) return;
        Workspace w = ensure_workspace(ctx, pl, s->n);
        RtcsmRecord* d_rec = (RtcsmRecord*)ctx->ensure(S_RECORDS, sizeof(RtcsmRecord));
        LGS_HIP_CHECK(hipMemsetAsync(d_rec, 0, sizeof(RtcsmRecord), ctx->stream));
        if (nv > 0) {
            dim3 g((nv + 255) / 256, pl.T);
            hipLaunchKernelGGL(k_project, g, dim3(256), 0, ctx->stream, pl, s->d_ranges, s->d_angles,
                               vidx, w.idx, d_rec, 0, -1.0, 0);
            LGS_HIP_CHECK(hipGetLastError());
        }
        if (coarse_scores) {
            dim3 g((pl.P + kCoarseBlock - 1) / kCoarseBlock, pl.T);
            hipLaunchKernelGGL(k_coarse, g, dim3(kCoarseBlock), 0, ctx->stream, pl, coarse->d, w.idx,
                               w.cscore, w.cflag, w.part_c, w.part_k);
            LGS_HIP_CHECK(hipGetLastError());
            LGS_HIP_CHECK(hipMemcpyAsync(coarse_scores, w.cscore, sizeof(double) * (size_t)pl.K,
                                         hipMemcpyDeviceToHost, ctx->stream));
        }
        if (fine_scores) {
            const size_t nf = (size_t)pl.T * nfx * nfy;
            double* d = (double*)ctx->ensure(S_DENSE_FINE, sizeof(double) * nf);
            dim3 g((nfx * nfy + 255) / 256, pl.T);
            hipLaunchKernelGGL(k_fine_dense, g, dim3(256), 0, ctx->stream, pl, grid->d, w.idx, nfx,
                               nfy, d);
            LGS_HIP_CHECK(hipGetLastError());
            LGS_HIP_CHECK(hipMemcpyAsync(fine_scores, d, sizeof(double) * nf, hipMemcpyDeviceToHost,
                                         ctx->stream));
        }
        LGS_HIP_CHECK(hipStreamSynchronize(ctx->stream));
    });
}

extern "C" int lgs_cost_greedy_endpoint(lgs_ctx* ctx, const lgs_grid* grid,
                                        const lgs_cost_ge_params* cost, const lgs_scan* scan,
                                        lgs_pose2d pose, double* out_cost)
{
    if (!ctx || !grid || !cost || !scan || !out_cost) return LGS_ERR_INVALID_ARG;
    return guarded(ctx, [&] {
        LGS_HIP_CHECK(hipSetDevice(ctx->device));
        CostPlan cp = make_cost_plan(grid, cost, scan);
        double* poses = (double*)ctx->ensure(S_POSES7, sizeof(double) * 21);
        int4* cidx = (int4*)ctx->ensure(S_COST_IDX, sizeof(int4) * 7 * (size_t)scan->n);
        double* terms = (double*)ctx->ensure(S_COST_TERM, sizeof(double) * 7 * (size_t)scan->n);
        RtcsmRecord* d_rec = (RtcsmRecord*)ctx->ensure(S_RECORDS, sizeof(RtcsmRecord));
        RtcsmRecord* h_rec = (RtcsmRecord*)ctx->ensure_pinned(sizeof(RtcsmRecord));
        double hp[3] = { pose.x, pose.y, pose.theta };
        LGS_HIP_CHECK(hipMemsetAsync(d_rec, 0, sizeof(RtcsmRecord), ctx->stream));
        LGS_HIP_CHECK(hipMemcpyAsync(poses, hp, sizeof(hp), hipMemcpyHostToDevice, ctx->stream));
        hipLaunchKernelGGL(k_cost_idx, dim3((scan->n + 255) / 256, 1), dim3(256), 0, ctx->stream, cp,
                           scan->d_ranges, scan->d_angles, poses, cidx, d_rec, ctx->guard_cap,
                           ctx->guard_eps, 0);
        LGS_HIP_CHECK(hipGetLastError());
        hipLaunchKernelGGL(k_cost_eval, dim3(1), dim3(256), 0, ctx->stream, cp, grid->d, cidx, terms,
                           d_rec->costs);
        LGS_HIP_CHECK(hipGetLastError());
        LGS_HIP_CHECK(hipMemcpyAsync(h_rec, d_rec, sizeof(RtcsmRecord), hipMemcpyDeviceToHost,
                                     ctx->stream));
        LGS_HIP_CHECK(hipStreamSynchronize(ctx->stream));
        if (h_rec->cost_guard_count > 0) {
            // exact host recomputation of the guarded cells, then re-evaluate
            std::vector<int4> fix;
            for (int b = 0; b < cp.N; ++b) {
                const double r = scan->h_ranges[b];
                if (r >= cp.max_range || r <= cp.min_range) continue;
                int cells[4];
                host_cost_cells(cp, scan, hp, b, cells);
                fix.push_back(make_int4(cells[0], cells[1], cells[2], cells[3]));
            }
            // rebuild the full index row on the host (N entries)
            std::vector<int4> row((size_t)cp.N, make_int4(INT_MIN, 0, 0, 0));
            size_t k = 0;
            for (int b = 0; b < cp.N; ++b) {
                const double r = scan->h_ranges[b];
                if (r >= cp.max_range || r <= cp.min_range) continue;
                row[b] = fix[k++];
            }
            LGS_HIP_CHECK(hipMemcpyAsync(cidx, row.data(), sizeof(int4) * row.size(),
                                         hipMemcpyHostToDevice, ctx->stream));
            hipLaunchKernelGGL(k_cost_eval, dim3(1), dim3(256), 0, ctx->stream, cp, grid->d, cidx,
                               terms, d_rec->costs);
            LGS_HIP_CHECK(hipGetLastError());
            LGS_HIP_CHECK(hipMemcpyAsync(h_rec, d_rec, sizeof(RtcsmRecord), hipMemcpyDeviceToHost,
                                         ctx->stream));
            LGS_HIP_CHECK(hipStreamSynchronize(ctx->stream));
        }
        *out_cost = h_rec->costs[0];
    });
}
