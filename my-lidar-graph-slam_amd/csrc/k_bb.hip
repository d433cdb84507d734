// k_bb.hip -- branch-and-bound matcher on MI355X.
//
// Restates ScanMatcherBranchBound::OptimizePose
// (C/mapping/scan_matcher_branch_bound.cpp:47-154) with ScorePixelAccurate
// (C/mapping/score_function_pixel_accurate.cpp:19-77) over the window-max
// pyramid of PrecomputeGridMaps (C/mapping/grid_map_builder.cpp:471-495).
//
// The reference walks a LIFO depth-first search whose pruning depends on the
// best score found so far, and its node scores recompute every hit point at
// the node's own pose, so parent scores do not bound child scores exactly
// (rounding): the visit order decides the result.  The device therefore does
// not search; it scores, level by level, every node the reference's search
// can visit:
//   * a node is visited only if each ancestor was expanded, i.e. scored above
//     the running best at its turn, which is >= the threshold thr0;
//   * before the first leaf is accepted the search only walks the first
//     descent (the last-pushed top node, then always the last-pushed child);
//     if that whole path scores above thr0 its leaf L1 is accepted and every
//     later expansion needs a score > s(L1).
// So expanding every node scored above thr_exp = (path valid ? s(L1) : thr0),
// plus the path nodes, covers the visited set.  The host then replays the
// reference's search over these scores, exactly, and the greedy-endpoint
// cost/covariance of the best pose come from k_cost (k_rtcsm.hip).
//
//   k_bb_trig    r cos(a), r sin(a) per valid beam and cos(theta_t), sin(theta_t)
//                per angle; a node's hit offsets come by rotation (r4), within
//                ~1e-13 cells of the reference's r cos(theta_t + a): inside the
//                guard band, like k_project's
//   k_bb_score   one lane per node: hit cells at the node pose (the
//                reference's own arithmetic), sequential fp64 beam-order sum
//                of the level's map values; cells within guard_eps of a cell
//                boundary are recorded and re-checked on the host with glibc
//   k_bb_expand  the four children of every node scored above thr_exp (or on
//                the first descent), wave-aggregated appends
//   k_bb_rescore exact re-score of a node from host (glibc) cells
#include "lgs_internal.hpp"

#include <algorithm>
#include <cfloat>
#include <cstring>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <unordered_map>

using namespace lgs;

namespace lgs {
void launch_precompute(lgs_ctx* ctx, const lgs_grid* in, int win, double* out, const PlaneGeom* planes);
void cost_summaries(lgs_ctx* ctx, const lgs_grid* grid, const lgs_cost_ge_params* cost, lgs_scan* const* scans,
                    const lgs_pose2d* best, int n, lgs_rtcsm_summary* out);
}  // namespace lgs

namespace {

constexpr int kBBMaxH = 12;   // NodeHeightMax limit (window 4096 cells)
constexpr int kBBBatch = 512; // matches per run_bb (one k_bb_score launch per level for all of them)

// One match of a batched branch-and-bound launch (device memory).
struct BBItem {
    double sx, sy, st;            // sensor pose (Compound(initialPose, relPose))
    double step_x, step_y, step_t;
    double min_x, min_y, res;     // map geometry
    double thr_exp;               // expansion threshold (see header)
    int W, H;
    int T, Nv, win_t;
    int px, py, pt, hmax;         // first descent's top node; path forced when path_ok
    int path_ok;
    const double* ranges;
    const double* angles;
    const int* vidx;              // valid beams (ScorePixelAccurate filter), beam order
    double* rca;                  // [Nv] r cos(a), r sin(a) of the valid beams
    double* rsa;
    double* tc;                   // [T] cos(theta_t), sin(theta_t) of the search angles
    double* ts;
    const double* maps[kBBMaxH + 1];
};

// node: x = item << 4 | level, y = x index, z = y index, w = theta index
__device__ __forceinline__ int node_item(int4 n) { return n.x >> 4; }
__device__ __forceinline__ int node_level(int4 n) { return n.x & 15; }

struct BBGuard {
    int level, node, v, pad;      // node index within its level's list
    int ix, iy, pad2, pad3;       // device cell
};

__global__ __launch_bounds__(256) void k_bb_trig(const BBItem* __restrict__ items)
{
    const BBItem& it = items[blockIdx.z];
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k < it.Nv) {
        const int i = it.vidx[k];
        double sn, cs;
        sincos(it.angles[i], &sn, &cs);
        const double r = it.ranges[i];
        it.rca[k] = r * cs;
        it.rsa[k] = r * sn;
    }
    if (k < it.T) {
        // nodePose.mTheta = sensorPose.mTheta + currentNode.mTheta * stepTheta (:96-99)
        const double th = it.st + (double)(k - it.win_t) * it.step_t;
        double sn, cs;
        sincos(th, &sn, &cs);
        it.tc[k] = cs;
        it.ts[k] = sn;
    }
}

constexpr int kBBPipe = 16;
// The cell index uses (hit - min) * (1 / res) instead of the reference's
// division: the product is within 1 ulp of the quotient (~1e-13 cells at
// map sizes here), far inside guard_eps, so every cell whose floor could
// differ from the reference's is guarded and re-checked on the host.
// One node's score (one lane): the reference's beam-order sum over the
// level's map, with the guard records of near-boundary cells.
__device__ __forceinline__ void score_node(const BBItem& it, int4 nd, int i, int level_id, double* __restrict__ scores,
                                           BBGuard* __restrict__ guards, int* __restrict__ nguard, int guard_cap,
                                           double guard_eps, int inject)
{
    const int h = node_level(nd);
    // nodePose (:96-99)
    const double nx = it.sx + (double)nd.y * it.step_x;
    const double ny = it.sy + (double)nd.z * it.step_y;
    const int Nv = it.Nv, W = it.W, H = it.H;
    const double* __restrict__ rca = it.rca;
    const double* __restrict__ rsa = it.rsa;
    const double ct = it.tc[nd.w + it.win_t], st = it.ts[nd.w + it.win_t];
    const double* __restrict__ map = it.maps[h];
    const double minx = it.min_x, miny = it.min_y, inv = 1.0 / it.res;
    double sum = 0.0;
    for (int v0 = 0; v0 < Nv; v0 += kBBPipe) {
        double cx[kBBPipe], cy[kBBPipe], val[kBBPipe];
#pragma unroll
        for (int j = 0; j < kBBPipe; ++j) {   // independent loads first
            const int v = min(v0 + j, Nv - 1);
            // ScanData::HitPoint (H/sensor/sensor_data.hpp:162-173) by rotation
            const double a = gload(rca + v), b = gload(rsa + v);
            cx[j] = ct * a - st * b;
            cy[j] = st * a + ct * b;
        }
#pragma unroll
        for (int j = 0; j < kBBPipe; ++j) {
            const int v = v0 + j;
            // WorldCoordinateToGridCellIndex of HitPoint (H/grid_map/grid_map.hpp:779-790)
            const double qx = (nx + cx[j] - minx) * inv;
            const double qy = (ny + cy[j] - miny) * inv;
            const double fx = floor(qx), fy = floor(qy);
            int ix = (int)fx, iy = (int)fy;
            const double ex = guard_eps + fabs(qx) * 1e-13, ey = guard_eps + fabs(qy) * 1e-13;
            const double rx = qx - fx, ry = qy - fy;
            if (v < Nv && (rx < ex || rx > 1.0 - ex || ry < ey || ry > 1.0 - ey)) {
                ix += inject;
                const int slot = atomicAdd(nguard, 1);
                if (slot < guard_cap) {
                    BBGuard g;
                    g.level = level_id;
                    g.node = i;
                    g.v = v;
                    g.ix = ix;
                    g.iy = iy;
                    g.pad = g.pad2 = g.pad3 = 0;
                    guards[slot] = g;
                }
            }
            // GridMap::Value(idx, unknown): 0.0 outside; unknown cells (0.0)
            // are skipped by the reference (:55-56), adding 0.0 is the same
            const bool inb = (v < Nv) & ((unsigned)ix < (unsigned)W) & ((unsigned)iy < (unsigned)H);
            val[j] = inb ? gload(map + ((size_t)iy * W + ix)) : 0.0;
        }
#pragma unroll
        for (int j = 0; j < kBBPipe; ++j) sum += val[j];
    }
    scores[i] = sum;
}

__global__ __launch_bounds__(256) void k_bb_score(const BBItem* __restrict__ items, const int4* __restrict__ nodes,
                                                  int n, int level_id, double* __restrict__ scores,
                                                  BBGuard* __restrict__ guards, int* __restrict__ nguard,
                                                  int guard_cap, double guard_eps, int inject)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int4 nd = nodes[i];
    // r05: a wave whose nodes all belong to one match (the common case: the
    // top nodes are listed per match, children follow their parents) reads
    // that match's fields and beam table through scalar loads -- the beam's
    // rotation terms (rca, rsa) then cost no vector memory instruction, only
    // the map gather does
    const int j = node_item(nd);
    const int j0 = __builtin_amdgcn_readfirstlane(j);
    const bool uniform = __ballot(j != j0) == 0ull;
    if (uniform) score_node(items[j0], nd, i, level_id, scores, guards, nguard, guard_cap, guard_eps, inject);
    else score_node(items[j], nd, i, level_id, scores, guards, nguard, guard_cap, guard_eps, inject);
}

// child[i] = the index of node i's first child in the next level's list (its
// four children are consecutive there), -1 when not expanded (k_bb_replay);
// ncount[item] += 4 per expanded node (nodes scored per match)
__global__ __launch_bounds__(256) void k_bb_expand(const BBItem* __restrict__ items, const int4* __restrict__ nodes,
                                                   const double* __restrict__ scores, int n,
                                                   int4* __restrict__ next, int* __restrict__ count, int cap,
                                                   int* __restrict__ overflow, int* __restrict__ child,
                                                   unsigned long long* __restrict__ ncount)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    bool ex = false;
    int4 nd = make_int4(0, 0, 0, 0);
    if (i < n) {
        nd = nodes[i];
        const int h = node_level(nd);
        if (h > 0) {
            const BBItem& it = items[node_item(nd)];
            const int off = (1 << it.hmax) - (1 << h);
            const bool path = it.path_ok && nd.w == it.pt && nd.y == it.px + off && nd.z == it.py + off;
            ex = scores[i] > it.thr_exp || path;
        }
    }
    const unsigned long long bal = __ballot(ex);
    if (bal == 0ull) {
        if (i < n) child[i] = -1;
        return;
    }
    const int lane = threadIdx.x & 63;
    const int leader = __ffsll((long long)bal) - 1;
    int base = 0;
    if (lane == leader) base = atomicAdd(count, 4 * __popcll(bal));
    base = __shfl(base, leader, 64);
    if (!ex) {
        if (i < n) child[i] = -1;
        return;
    }
    const int pos = base + 4 * __popcll(bal & ((1ull << lane) - 1ull));
    if (pos + 4 > cap) {
        *overflow = 1;
        child[i] = -1;
        return;
    }
    child[i] = pos;
    atomicAdd(ncount + node_item(nd), 4ull);
    // :123-135: children (x, y), (x + ws, y), (x, y + ws), (x + ws, y + ws)
    const int h = node_level(nd) - 1, ws = 1 << h;
    const int head = (node_item(nd) << 4) | h;
    next[pos + 0] = make_int4(head, nd.y, nd.z, nd.w);
    next[pos + 1] = make_int4(head, nd.y + ws, nd.z, nd.w);
    next[pos + 2] = make_int4(head, nd.y, nd.z + ws, nd.w);
    next[pos + 3] = make_int4(head, nd.y + ws, nd.z + ws, nd.w);
}

// Exact re-score of listed nodes (one workgroup each) from host cells:
// cells[k * Nmax + v] for valid beam v; lanes load, lane 0 adds in beam order.
__global__ __launch_bounds__(64) void k_bb_rescore(const double* const* __restrict__ maps, const int* __restrict__ dims,
                                                   const int2* __restrict__ cells, const int* __restrict__ nv,
                                                   int Nmax, double* const* __restrict__ out)
{
    __shared__ double buf[64];
    const int k = blockIdx.x;
    const double* __restrict__ map = maps[k];
    const int W = dims[2 * k], H = dims[2 * k + 1];
    const int n = nv[k];
    double sum = 0.0;
    for (int v0 = 0; v0 < n; v0 += 64) {
        const int v = v0 + threadIdx.x;
        double val = 0.0;
        if (v < n) {
            const int2 c = cells[(size_t)k * Nmax + v];
            if (((unsigned)c.x < (unsigned)W) & ((unsigned)c.y < (unsigned)H)) val = map[(size_t)c.y * W + c.x];
        }
        buf[threadIdx.x] = val;
        __syncthreads();
        if (threadIdx.x == 0) {
            const int m = min(64, n - v0);
            for (int j = 0; j < m; ++j) sum += buf[j];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) *out[k] = sum;   // the node's slot in its level's score list
}

// The guarded nodes' coordinates (node lists stay on the device).
__global__ __launch_bounds__(256) void k_bb_guard_nodes(const int4* const* __restrict__ lists,
                                                       const BBGuard* __restrict__ guards, int ng,
                                                       int4* __restrict__ out)
{
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= ng) return;
    out[k] = lists[guards[k].level][guards[k].node];
}

// The reference's search (:81-140) over the scored levels, one thread per
// match: the LIFO order walked with a cursor per level instead of a stack of
// nodes (the top nodes, pushed in (x, y, t) order, pop last first; an
// expanded node's four children are consecutive in the next level's list and
// pop 3, 2, 1, 0).  Expanding a node loads its four children's scores and
// child indices at once into LDS, so a visit costs no memory round trip of
// its own.  A node the search expands that the device did not expand (child
// index -1) can only follow a guard-corrected path score: the match fails and
// is rerun over the thr0 superset (as the host replay did).
struct BBReplay {
    const double* scores[kBBMaxH + 1];   // per level id l = Hm - h
    const int* child[kBBMaxH + 1];
    const int4* leaves;                  // level Hm's node list (h = 0)
    int hm;
};
struct BBResult {
    double score;
    int x, y, t, failed;
    long long visited;
};
// One match per wave (lane 0): lanes of one wave walking different matches
// diverge at every visit, and a wave then pays a memory round trip in every
// step where any of its lanes expands (measured 8.7 ms for 512 matches as 8
// waves of 64, vs one round trip per expansion of its own here).
constexpr int kReplayLanes = 1;   // matches per wave
__global__ __launch_bounds__(64) void k_bb_replay(BBReplay R, const int* __restrict__ top_off,
                                                  const double* __restrict__ thr0, int n, BBResult* __restrict__ out)
{
    __shared__ double s_sc[kBBMaxH + 1][4][kReplayLanes];   // the group of four being walked at each level
    __shared__ int s_cb[kBBMaxH + 1][4][kReplayLanes];
    __shared__ int s_base[kBBMaxH + 1][kReplayLanes];
    __shared__ int s_k[kBBMaxH + 1][kReplayLanes];          // next child of the group to visit (3 .. 0)
    const int lane = threadIdx.x;
    if (lane >= kReplayLanes) return;
    const int j = blockIdx.x * kReplayLanes + lane;
    if (j >= n) return;
    const int hm = R.hm;
    const int t0 = top_off[j], t1 = top_off[j + 1];
    double smax = thr0[j];
    int leaf = -1, failed = 0;
    long long visited = 0;
    double ns = 0.0;
    int ncb = -1;
    if (t1 > t0) {
        ns = R.scores[0][t1 - 1];
        ncb = hm > 0 ? R.child[0][t1 - 1] : -1;
    }
    for (int top = t1 - 1; top >= t0 && !failed; --top) {
        double s = ns;
        int cb = ncb, idx = top;
        if (top > t0) {   // the next top node's entries, ahead of this one's subtree
            ns = R.scores[0][top - 1];
            ncb = hm > 0 ? R.child[0][top - 1] : -1;
        }
        int l = 0;
        for (;;) {
            ++visited;
            if (s > smax) {   // else pruned: score <= scoreMax (:105-109)
                if (l == hm) {   // leaf (:112-119)
                    smax = s;
                    leaf = idx;
                } else if (cb < 0) {
                    failed = 1;
                    break;
                } else {   // expand (:120-137)
                    ++l;
                    double c[4];
                    int g[4] = { 0, 0, 0, 0 };
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        c[q] = R.scores[l][cb + q];
                        if (l < hm) g[q] = R.child[l][cb + q];
                    }
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        s_sc[l][q][lane] = c[q];
                        s_cb[l][q][lane] = g[q];
                    }
                    s_base[l][lane] = cb;
                    s_k[l][lane] = 3;
                    s = c[3];
                    idx = cb + 3;
                    cb = g[3];
                    continue;
                }
            }
            while (l > 0 && s_k[l][lane] == 0) --l;   // the group is done: back up
            if (l == 0) break;
            const int q = --s_k[l][lane];
            s = s_sc[l][q][lane];
            cb = s_cb[l][q][lane];
            idx = s_base[l][lane] + q;
        }
    }
    BBResult r;
    r.score = smax;
    r.failed = failed;
    r.visited = visited;
    r.x = r.y = r.t = 0;
    if (leaf >= 0) {
        const int4 nd = R.leaves[leaf];
        r.x = nd.y;
        r.y = nd.z;
        r.t = nd.w;
    }
    out[j] = r;
}

// ------------------------------------------------------------------ host
inline size_t align256(size_t b) { return (b + 255) & ~(size_t)255; }

// Per-batch device arena carved from one slot (sizes known before the launch).
struct Carver {
    char* base;
    size_t off = 0;
    explicit Carver(char* b) : base(b) {}
    template <class T>
    T* take(size_t n)
    {
        T* p = (T*)(base + off);
        off += align256(sizeof(T) * std::max<size_t>(n, 1));
        return p;
    }
};

struct BBHost {   // host plan of one match
    lgs_pose2d sensor;
    double step_x, step_y, step_t;
    int win_x, win_y, win_t, T, Nv, N;
    double thr0;
    std::vector<int> vidx;
    std::vector<int> top_x, top_y;
};

BBHost make_bb_plan(const lgs_grid* grid, const lgs_bb_params* p, const lgs_scan* scan, lgs_pose2d init,
                    double nthr)
{
    BBHost b;
    b.sensor = compound(init, scan->rel);   // :54-56
    // ComputeSearchStep (:178-198)
    const double maxRange = std::min(scan->max_elem, p->scan_range_max);
    const double theta = grid->res / maxRange;
    b.step_x = grid->res;
    b.step_y = grid->res;
    b.step_t = std::acos(1.0 - 0.5 * theta * theta);
    // :65-70
    b.win_x = (int)std::ceil(0.5 * p->range_x / b.step_x);
    b.win_y = (int)std::ceil(0.5 * p->range_y / b.step_y);
    b.win_t = (int)std::ceil(0.5 * p->range_theta / b.step_t);
    b.T = 2 * b.win_t + 1;
    b.N = scan->n;
    b.thr0 = nthr * (double)scan->n;   // :73-75
    // ScorePixelAccurate's beam filter (:27-41)
    const double minRange = std::max(p->score_usable_range_min, scan->min_range);
    const double maxR = std::min(p->score_usable_range_max, scan->max_range);
    for (int i = 0; i < scan->n; ++i) {
        const double r = scan->h_ranges[i];
        if (r >= maxR || r <= minRange) continue;
        b.vidx.push_back(i);
    }
    b.Nv = (int)b.vidx.size();
    const int wmax = 1 << p->node_height_max;   // :81-88
    for (int x = -b.win_x; x <= b.win_x; x += wmax) b.top_x.push_back(x);
    for (int y = -b.win_y; y <= b.win_y; y += wmax) b.top_y.push_back(y);
    return b;
}

// exact hit cell of valid beam v at a node pose (glibc sincos, the reference's arithmetic)
void host_bb_cell(const BBHost& b, const lgs_grid* g, const lgs_scan* scan, int x, int y, int t, int v, int& ix,
                  int& iy)
{
    const double nx = b.sensor.x + (double)x * b.step_x;
    const double ny = b.sensor.y + (double)y * b.step_y;
    const double th = b.sensor.theta + (double)t * b.step_t;
    const int i = b.vidx[v];
    double s, c;
    ref_sincos(th + scan->h_angles[i], s, c);
    const double r = scan->h_ranges[i];
    ix = (int)std::floor((nx + r * c - g->min_x) / g->res);
    iy = (int)std::floor((ny + r * s - g->min_y) / g->res);
}

struct BBLevel {
    int4* d_nodes = nullptr;
    double* d_scores = nullptr;
    int* d_child = nullptr;   // first-child index per node (k_bb_expand), -1 = not expanded
    int n = 0;
};

// Run n branch-and-bound matches: grids[j] (fine map, its geometry) and
// pyr[j][0..H] (the map pyramid, device pointers).
// no_path: expand with thr0 everywhere (the fallback when a guard-corrected
// first descent changed the threshold the superset was built with).
void run_bb(lgs_ctx* ctx, const lgs_bb_params* p, const lgs_cost_ge_params* cost, const lgs_grid* const* grids,
            const double* const* const* pyr, lgs_scan* const* scans, const lgs_pose2d* init, int n, double nthr,
            lgs_rtcsm_summary* out, bool no_path = false)
{
    for (int k = 0; k < n; ++k) grid_acquire(ctx, grids[k]);
    LGS_HIP_CHECK(hipSetDevice(ctx->device));
    scans_to_device(ctx, scans, n);
    std::memset(out, 0, sizeof(lgs_rtcsm_summary) * (size_t)n);
    // LGS_BB_TIMING=1: per-phase host wall times on stderr (diagnostics)
    static const bool timing = std::getenv("LGS_BB_TIMING") != nullptr;
    auto t_prev = std::chrono::steady_clock::now();
    double t_ms[6] = {};
    auto lap = [&](int k) {
        if (!timing) return;
        const auto now = std::chrono::steady_clock::now();
        t_ms[k] += std::chrono::duration<double, std::milli>(now - t_prev).count();
        t_prev = now;
    };
    const int Hm = p->node_height_max;
    // the thr0 rerun fixes each level's guards before expanding it: a guard-
    // corrected score that crosses thr0 then decides the expansion too
    const bool careful = no_path;
    std::vector<BBHost> plans;
    plans.reserve((size_t)n);
    int Tmax = 1, NvMax = 1;
    size_t trig_doubles = 0, vtot = 0;
    for (int j = 0; j < n; ++j) {
        plans.push_back(make_bb_plan(grids[j], p, scans[j], init[j], nthr));
        Tmax = std::max(Tmax, plans[j].T);
        NvMax = std::max(NvMax, plans[j].Nv);
        trig_doubles += 2 * ((size_t)plans[j].T + std::max(plans[j].Nv, 1));
        vtot += plans[j].vidx.size();
    }
    // device scratch: trig tables + the valid-beam lists (one copy for the batch)
    const size_t bytes = align256(sizeof(double) * trig_doubles) + 256 * (size_t)n * 4 + align256(sizeof(int) * vtot);
    Carver cv((char*)ctx->ensure(S_BB0, bytes));
    int* d_vidx_all = cv.take<int>(vtot);
    std::vector<int> h_vidx;
    h_vidx.reserve(vtot);
    std::vector<BBItem> items((size_t)n);
    for (int j = 0; j < n; ++j) {
        const BBHost& b = plans[j];
        BBItem& it = items[j];
        std::memset(&it, 0, sizeof(it));
        it.sx = b.sensor.x;
        it.sy = b.sensor.y;
        it.st = b.sensor.theta;
        it.step_x = b.step_x;
        it.step_y = b.step_y;
        it.step_t = b.step_t;
        it.min_x = grids[j]->min_x;
        it.min_y = grids[j]->min_y;
        it.res = grids[j]->res;
        it.W = grids[j]->w;
        it.H = grids[j]->h;
        it.T = b.T;
        it.Nv = b.Nv;
        it.win_t = b.win_t;
        it.px = b.top_x.back();
        it.py = b.top_y.back();
        it.pt = b.win_t;
        it.hmax = Hm;
        it.thr_exp = b.thr0;
        it.ranges = scans[j]->d_ranges;
        it.angles = scans[j]->d_angles;
        it.rca = cv.take<double>((size_t)std::max(b.Nv, 1));
        it.rsa = cv.take<double>((size_t)std::max(b.Nv, 1));
        it.tc = cv.take<double>((size_t)b.T);
        it.ts = cv.take<double>((size_t)b.T);
        it.vidx = d_vidx_all + h_vidx.size();
        h_vidx.insert(h_vidx.end(), b.vidx.begin(), b.vidx.end());
        for (int h = 0; h <= Hm; ++h) it.maps[h] = pyr[j][h];
    }
    // host <-> device copies of this path go through the context's pinned
    // buffer (r05: copies to / from fresh pageable vectors stalled a call for
    // 20-28 ms now and then -- the runtime pinning their new pages); each is
    // consumed before the buffer is written again (the stream orders the
    // device side, a sync precedes every host read)
    if (!h_vidx.empty()) {
        int* pv = (int*)ctx->ensure_pinned(sizeof(int) * h_vidx.size());
        std::memcpy(pv, h_vidx.data(), sizeof(int) * h_vidx.size());
        LGS_HIP_CHECK(hipMemcpyAsync(d_vidx_all, pv, sizeof(int) * h_vidx.size(), hipMemcpyHostToDevice,
                                     ctx->stream));
    }
    // guards (shared by every level of the batch)
    // [0] guards, [1] children, [2] overflow; from byte 256 the per-match scored-node counters
    int* d_counts = (int*)ctx->ensure(S_BB3, 256 + sizeof(unsigned long long) * (size_t)n);
    // guard records: guard_cap per 64 matches (the batch grew from 64 to kBBBatch matches)
    const int gcap = ctx->guard_cap * std::max(1, (n + 63) / 64);
    BBGuard* d_guards = (BBGuard*)ctx->ensure(S_BB4, sizeof(BBGuard) * (size_t)std::max(gcap, 1));
    LGS_HIP_CHECK(hipMemsetAsync(d_counts, 0, 256, ctx->stream));

    // pass 1: trig tables and the first descent of every match
    std::vector<int4> path((size_t)n * (Hm + 1));
    for (int j = 0; j < n; ++j)
        for (int h = Hm; h >= 0; --h) {
            const int off = (1 << Hm) - (1 << h);
            path[(size_t)j * (Hm + 1) + (Hm - h)] = make_int4((j << 4) | h, items[j].px + off, items[j].py + off,
                                                              items[j].pt);
        }
    double* d_pscores = (double*)ctx->ensure(S_BB5, sizeof(double) * path.size());
    std::vector<double> pscores(path.size());
    {
        Upload up(ctx);
        const size_t ioff = up.append(items.data(), items.size());
        const size_t poff = up.append(path.data(), path.size());
        up.flush();
        const BBItem* d_items = up.at<BBItem>(ioff);
        dim3 g((std::max(NvMax, Tmax) + 255) / 256, 1, n);
        hipLaunchKernelGGL(k_bb_trig, g, dim3(256), 0, ctx->stream, d_items);
        LGS_HIP_CHECK(hipGetLastError());
        const int np = (int)path.size();
        hipLaunchKernelGGL(k_bb_score, dim3((np + 255) / 256), dim3(256), 0, ctx->stream, d_items,
                           up.at<int4>(poff), np, -1, d_pscores, d_guards, d_counts, gcap, ctx->guard_eps,
                           ctx->inject_index ? 1 : 0);
        LGS_HIP_CHECK(hipGetLastError());
        double* pp = (double*)ctx->ensure_pinned(sizeof(double) * (size_t)np);
        LGS_HIP_CHECK(hipMemcpyAsync(pp, d_pscores, sizeof(double) * np, hipMemcpyDeviceToHost, ctx->stream));
        ctx->sync();
        std::memcpy(pscores.data(), pp, sizeof(double) * (size_t)np);
    }
    // the path scores may carry unchecked guards: they only choose thr_exp,
    // and a wrong choice is caught below (a node missing from the table)
    for (int j = 0; j < n; ++j) {
        bool ok = !no_path;
        for (int k = 0; k <= Hm; ++k) ok &= pscores[(size_t)j * (Hm + 1) + k] > plans[j].thr0;
        items[j].path_ok = ok ? 1 : 0;
        if (ok) items[j].thr_exp = std::max(plans[j].thr0, pscores[(size_t)j * (Hm + 1) + Hm]);
    }
    LGS_HIP_CHECK(hipMemsetAsync(d_counts, 0, 256, ctx->stream));
    lap(0);

    // Guard records [g0, g1) of levels lv0 .. lv1: exact glibc cells; nodes
    // with any differing cell are re-scored from host cells in place (past
    // guard_cap records every node of those levels is re-scored).  Called once
    // after the last level, or (careful) after each level's scoring, before
    // its expansion: then every expansion sees exact scores.
    std::vector<BBLevel> levels((size_t)Hm + 1);   // index = Hm - h
    auto fix_guards = [&](int g0, int g1, int lv0, int lv1) {
        const int ngc = std::max(0, std::min(g1, gcap) - g0);
        std::vector<BBGuard> guards((size_t)ngc);
        std::vector<int4> gnodes((size_t)ngc);
        if (ngc > 0) {
            // the guarded nodes' coordinates, gathered on the device (also
            // past guard_cap: the first gcap records still credit their
            // matches' guard_hits; the nodes are then all re-scored below)
            std::vector<const int4*> lists((size_t)Hm + 1, nullptr);
            for (int l = 0; l <= lv1; ++l) lists[(size_t)l] = levels[(size_t)l].d_nodes;
            Upload ug(ctx);
            const size_t lo = ug.append(lists.data(), lists.size());
            ug.flush();
            int4* d_gn = (int4*)ctx->ensure(S_BB5, sizeof(int4) * (size_t)ngc);
            hipLaunchKernelGGL(k_bb_guard_nodes, dim3((ngc + 255) / 256), dim3(256), 0, ctx->stream,
                               ug.at<const int4*>(lo), d_guards + g0, ngc, d_gn);
            LGS_HIP_CHECK(hipGetLastError());
            const size_t gb = sizeof(BBGuard) * guards.size(), nb = sizeof(int4) * gnodes.size();
            const size_t gbo = (gb + 15) & ~(size_t)15;
            char* pg = (char*)ctx->ensure_pinned(gbo + nb);
            LGS_HIP_CHECK(hipMemcpyAsync(pg, d_guards + g0, gb, hipMemcpyDeviceToHost, ctx->stream));
            LGS_HIP_CHECK(hipMemcpyAsync(pg + gbo, d_gn, nb, hipMemcpyDeviceToHost, ctx->stream));
            ctx->sync();
            std::memcpy(guards.data(), pg, gb);
            std::memcpy(gnodes.data(), pg + gbo, nb);
        }
        std::vector<std::pair<int, int>> dirty;   // (level id, node index)
        std::vector<int4> dnodes;
        if (g1 > gcap) {
            for (int l = lv0; l <= lv1; ++l) {
                const BBLevel& L = levels[(size_t)l];
                std::vector<int4> all((size_t)L.n);
                if (L.n)
                    LGS_HIP_CHECK(hipMemcpy(all.data(), L.d_nodes, sizeof(int4) * (size_t)L.n, hipMemcpyDeviceToHost));
                for (int i = 0; i < L.n; ++i) {
                    dirty.push_back({ l, i });
                    dnodes.push_back(all[(size_t)i]);
                }
            }
        } else {
            std::vector<std::pair<std::pair<int, int>, int4>> dl;
            for (int k = 0; k < ngc; ++k) {
                const BBGuard& g = guards[(size_t)k];
                const int4 nd = gnodes[(size_t)k];
                const int j = nd.x >> 4;
                int ix, iy;
                host_bb_cell(plans[j], grids[j], scans[j], nd.y, nd.z, nd.w, g.v, ix, iy);
                if (ix != g.ix || iy != g.iy) dl.push_back({ { g.level, g.node }, nd });
            }
            std::sort(dl.begin(), dl.end(), [](const auto& a, const auto& b) { return a.first < b.first; });
            for (size_t k = 0; k < dl.size(); ++k)
                if (k == 0 || dl[k].first != dl[k - 1].first) {
                    dirty.push_back(dl[k].first);
                    dnodes.push_back(dl[k].second);
                }
        }
        for (int k = 0; k < ngc; ++k) out[gnodes[(size_t)k].x >> 4].guard_hits += 1;
        if (!dirty.empty()) {
            const int nd_n = (int)dirty.size();
            std::vector<int2> cells((size_t)nd_n * NvMax);
            std::vector<int> nvs((size_t)nd_n), dims((size_t)2 * nd_n);
            std::vector<const double*> maps((size_t)nd_n);
            std::vector<double*> slots((size_t)nd_n);
            for (int k = 0; k < nd_n; ++k) {
                const int4 nd = dnodes[(size_t)k];
                const int j = nd.x >> 4, h = nd.x & 15;
                nvs[k] = plans[j].Nv;
                dims[2 * k] = grids[j]->w;
                dims[2 * k + 1] = grids[j]->h;
                maps[k] = pyr[j][h];
                slots[k] = levels[(size_t)dirty[k].first].d_scores + dirty[k].second;
                for (int v = 0; v < plans[j].Nv; ++v) {
                    int ix, iy;
                    host_bb_cell(plans[j], grids[j], scans[j], nd.y, nd.z, nd.w, v, ix, iy);
                    cells[(size_t)k * NvMax + v] = make_int2(ix, iy);
                }
                out[j].fixups = 1;
            }
            // (the staging is reused by the next upload only after this
            // copy has read it: Upload::copy waits for the stream)
            Upload u2(ctx);
            const size_t co = u2.append(cells.data(), cells.size());
            const size_t no = u2.append(nvs.data(), nvs.size());
            const size_t dof = u2.append(dims.data(), dims.size());
            const size_t mo = u2.append(maps.data(), maps.size());
            const size_t so = u2.append(slots.data(), slots.size());
            u2.flush();
            hipLaunchKernelGGL(k_bb_rescore, dim3(nd_n), dim3(64), 0, ctx->stream, u2.at<const double*>(mo),
                               u2.at<int>(dof), u2.at<int2>(co), u2.at<int>(no), NvMax, u2.at<double*>(so));
            LGS_HIP_CHECK(hipGetLastError());
        }
    };

    // pass 2: level by level, every node the search can visit
    unsigned long long* d_ncount = nullptr;
    {
        std::vector<int4> top;
        for (int j = 0; j < n; ++j)
            for (int x : plans[j].top_x)
                for (int y : plans[j].top_y)
                    for (int t = -plans[j].win_t; t <= plans[j].win_t; ++t)
                        top.push_back(make_int4((j << 4) | Hm, x, y, t));
        Upload up(ctx);
        const size_t ioff = up.append(items.data(), items.size());
        const size_t toff = up.append(top.data(), top.size());
        up.flush();
        const BBItem* d_items = up.at<BBItem>(ioff);
        if (careful) {   // the per-level guard fixes upload through the same slot
            BBItem* keep = (BBItem*)ctx->ensure_aux(3 * (kBBMaxH + 1), sizeof(BBItem) * (size_t)n);
            LGS_HIP_CHECK(hipMemcpyAsync(keep, d_items, sizeof(BBItem) * (size_t)n, hipMemcpyDeviceToDevice,
                                         ctx->stream));
            d_items = keep;
        }
        int gprev = 0;   // careful: guard records already fixed
        // scored nodes per match: its top nodes + 4 per expanded node (k_bb_expand)
        d_ncount = (unsigned long long*)((char*)d_counts + 256);
        LGS_HIP_CHECK(hipMemsetAsync(d_ncount, 0, sizeof(unsigned long long) * (size_t)n, ctx->stream));
        // node/score buffers per level: grown by the host between levels
        int cur_n = (int)top.size();
        int4* cur_nodes = (int4*)ctx->ensure(S_BB1, sizeof(int4) * (size_t)cur_n);
        LGS_HIP_CHECK(hipMemcpyAsync(cur_nodes, up.at<int4>(toff), sizeof(int4) * (size_t)cur_n,
                                     hipMemcpyDeviceToDevice, ctx->stream));
        for (int h = Hm; h >= 0; --h) {
            BBLevel& L = levels[(size_t)(Hm - h)];
            L.n = cur_n;
            L.d_nodes = cur_nodes;
            // per-level buffers: aux 2l = scores, 2l + 1 = the next level's nodes
            L.d_scores = (double*)ctx->ensure_aux(2 * (Hm - h), sizeof(double) * (size_t)std::max(cur_n, 1));
            if (cur_n > 0) {
                // algorithmic bytes: 8 B per (node, valid beam) map lookup
                double lookups = 0.0;
                for (int j = 0; j < n; ++j) lookups += (double)plans[j].Nv;
                const int tok = ctx->timing_begin(K_BB_SCORE, 8.0 * lookups / n * cur_n);
                hipLaunchKernelGGL(k_bb_score, dim3((cur_n + 255) / 256), dim3(256), 0, ctx->stream, d_items,
                                   cur_nodes, cur_n, Hm - h, L.d_scores, d_guards, d_counts, gcap,
                                   ctx->guard_eps, ctx->inject_index ? 1 : 0);
                ctx->timing_end(tok);
                LGS_HIP_CHECK(hipGetLastError());
            }
            if (careful) {   // this level's guards, before its expansion
                int ng = 0;
                LGS_HIP_CHECK(hipMemcpyAsync(&ng, d_counts, sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
                ctx->sync();
                fix_guards(gprev, ng, Hm - h, Hm - h);
                gprev = ng;
            }
            if (h == 0 || cur_n == 0) break;
            const int cap = 4 * cur_n;
            int4* next = (int4*)ctx->ensure_aux(2 * (Hm - h) + 1, sizeof(int4) * (size_t)cap);
            L.d_child = (int*)ctx->ensure_aux(2 * (kBBMaxH + 1) + (Hm - h), sizeof(int) * (size_t)cur_n);
            LGS_HIP_CHECK(hipMemsetAsync(d_counts + 1, 0, 2 * sizeof(int), ctx->stream));
            {
                const int tok = ctx->timing_begin(K_BB_EXPAND, 0.0);
                hipLaunchKernelGGL(k_bb_expand, dim3((cur_n + 255) / 256), dim3(256), 0, ctx->stream, d_items,
                                   cur_nodes, L.d_scores, cur_n, next, d_counts + 1, cap, d_counts + 2, L.d_child,
                                   d_ncount);
                ctx->timing_end(tok);
                LGS_HIP_CHECK(hipGetLastError());
            }
            int cnt[2] = { 0, 0 };
            LGS_HIP_CHECK(hipMemcpyAsync(cnt, d_counts + 1, 2 * sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
            ctx->sync();
            LGS_REQUIRE(cnt[1] == 0, "branch-and-bound: child list overflow");
            cur_n = cnt[0];
            cur_nodes = next;
        }
        if (careful && ctx->profile) ctx->harvest();
        if (!careful) {
            int ng = 0;
            LGS_HIP_CHECK(hipMemcpyAsync(&ng, d_counts, sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
            ctx->sync();
            if (ctx->profile) ctx->harvest();
            fix_guards(0, ng, 0, Hm);
        }
    }
    lap(1);
    // the reference's search (:81-140) over the scored levels on the device
    // (k_bb_replay, one thread per match)
    std::vector<int> top_off((size_t)n + 1, 0);
    std::vector<double> thr0((size_t)n);
    for (int j = 0; j < n; ++j) {
        const BBHost& b = plans[j];
        top_off[(size_t)j + 1] = top_off[(size_t)j] + (int)(b.top_x.size() * b.top_y.size()) * b.T;
        thr0[(size_t)j] = b.thr0;
    }
    BBReplay R;
    std::memset(&R, 0, sizeof(R));
    R.hm = Hm;
    for (int l = 0; l <= Hm; ++l) {
        R.scores[l] = levels[(size_t)l].d_scores;
        R.child[l] = levels[(size_t)l].d_child;
    }
    R.leaves = levels[(size_t)Hm].d_nodes;
    std::vector<BBResult> res((size_t)n);
    std::vector<unsigned long long> ncount((size_t)n);
    {
        Upload ur(ctx);
        const size_t to = ur.append(top_off.data(), top_off.size());
        const size_t ho = ur.append(thr0.data(), thr0.size());
        ur.flush();
        BBResult* d_res = (BBResult*)ctx->ensure(S_BB5, sizeof(BBResult) * (size_t)n);
        hipLaunchKernelGGL(k_bb_replay, dim3((n + kReplayLanes - 1) / kReplayLanes), dim3(64), 0, ctx->stream, R,
                           ur.at<int>(to),
                           ur.at<double>(ho), n, d_res);
        LGS_HIP_CHECK(hipGetLastError());
        const size_t rb = sizeof(BBResult) * (size_t)n, cb = sizeof(unsigned long long) * (size_t)n;
        const size_t rbo = (rb + 15) & ~(size_t)15;
        char* pr = (char*)ctx->ensure_pinned(rbo + cb);
        LGS_HIP_CHECK(hipMemcpyAsync(pr, d_res, rb, hipMemcpyDeviceToHost, ctx->stream));
        LGS_HIP_CHECK(hipMemcpyAsync(pr + rbo, d_ncount, cb, hipMemcpyDeviceToHost, ctx->stream));
        ctx->sync();
        std::memcpy(res.data(), pr, rb);
        std::memcpy(ncount.data(), pr + rbo, cb);
    }
    for (auto& L : levels) L.d_nodes = nullptr, L.d_scores = nullptr, L.d_child = nullptr;
    std::vector<lgs_pose2d> best((size_t)n);
    std::vector<char> failed((size_t)n, 0);
    for (int j = 0; j < n; ++j) {
        const BBHost& b = plans[j];
        const BBResult& r = res[(size_t)j];
        if (r.failed) {
            failed[(size_t)j] = no_path ? 2 : 1;   // 1: rerun with the thr0 superset
            continue;
        }
        const bool got = r.score > b.thr0;   // a leaf was accepted
        const int bx = got ? r.x : 0, by = got ? r.y : 0, bt = got ? r.t : 0;
        const lgs_pose2d bestPose = got ? lgs_pose2d{ b.sensor.x + (double)bx * b.step_x,
                                                      b.sensor.y + (double)by * b.step_y,
                                                      b.sensor.theta + (double)bt * b.step_t }
                                        : b.sensor;
        lgs_rtcsm_summary& o = out[j];
        const int gh = o.guard_hits, fx = o.fixups;
        std::memset(&o, 0, sizeof(o));
        o.guard_hits = gh;
        o.fixups = fx;
        o.pose_found = r.score > b.thr0;   // :142-144
        o.initial_pose = init[j];
        o.score_max = r.score;
        o.score_threshold = b.thr0;
        o.best_win[0] = bx;
        o.best_win[1] = by;
        o.best_win[2] = bt;
        o.win[0] = b.win_x;
        o.win[1] = b.win_y;
        o.win[2] = b.win_t;
        o.steps[0] = b.step_x;
        o.steps[1] = b.step_y;
        o.steps[2] = b.step_t;
        o.best_sensor_pose = bestPose;
        o.coarse_blocks = (int64_t)(top_off[(size_t)j + 1] - top_off[(size_t)j]) + (int64_t)ncount[(size_t)j];
        o.fine_blocks = r.visited;
        best[j] = bestPose;
    }
    for (int j = 0; j < n; ++j)
        LGS_REQUIRE(failed[(size_t)j] != 2, "branch-and-bound: the search reached a node the device did not score");
    lap(2);
    // cost and covariance at the best poses (:146-153), grouped by map
    std::vector<int> order, redo;
    for (int j = 0; j < n; ++j) (failed[(size_t)j] ? redo : order).push_back(j);
    std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return grids[a] < grids[b]; });
    for (size_t k0 = 0; k0 < order.size();) {
        size_t k1 = k0;
        while (k1 < order.size() && grids[order[k1]] == grids[order[k0]]) ++k1;
        std::vector<lgs_scan*> sc;
        std::vector<lgs_pose2d> bp;
        std::vector<lgs_rtcsm_summary> tmp;
        for (size_t k = k0; k < k1; ++k) {
            sc.push_back(scans[order[k]]);
            bp.push_back(best[order[k]]);
            tmp.push_back(out[order[k]]);
        }
        cost_summaries(ctx, grids[order[k0]], cost, sc.data(), bp.data(), (int)sc.size(), tmp.data());
        for (size_t k = k0; k < k1; ++k) out[order[k]] = tmp[k - k0];
        k0 = k1;
    }
    lap(3);
    if (timing) {
        int64_t nodes = 0;
        for (int j = 0; j < n; ++j) nodes += out[j].coarse_blocks;
        std::fprintf(stderr, "bb n=%d nodes=%lld: trig+path %.2f ms, levels %.2f ms, replay %.2f ms, cost %.2f ms\n",
                     n, (long long)nodes, t_ms[0], t_ms[1], t_ms[2], t_ms[3]);
    }
    if (!redo.empty()) {
        std::vector<const lgs_grid*> g2;
        std::vector<const double* const*> p2;
        std::vector<lgs_scan*> s2;
        std::vector<lgs_pose2d> i2;
        for (int j : redo) {
            g2.push_back(grids[j]);
            p2.push_back(pyr[j]);
            s2.push_back(scans[j]);
            i2.push_back(init[j]);
        }
        std::vector<lgs_rtcsm_summary> o2(redo.size());
        run_bb(ctx, p, cost, g2.data(), p2.data(), s2.data(), i2.data(), (int)redo.size(), nthr, o2.data(), true);
        for (size_t k = 0; k < redo.size(); ++k) out[redo[k]] = o2[k];
    }
}

void check_bb(const lgs_bb_params* p, const lgs_cost_ge_params* c)
{
    LGS_REQUIRE(p && c, "null argument");
    LGS_REQUIRE(p->node_height_max >= 0 && p->node_height_max <= kBBMaxH, "node_height_max must be in [0, 12]");
    LGS_REQUIRE(p->range_x >= 0 && p->range_y >= 0 && p->range_theta >= 0, "negative search range");
    LGS_REQUIRE(c->kernel_size >= 0, "negative kernel size");
}

// PrecomputeGridMaps into n_maps x (H+1) scratch maps of S_BB2; returns the pointers
std::vector<std::vector<const double*>> pyramids(lgs_ctx* ctx, const lgs_grid* const* maps, int n_maps, int Hm)
{
    for (int k = 0; k < n_maps; ++k) grid_acquire(ctx, maps[k]);
    size_t total = 0;
    for (int m = 0; m < n_maps; ++m) total += (size_t)(Hm + 1) * align256(sizeof(double) * (size_t)maps[m]->w * maps[m]->h);
    char* base = (char*)ctx->ensure(S_BB2, std::max<size_t>(total, 16));
    std::vector<std::vector<const double*>> out((size_t)n_maps);
    size_t off = 0;
    for (int m = 0; m < n_maps; ++m) {
        for (int h = 0; h <= Hm; ++h) {
            double* d = (double*)(base + off);
            off += align256(sizeof(double) * (size_t)maps[m]->w * maps[m]->h);
            launch_precompute(ctx, maps[m], 1 << h, d, nullptr);
            out[m].push_back(d);
        }
    }
    return out;
}

}  // namespace

extern "C" int lgs_grid_precompute_pyramid(lgs_ctx* ctx, const lgs_grid* in, int node_height_max,
                                           lgs_grid* const* pyramid)
{
    if (!ctx || !in || !pyramid || node_height_max < 0 || node_height_max > kBBMaxH) return LGS_ERR_INVALID_ARG;
    return guarded(ctx, [&] {
        LGS_HIP_CHECK(hipSetDevice(ctx->device));
        for (int h = 0; h <= node_height_max; ++h) {
            LGS_REQUIRE(pyramid[h] && pyramid[h]->w == in->w && pyramid[h]->h == in->h,
                        "pyramid grids must have the input's size");
            launch_precompute(ctx, in, 1 << h, pyramid[h]->d, nullptr);
        }
        ctx->sync();
    });
}

extern "C" int lgs_bb_optimize_pose_batch(lgs_ctx* ctx, const lgs_grid* grid, const lgs_grid* const* pyramid,
                                          const lgs_bb_params* params, const lgs_cost_ge_params* cost,
                                          const lgs_scan* const* scans, const lgs_pose2d* initial, int n,
                                          double nthr, lgs_rtcsm_summary* out)
{
    if (!ctx || !grid || !pyramid || !scans || !initial || !out || n < 0) return LGS_ERR_INVALID_ARG;
    if (n == 0) return LGS_OK;
    return guarded(ctx, [&] {
        check_bb(params, cost);
        std::vector<const double*> pyr;
        for (int h = 0; h <= params->node_height_max; ++h) {
            LGS_REQUIRE(pyramid[h] && pyramid[h]->w == grid->w && pyramid[h]->h == grid->h,
                        "pyramid grids must have the map's size");
            pyr.push_back(pyramid[h]->d);
        }
        std::vector<const double* const*> pp((size_t)n, pyr.data());
        std::vector<const lgs_grid*> grids((size_t)n, grid);
        std::vector<lgs_scan*> sc((size_t)n);
        for (int j = 0; j < n; ++j) {
            LGS_REQUIRE(scans[j] && scans[j]->n >= 1, "empty scan");
            sc[j] = const_cast<lgs_scan*>(scans[j]);
        }
        for (int j0 = 0; j0 < n; j0 += kBBBatch) {
            const int m = std::min(kBBBatch, n - j0);
            run_bb(ctx, params, cost, grids.data() + j0, pp.data() + j0, sc.data() + j0, initial + j0, m, nthr,
                   out + j0);
        }
    });
}

extern "C" int lgs_bb_optimize_pose_query(lgs_ctx* ctx, const lgs_grid* grid, const lgs_bb_params* params,
                                          const lgs_cost_ge_params* cost, const lgs_scan* scan,
                                          lgs_pose2d initial, lgs_rtcsm_summary* out)
{
    if (!ctx || !grid || !scan || !out) return LGS_ERR_INVALID_ARG;
    return guarded(ctx, [&] {
        check_bb(params, cost);
        LGS_REQUIRE(scan->n >= 1, "empty scan");
        auto pyr = pyramids(ctx, &grid, 1, params->node_height_max);   // ComputeCoarserMaps (:157-165)
        const double* const* pp = pyr[0].data();
        lgs_scan* s = const_cast<lgs_scan*>(scan);
        run_bb(ctx, params, cost, &grid, &pp, &s, &initial, 1, DBL_MIN, out);
    });
}

extern "C" int lgs_loop_detect_bb(lgs_ctx* ctx, const lgs_bb_params* params, const lgs_cost_ge_params* cost,
                                  double score_threshold, const lgs_loop_query* queries, int num_queries,
                                  const lgs_loop_candidate* candidates, int num_candidates,
                                  lgs_loop_result* results)
{
    if (!ctx || !params || !cost || (num_queries > 0 && !queries) || num_queries < 0 || num_candidates < 0 ||
        (num_candidates > 0 && (!candidates || !results)))
        return LGS_ERR_INVALID_ARG;
    return guarded(ctx, [&] {
        check_bb(params, cost);
        LGS_REQUIRE(score_threshold > 0.0 && score_threshold <= 1.0, "score threshold must be in (0, 1] (:18-19)");
        int covered = 0;
        for (int q = 0; q < num_queries; ++q) {
            const lgs_loop_query& Q = queries[q];
            LGS_REQUIRE(Q.map, "loop query without a local map");
            LGS_REQUIRE(Q.first_candidate == covered && Q.num_candidates >= 0 &&
                            Q.first_candidate + Q.num_candidates <= num_candidates,
                        "loop queries must cover the candidates contiguously and in order");
            covered += Q.num_candidates;
            for (int j = 0; j < Q.num_candidates; ++j)
                LGS_REQUIRE(candidates[Q.first_candidate + j].scan, "loop candidate without a scan");
        }
        LGS_REQUIRE(covered == num_candidates, "loop queries must cover every candidate");
        // batches of whole queries, at most ~kBBBatch candidates: each query's
        // pyramid once per batch (LocalMapInfo caches it, :45-55)
        for (int q0 = 0; q0 < num_queries;) {
            int q1 = q0, m = 0;
            while (q1 < num_queries && (m == 0 || m + queries[q1].num_candidates <= kBBBatch))
                m += queries[q1++].num_candidates;
            std::vector<const lgs_grid*> qmaps;
            for (int q = q0; q < q1; ++q) qmaps.push_back(queries[q].map);
            auto pyr = pyramids(ctx, qmaps.data(), (int)qmaps.size(), params->node_height_max);
            std::vector<const lgs_grid*> grids;
            std::vector<const double* const*> pp;
            std::vector<lgs_scan*> sc;
            std::vector<lgs_pose2d> poses;
            std::vector<int> cand, qof;
            for (int q = q0; q < q1; ++q)
                for (int j = 0; j < queries[q].num_candidates; ++j) {
                    const lgs_loop_candidate& c = candidates[queries[q].first_candidate + j];
                    grids.push_back(queries[q].map);
                    pp.push_back(pyr[(size_t)(q - q0)].data());
                    sc.push_back(const_cast<lgs_scan*>(c.scan));
                    poses.push_back(c.node_pose);
                    cand.push_back(queries[q].first_candidate + j);
                    qof.push_back(q);
                }
            std::vector<lgs_rtcsm_summary> sums(cand.size());
            if (!cand.empty())
                run_bb(ctx, params, cost, grids.data(), pp.data(), sc.data(), poses.data(), (int)cand.size(),
                       score_threshold, sums.data());
            for (size_t k = 0; k < cand.size(); ++k) {
                const lgs_loop_query& Q = queries[qof[k]];
                lgs_loop_result& r = results[cand[k]];
                std::memset(&r, 0, sizeof(r));
                const lgs_rtcsm_summary& s = sums[k];
                r.found = s.pose_found;   // FindCorrespondingPose (:99-117)
                r.start_node_index = Q.local_map_node_index;
                r.end_node_index = candidates[cand[k]].node_index;
                r.start_node_pose = Q.local_map_node_pose;
                r.estimated_pose = s.estimated_pose;
                r.score = s.score_max;
                r.normalized_cost = s.normalized_cost;
                if (s.pose_found) r.relative_pose = inverse_compound(Q.local_map_node_pose, s.estimated_pose);
                std::memcpy(r.covariance, s.covariance, sizeof(r.covariance));
            }
            q0 = q1;
        }
    });
}
