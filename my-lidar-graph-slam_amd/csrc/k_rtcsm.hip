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
//               (c > thr) && (unsafe || c >= L)  -> ordered list, compacted per
//               1024-block segment (ballot + LDS prefix); consumers rebuild the
//               segment prefix in LDS, so no separate scan pass is needed.
//   k_fine      EvaluateHighResolutionMap (:227-256) for listed blocks: block
//               max and its first position in the reference's (x, y) order.
//   k_replay    the reference's acceptance rule `c > s && f > s` replayed in
//               block order over the list; detects the one case the pruning
//               proof does not cover (unsafe block with c < L <= f) and asks
//               the host for an exact dense rerun.
//   k_cost_*    CostGreedyEndpoint::Cost at the best pose and its six
//               central-difference neighbours (C/mapping/cost_function_greedy_endpoint.cpp:32-171).
#include "lgs_internal.hpp"

#include <algorithm>
#include <cfloat>
#include <cstring>
#include <map>
#include <mutex>
#include <thread>
#include <type_traits>

using namespace lgs;

namespace lgs {
void launch_precompute(lgs_ctx* ctx, const lgs_grid* in, int win, double* out, const PlaneGeom* planes);
void launch_precompute_jobs(lgs_ctx* ctx, const PrecompJob* d_jobs, int njobs, int maxW, int maxH, int win);
bool precompute_planes_ok(const lgs_grid* in, int win);
void precompute_tile_grid(int maxW, int maxH, int win, int njobs, int* gx, int* gy, int* rows);
}

namespace {


// Superblock plane element: fp16 rounded toward +inf from the fp64 maxima, so
// every stored value is >= the coarse values it bounds (the bound's sum is
// taken in fp64).
typedef _Float16 SuperT;   // built from the planes' fp16 round-up copies (half_round_up_bits)

constexpr int kMaxBatchItems = 64;   // matches per batched launch chain (run_chunked)
constexpr int kPipe = 16;   // seq_sum gathers in flight per batch (index arrays padded by 2*kPipe)
constexpr int kPad = 4 * kPipe;   // cbase padding past the last row (seq_sum4's look-ahead)

// One match of a batched launch (DESIGN.md §3 "batched matching").  A batch's
// items are uploaded once to device memory; every stage is ONE launch for the
// whole batch, a grid dimension selecting the item, and each workgroup reads
// its item through a `const __restrict__` kernel argument with a uniform index
// (scalar loads).  Items of one batch share the search parameters (P, ncx,
// ncy, nsb2, low_res); T and Nv differ per scan (grids use the maxima and
// workgroups past an item's extent exit).  Items matching against the same
// map share its coarse planes (cmap/super/negflag/pgen).
struct MatchItem {
    RtcsmPlan pl;
    CostPlan cp;
    const double* grid;      // fine map
    const double* ranges;
    const double* angles;
    const double* cmap;      // coarse map: padded phase planes (or the plain map)
    const SuperT* super;     // superblock planes of cmap (SuperT, rounded up)
    const int* negflag;      // stamped with pgen when the planes hold a negative cell
    int pgen;                // build stamp of the planes
    int gen;                 // this match's generation stamp
    RtcsmRecord* rec;
    int* keepc;              // this item's two work-list counters (k_keep; null: no list), zeroed by k_seed_super
    int2* idx;
    int* cbase;
    int* tedge;
    double* cscore;
    uint8_t* cflag;
    int* list;
    int* segcnt;
    int nseg;
    int* dlist;              // selected blocks, dense in block order (k_compact)
    int* nsel;               // their number
    int frows;
    double* fval;
    int* fpos;
    double* part_c;
    long long* part_k;
    int nparts;
    double* Lp;
    double* Lc;
    double* seedm;           // wide seed: nseedm (coarse score, block, sum of |terms|) triples
    int nseedm;              // candidates of the wide seed (k_seed_members workgroups)
    double* sbound;
    double* poses7;
    int4* cidx;
    double* terms;
    // lean projection (LGS_OPT_LEAN_PROJECT): k_project
    // does not run; k_beams writes these two tables and every kernel that
    // stages a superblock-base, coarse-base or cell row forms it itself
    // (lean_super_row / lean_cell: k_project's arithmetic, bit for bit)
    double4* btab;           // per valid beam v: range, cos, sin of its angle (glibc-free ocml sincos, as k_project)
    double2* atab;           // per search angle t: cos, sin of the sensor angle
    int lean;                // 1: no (angle, beam) row (idx, cbase) is written
    int inject;              // LGS_OPT_INJECT_INDEX (tests): a guarded projection's x index + 1
    int gcap;                // guard records the record holds (guard_cap)
    double geps;             // the projection guard's epsilon (near_boundary)
};
typedef const MatchItem* __restrict__ Items;

// XCD-aware workgroup order (speed only, never correctness).  Blocks b and
// b + 8 are observed to share an XCD (round-robin dispatch, MI355X_MICROARCH.md
// §Workgroup dispatch); the bijective remap gives each XCD a contiguous range
// of logical workgroups, x fastest, then y, then z.  Grids order their
// dimensions so that an item's (one map's) workgroups are contiguous: they
// then meet in one XCD's L2 instead of all eight.  Only for kernels whose
// workgroups carry even work (k_super, k_super_planes, k_project, the
// precompute): where the work concentrates on few workgroups of an item
// (k_coarse_rows, k_fine) the remap loads one XCD and idles the rest.
struct Blk {
    int x, y, z;
};
__device__ __forceinline__ Blk xcd_block()
{
    const int gx = gridDim.x, gy = gridDim.y, gz = gridDim.z;
    const int nwg = gx * gy * gz;
    const int b = blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z);
    const int xcd = b & 7, q = nwg >> 3, r = nwg & 7;
    const int l = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (b >> 3);
    // uniform by construction; readfirstlane tells the compiler, so that a
    // descriptor indexed by it is read with scalar loads (hoisted out of
    // loops) instead of per-iteration vector loads (seen in k_project)
    return { __builtin_amdgcn_readfirstlane(l % gx), __builtin_amdgcn_readfirstlane((l / gx) % gy),
             __builtin_amdgcn_readfirstlane(l / (gx * gy)) };
}

// Per-set superblock-plane job: one coarse map's padded phase planes.
struct PlaneJob {
    RtcsmPlan pl;            // layout fields (Wqp, Hqp, pstride, pstride4, sub4, Wq4)
    const unsigned short* planes16;   // the planes rounded up to fp16 (same layout)
    SuperT* super;
    unsigned* zt;   // k_super_hv's zero-tile words of this set (null: none), see ZeroTiles
    int* negflag;   // stamped with pgen when a bound value exceeds 1 (8-bit units cannot hold it)
    int pgen;
};

// 8-bit superblock units (r06, octet layouts): 4 fp16 round-up maxima (bits
// 16 i of v, i < 4) -> 4 bytes ceil(255 h) (exact: h has 11 significant
// bits, so 255 h is exact in fp32, and ceil(255 h) / 255 >= h).  The bound is
// then an exact integer sum / 255 (no fp32 partials).  A value above 1 (not an
// occupancy probability) sets *over: the set's bounds are disabled (negflag,
// as for negative cells).  Bit patterns of +0 and positive fp16 values order
// like the values, so the maxima taken on them stay maxima here.
__device__ __forceinline__ unsigned quad_u8(unsigned long long v, bool& over)
{
    unsigned r = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const float h = (float)__builtin_bit_cast(_Float16, (unsigned short)(v >> (16 * i)));
        over |= h > 1.0f;
        const float q = fminf(fmaxf(ceilf(h * 255.0f), 0.0f), 255.0f);
        r |= (unsigned)q << (8 * i);
    }
    return r;
}

// The fp16 round-up copy of padded planes and the negative-cell stamp, for
// planes the batched precompute did not write (phase-plane copies of
// supplied or odd-sized coarse maps, windows > 8): one thread per cell.
__global__ __launch_bounds__(256) void k_planes16(const double* __restrict__ P, unsigned short* __restrict__ P16,
                                                  long long n, int* __restrict__ negflag, int pgen)
{
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double v = P[i];
    P16[i] = half_round_up_bits(v);
    if (v < 0.0) *negflag = pgen;
}

// Generation-tagged counter (gen << 32 | count): a word left by an earlier
// match counts as zero, so records need no memset.  Returns this caller's slot.
__device__ __forceinline__ int tagged_add(unsigned long long* w, unsigned gen, unsigned k)
{
    unsigned long long cur = *(volatile unsigned long long*)w, assumed;
    unsigned cnt;
    do {
        assumed = cur;
        cnt = ((unsigned)(assumed >> 32) == gen) ? (unsigned)assumed : 0u;
        cur = atomicCAS(w, assumed, ((unsigned long long)gen << 32) | (unsigned long long)(cnt + k));
    } while (cur != assumed);
    return (int)cnt;
}

// Slot of a guard record: the active lanes with want = true take consecutive
// slots with ONE compare-and-swap loop per wave (a loop per lane on one
// address serialises thousands of retries when many hit points sit on cell
// boundaries: axis-aligned walls, measured 7 ms per k_cost launch).  Every
// active lane must call it; lanes without a record get -1.
__device__ __forceinline__ int tagged_slot_wave(unsigned long long* w, unsigned gen, bool want)
{
    const unsigned long long m = __ballot(want);
    if (m == 0ull) return -1;
    const int lane = (int)__lane_id();
    const int leader = __ffsll((unsigned long long)m) - 1;
    int base = 0;
    if (lane == leader) base = tagged_add(w, gen, (unsigned)__popcll(m));
    base = __shfl(base, leader, 64);
    return want ? base + (int)__popcll(m & ((1ull << lane) - 1ull)) : -1;
}

__device__ __forceinline__ bool near_boundary(double q, double eps)
{
    const double f = q - floor(q);
    const double e = eps + fabs(q) * 1e-13;
    return f < e || f > 1.0 - e;
}

// --------------------------------------------------------------------------
// k_project: idx[t][v] = WorldCoordinateToGridCellIndex(HitPoint(pose_t, beam))
// --------------------------------------------------------------------------

// floor(a / b) and the remainder in [0, b) for a runtime divisor b > 0
// (any int a): one fp64 multiply by 1/b, floor and a +-1 correction -- exact,
// and a fraction of the two branchy integer divisions it replaces (k_project
// spent most of its VALU issue on those)
__device__ __forceinline__ void floor_divmod(int a, int b, double inv_b, int& q, int& r)
{
    q = (int)floor((double)a * inv_b);
    r = a - q * b;
    if (r < 0) {
        --q;
        r += b;
    } else if (r >= b) {
        ++q;
        r -= b;
    }
}

// A beam's coarse lattice start bx = ix - winX, by = iy - winY as (plane
// column qx0 = floor(bx / lr), plane row qy0, phase rx = bx mod lr, ry).
struct BeamLattice {
    int qx0, qy0, rx, ry;
};
__device__ __forceinline__ BeamLattice beam_lattice(int ix, int iy, const RtcsmPlan& pl, double inv_lr)
{
    BeamLattice b;
    floor_divmod(ix - pl.win_x, pl.low_res, inv_lr, b.qx0, b.rx);
    floor_divmod(iy - pl.win_y, pl.low_res, inv_lr, b.qy0, b.ry);
    return b;
}

// Per (angle, beam) base offset of the coarse stage in the padded phase-plane
// layout (see k_decimate): the beam's lattice start lies in plane (rx, ry) at
// (qx0, qy0).  If its ncx x ncy window touches the map, the window lies
// inside the M-wide zero margins (M >= ncx, ncy) and the base is direct;
// otherwise every read is 0.0 (GridMap::Value out of bounds) and the base
// points at the all-zero top-left margin of plane 0.  The coarse lanes then
// read base + jy * Wqp + jx with no bounds test.
__device__ __forceinline__ int coarse_base_l(const BeamLattice& b, const RtcsmPlan& pl)
{
    const int lr = pl.low_res;
    const bool touches = (b.qx0 < pl.Wq) & (b.qx0 + pl.ncx > 0) & (b.qy0 < pl.Hq) & (b.qy0 + pl.ncy > 0);
    return touches ? (int)((b.ry * lr + b.rx) * pl.pstride + (long long)(b.qy0 + pl.M) * pl.Wqp + (b.qx0 + pl.M)) : 0;
}

// Superblock base of the same beam in the compact superblock planes: the
// padded position (Qx, Qy) of its lattice start, in sub-phase (Qx & 3, Qy & 3)
// at (Qx >> 2, Qy >> 2); superblock (a, b) is then base + b * Wq4 + a.  0 (an
// all-zero margin corner) when the coarse window misses the map.
__device__ __forceinline__ int super_base_l(const BeamLattice& b, const RtcsmPlan& pl)
{
    const int lr = pl.low_res;
    const int qx0 = b.qx0, qy0 = b.qy0, rx = b.rx, ry = b.ry;
    // the strip qx = -1 (rx > 0) / qy = -1 (ry > 0) holds the clamped values
    // of k_super_planes: a window that reaches only the strip still counts
    const bool touches = (qx0 < pl.Wq) & (qx0 + pl.ncx > (rx > 0 ? -1 : 0)) & (qy0 < pl.Hq) &
                         (qy0 + pl.ncy > (ry > 0 ? -1 : 0));
    const int Qx = qx0 + pl.M, Qy = qy0 + pl.M;
    if (pl.oct) {
        const int Yr = Qy >> 2;
        return touches ? (int)((((ry * lr + rx) * pl.pstrideO + ((Qy & 3) * 4 + (Qx & 3)) * pl.subO +
                                 (long long)(Yr >> 2) * pl.Wq4 + (Qx >> 2)) << 2) | (Yr & 3))
                       : 0;
    }
    return touches ? (int)((ry * lr + rx) * pl.pstride4 + ((Qy & 3) * 4 + (Qx & 3)) * pl.sub4 +
                           (long long)(Qy >> 2) * pl.Wq4 + (Qx >> 2))
                   : 0;
}

// Checked build (LGS_CHECK_OFFSETS: liblgs_hip_checked.so, VERDICT r05 item
// 5): the consumers test every coarse / superblock base they form or read
// against its padded plane before using it -- the window a base opens must
// lie inside one plane (coarse: ncx x ncy cells from the base; superblock:
// nsbx units from the base's unit).  Checks are counted per wave; a
// violation is counted and the first one kept (kind << 60 | t << 32 | v, base),
// read back by lgs_debug_offset_checks.  Round 5's "nowrite" variant read
// unwritten rows as bases and faulted: such a row would
// land here as a counted violation, not as an illegal address.
#ifdef LGS_CHECK_OFFSETS
__device__ unsigned long long g_offchk[4];   // checked, violations, first (kind|t|v), first base
__device__ __forceinline__ void offchk_note(bool ok, int kind, int t, int v, long long base)
{
    const unsigned long long act = __ballot(1), bad = __ballot(!ok);
    const int lane = (int)__lane_id();
    if (lane == __ffsll((long long)act) - 1) {
        atomicAdd(&g_offchk[0], (unsigned long long)__popcll(act));
        if (bad) atomicAdd(&g_offchk[1], (unsigned long long)__popcll(bad));
    }
    if (!ok && atomicCAS(&g_offchk[2], 0ull,
                         ((unsigned long long)kind << 60) | ((unsigned long long)(unsigned)t << 32) | (unsigned)v) == 0ull)
        g_offchk[3] = (unsigned long long)base;
}
__device__ __forceinline__ void chk_coarse(const RtcsmPlan& pl, int b, int t, int v)
{
    const long long all = (long long)pl.low_res * pl.low_res * pl.pstride;
    bool ok = b >= 0 && b < all;
    if (ok) {
        const long long o = b % pl.pstride;
        ok = o / pl.Wqp + pl.ncy <= pl.Hqp && o % pl.Wqp + pl.ncx <= pl.Wqp;
    }
    offchk_note(ok, 1, t, v, b);
}
__device__ __forceinline__ void chk_super(const RtcsmPlan& pl, int c, int t, int v)
{
    bool ok;
    if (pl.oct) {
        const long long u = (long long)(c >> 2), all = (long long)pl.low_res * pl.low_res * pl.pstrideO;
        ok = c >= 0 && u + pl.nsbx <= all && u % pl.Wq4 + pl.nsbx <= pl.Wq4;
    } else {
        const long long all = (long long)pl.low_res * pl.low_res * pl.pstride4;
        ok = c >= 0 && (long long)c + (long long)(pl.nsby - 1) * pl.Wq4 + pl.nsbx <= all &&
             c % pl.Wq4 + pl.nsbx <= pl.Wq4;
    }
    offchk_note(ok, 2, t, v, c);
}
#define LGS_CHK_COARSE(pl, b, t, v) chk_coarse(pl, b, t, v)
#define LGS_CHK_SUPER(pl, c, t, v) chk_super(pl, c, t, v)
#else
#define LGS_CHK_COARSE(pl, b, t, v) ((void)0)
#define LGS_CHK_SUPER(pl, c, t, v) ((void)0)
#endif

__device__ __forceinline__ int coarse_base(int ix, int iy, const RtcsmPlan& pl)
{
    return coarse_base_l(beam_lattice(ix, iy, pl, 1.0 / pl.low_res), pl);
}
__device__ __forceinline__ int super_base(int ix, int iy, const RtcsmPlan& pl)
{
    return super_base_l(beam_lattice(ix, iy, pl, 1.0 / pl.low_res), pl);
}

// Coarse value C(x, y) of an in-map coarse cell in the padded phase planes.
__device__ __forceinline__ double coarse_at(const double* __restrict__ cmap, int x, int y, const RtcsmPlan& pl)
{
    const int lr = pl.low_res;
    return cmap[(long long)((y % lr) * lr + x % lr) * pl.pstride + (long long)(y / lr + pl.M) * pl.Wqp +
                (x / lr + pl.M)];
}

// One beam of the unsafe test of block (x0, y0) (its coarse read at x, y):
// true if the read lies in the strip left of / below the map while the
// block's fine reads of the beam overlap the map.  Then C(max(x, 0),
// max(y, 0)) bounds those fine reads and is added to ext.
__device__ __forceinline__ bool strip_read(const double* __restrict__ cmap, int x, int y, const RtcsmPlan& pl,
                                           double& ext)
{
    const int lo = -(pl.low_res - 1);
    const bool s = (x >= lo) & (x < pl.W) & (y >= lo) & (y < pl.H) & ((x < 0) | (y < 0));
    if (s) ext += coarse_at(cmap, max(x, 0), max(y, 0), pl);
    return s;
}

// blockDim == 256.  ComputeScanIndices keeps the beams with range <
// ScanRangeMax, in beam order (:192-193); each block finds its 256 valid
// beams v0..v0+255 with a block-wide prefix count over the scan (no host
// upload of the compaction), then projects them for kProjRows search angles
// (fewer, longer waves: the GPU's wave slots, not its ALUs, are what
// concurrent matches compete for).
// cos/sin(th_t + a_i) by rotation: one sincos per beam and one per search
// angle (shared through LDS) instead of one per (angle, beam).  The rotation
// differs from glibc's cos/sin of the rounded sum th_t + a_i by a few ulps
// plus the rounding of that sum (<= 2^-53 |th + a|): with ranges <= 100 m and
// cells >= 1 mm that is < 1e-11 cells, far inside the 1e-9-cell guard, so
// every projection whose glibc floor could differ is still guarded and
// re-checked on the host.
constexpr int kProjRows = 16;
constexpr int kProjRowsLone = 4;   // measured (lone config-2 scan): 16: 16.1 us, 8: 12.3, 4: 10.7, 2: 10.4
template <int ROWS>
__global__ __launch_bounds__(256) void k_project(Items items, int guard_cap, double guard_eps, int inject, DevTs dts)
{
    const DtsScope dts_scope(dts);
    const Blk wg = xcd_block();
    const MatchItem& it = items[wg.z];
    const RtcsmPlan& pl = it.pl;
    if (wg.y * ROWS >= pl.T) return;   // past this item's angles (uniform)
    const double* __restrict__ ranges = it.ranges;
    const double* __restrict__ angles = it.angles;
    // global (not flat) stores: the item's pointers come through a struct
    typedef __attribute__((address_space(1))) unsigned long long gu64_t;   // int2 {x, y}: x in the low half
    typedef __attribute__((address_space(1))) int gint_t;
    gu64_t* __restrict__ idx = (gu64_t*)it.idx;
    gint_t* __restrict__ cbase = (gint_t*)it.cbase;
    gint_t* __restrict__ tedge = (gint_t*)it.tedge;
    const int gen = it.gen;
    RtcsmRecord* rec = it.rec;
    __shared__ int s_map[256];
    __shared__ int s_wsum[4];
    __shared__ double s_ct[ROWS], s_st[ROWS];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    if (tid < ROWS) {
        // currentSensorPose.mTheta = sensorPose.mTheta + stepTheta * t (:90-91)
        const int t = wg.y * ROWS + tid - pl.win_t;
        const double th = pl.st + pl.step_t * (double)t;
        double sn, cs;
        sincos(th, &sn, &cs);
        s_ct[tid] = cs;
        s_st[tid] = sn;
    }
    const int v0 = wg.x * 256;
    const int chunk = (pl.N + 255) / 256;
    const int lo = min(tid * chunk, pl.N), hi = min(lo + chunk, pl.N);
    int nvalid = 0;
    for (int i = lo; i < hi; ++i) nvalid += !(ranges[i] >= pl.rmax);
    int incl = nvalid;
    for (int off = 1; off < 64; off <<= 1) {
        const int t = __shfl_up(incl, off, 64);
        if (lane >= off) incl += t;
    }
    if (lane == 63) s_wsum[wid] = incl;
    __syncthreads();
    int pos = incl - nvalid;
    for (int j = 0; j < wid; ++j) pos += s_wsum[j];
    for (int i = lo; i < hi; ++i)
        if (!(ranges[i] >= pl.rmax)) {
            const int r = pos - v0;
            if (r >= 0 && r < 256) s_map[r] = i;
            ++pos;
        }
    __syncthreads();
    const int v = v0 + tid;
    // seq_sum's look-ahead reads up to kPad entries past the last row:
    // keep them at the zero margin (base 0)
    if (wg.x == 0 && wg.y == 0 && tid < kPad) {
        cbase[(size_t)pl.T * pl.Nv + tid] = 0;
        cbase[pl.sb_off + (size_t)pl.T * pl.Nv + tid] = 0;
    }
    if (v >= pl.Nv) return;
    const int i = s_map[tid];
    const double r = ranges[i];
    const double a = angles[i];
    double sa, ca;
    sincos(a, &sa, &ca);
    const int tt1 = min(pl.T, (wg.y + 1) * ROWS);
    const double inv_res = 1.0 / pl.res;
    const double inv_lr = 1.0 / pl.low_res;
    for (int tt = wg.y * ROWS; tt < tt1; ++tt) {
    // HitPoint: cos(sensorPose.mTheta + scanAngle) (H/sensor/sensor_data.hpp:168-172),
    // by rotation (see ROWS)
    const int kr = tt - wg.y * ROWS;
    const double c = s_ct[kr] * ca - s_st[kr] * sa;
    const double s = s_st[kr] * ca + s_ct[kr] * sa;
    const double hx = pl.sx + r * c;
    const double hy = pl.sy + r * s;
    // x / res as x * (1 / res): differs from the quotient by a few ulps, far
    // inside the guard (eps + |q| 1e-13), so every cell whose floor could
    // differ from the reference's division is still re-checked on the host
    const double qx = (hx - pl.min_x) * inv_res;
    const double qy = (hy - pl.min_y) * inv_res;
    int ix = (int)floor(qx);
    int iy = (int)floor(qy);
    const bool guarded = near_boundary(qx, guard_eps) || near_boundary(qy, guard_eps);
    const int slot = tagged_slot_wave(&rec->guard_word, (unsigned)gen, guarded);
    if (guarded) {
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
    const size_t o = (size_t)tt * pl.Nv + v;
    idx[o] = ((unsigned long long)(unsigned)iy << 32) | (unsigned)ix;
    const BeamLattice bl = beam_lattice(ix, iy, pl, inv_lr);
    cbase[o] = coarse_base_l(bl, pl);
    cbase[pl.sb_off + o] = super_base_l(bl, pl);
    // this angle has a beam whose coarse lattice starts left of / below the
    // map: k_coarse must run its unsafe-block check (generation-stamped flag;
    // one store per wave and angle)
    const unsigned long long edge = __ballot(ix - pl.win_x < 0 || iy - pl.win_y < 0);
    if (edge && lane == __ffsll((long long)edge) - 1) tedge[tt] = gen;
    }
}

// Lean projection: the cell of (angle t, valid beam v)
// from the tables k_project wrote, with k_project's arithmetic operation for
// operation (-ffp-contract=off: the same roundings, so the same bits), its
// guard test included (LGS_OPT_INJECT_INDEX shifts a guarded x index here
// exactly as there).  Only batches whose every consumer forms its rows this
// way run lean (lean_rows on the host); guard fix-up reruns and lone matches
// materialise the rows.
__device__ __forceinline__ int2 lean_cell(const MatchItem& it, int t, int v)
{
    const RtcsmPlan& pl = it.pl;
    const double4 b = it.btab[v];   // r, cos a, sin a
    const double2 a = it.atab[t];   // cos th_t, sin th_t
    const double c = a.x * b.y - a.y * b.z;
    const double s = a.y * b.y + a.x * b.z;
    const double hx = pl.sx + b.x * c;
    const double hy = pl.sy + b.x * s;
    const double inv_res = 1.0 / pl.res;
    const double qx = (hx - pl.min_x) * inv_res;
    const double qy = (hy - pl.min_y) * inv_res;
    int ix = (int)floor(qx);
    const int iy = (int)floor(qy);
    if (it.inject && (near_boundary(qx, it.geps) || near_boundary(qy, it.geps))) ix += it.inject;
    return make_int2(ix, iy);
}
__device__ __forceinline__ int lean_coarse_base(const MatchItem& it, int t, int v)
{
    const int2 q = lean_cell(it, t, v);
    return coarse_base_l(beam_lattice(q.x, q.y, it.pl, 1.0 / it.pl.low_res), it.pl);
}

// Lean batches (r06): k_beams replaces k_project -- per item, the valid-beam
// compaction (ComputeScanIndices' filter, :192-193) and the two tables
// (range, cos, sin per valid beam: one sincos per beam; cos, sin per search
// angle) -- and k_super_oct forms each angle's superblock-base row in LDS
// with k_project's arithmetic (lean_super_row), records its guarded
// projections and the angle's edge flag: no (angle, beam) row is written to
// memory at all (k_project wrote 4-16 B per (angle, beam), 0.085-0.106 ms
// per 64 config-2 queries).  Grid (ceil(NvMax / 256), 1, items).
__global__ __launch_bounds__(256) void k_beams(Items items, DevTs dts)
{
    const DtsScope dts_scope(dts);
    const MatchItem& it = items[blockIdx.z];
    const RtcsmPlan& pl = it.pl;
    const double* __restrict__ ranges = it.ranges;
    const double* __restrict__ angles = it.angles;
    __shared__ int s_map[256];
    __shared__ int s_wsum[4];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    if (blockIdx.x == 0)
        for (int tt = tid; tt < pl.T; tt += 256) {
            // currentSensorPose.mTheta = sensorPose.mTheta + stepTheta * t (:90-91), as k_project
            const double th = pl.st + pl.step_t * (double)(tt - pl.win_t);
            double sn, cs;
            sincos(th, &sn, &cs);
            it.atab[tt] = make_double2(cs, sn);
        }
    const int v0 = blockIdx.x * 256;
    if (v0 >= pl.Nv) return;   // past this item's valid beams (uniform)
    const int chunk = (pl.N + 255) / 256;
    const int lo = min(tid * chunk, pl.N), hi = min(lo + chunk, pl.N);
    int nvalid = 0;
    for (int i = lo; i < hi; ++i) nvalid += !(ranges[i] >= pl.rmax);
    int incl = nvalid;
    for (int off = 1; off < 64; off <<= 1) {
        const int u = __shfl_up(incl, off, 64);
        if (lane >= off) incl += u;
    }
    if (lane == 63) s_wsum[wid] = incl;
    __syncthreads();
    int pos = incl - nvalid;
    for (int j = 0; j < wid; ++j) pos += s_wsum[j];
    for (int i = lo; i < hi; ++i)
        if (!(ranges[i] >= pl.rmax)) {
            const int r = pos - v0;
            if (r >= 0 && r < 256) s_map[r] = i;
            ++pos;
        }
    __syncthreads();
    const int v = v0 + tid;
    if (v >= pl.Nv) return;
    const int i = s_map[tid];
    double sa, ca;
    sincos(angles[i], &sa, &ca);
    it.btab[v] = make_double4(ranges[i], ca, sa, 0.0);
}

// The superblock-base row of angle t into LDS (block-wide), with k_project's
// guard records (gen-tagged slots of the item's record, the injected index
// shift of LGS_OPT_INJECT_INDEX) and the angle's edge flag.  Every thread of
// the block must call it (a barrier inside).
__device__ __forceinline__ void lean_super_row(const MatchItem& it, int t, int* srow)
{
    const RtcsmPlan& pl = it.pl;
    RtcsmRecord* rec = it.rec;
    const double inv_res = 1.0 / pl.res, inv_lr = 1.0 / pl.low_res;
    const double2 at = it.atab[t];
    int edge = 0;
    for (int v = threadIdx.x; v < pl.Nv; v += blockDim.x) {
        const double4 b = it.btab[v];
        const double c = at.x * b.y - at.y * b.z;
        const double s = at.y * b.y + at.x * b.z;
        const double hx = pl.sx + b.x * c;
        const double hy = pl.sy + b.x * s;
        const double qx = (hx - pl.min_x) * inv_res;
        const double qy = (hy - pl.min_y) * inv_res;
        int ix = (int)floor(qx);
        const int iy = (int)floor(qy);
        const bool guarded = near_boundary(qx, it.geps) || near_boundary(qy, it.geps);
        const int slot = tagged_slot_wave(&rec->guard_word, (unsigned)it.gen, guarded);
        if (guarded) {
            if (slot < it.gcap) {
                GuardRec g;
                g.t = t;
                g.v = v;
                g.ix = ix + it.inject;
                g.iy = iy;
                rec->guard[slot] = g;
            }
            ix += it.inject;
        }
        srow[v] = super_base_l(beam_lattice(ix, iy, pl, inv_lr), pl);
        LGS_CHK_SUPER(pl, srow[v], t, v);
        edge |= (ix - pl.win_x < 0 || iy - pl.win_y < 0) ? 1 : 0;
    }
    // this angle has a beam whose coarse lattice starts left of / below the
    // map: the unsafe-block check runs for it (generation-stamped flag)
    if (__syncthreads_or(edge) && threadIdx.x == 0) it.tedge[t] = it.gen;
}
__global__ void k_patch(Items items, const int4* __restrict__ patches, int n)
{
    const RtcsmPlan& pl = items[0].pl;
    int2* __restrict__ idx = items[0].idx;
    int* __restrict__ cbase = items[0].cbase;
    int* __restrict__ tedge = items[0].tedge;
    const int gen = items[0].gen;
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    const int4 p = patches[k];
    const size_t o = (size_t)p.x * pl.Nv + p.y;
    idx[o] = make_int2(p.z, p.w);
    cbase[o] = coarse_base(p.z, p.w, pl);
    cbase[pl.sb_off + o] = super_base(p.z, p.w, pl);
    if (p.z - pl.win_x < 0 || p.w - pl.win_y < 0) tedge[p.x] = gen;
}

// full host projection -> coarse info
__global__ void k_cinfo(Items items)
{
    const RtcsmPlan& pl = items[0].pl;
    const int2* __restrict__ idx = items[0].idx;
    int* __restrict__ cbase = items[0].cbase;
    int* __restrict__ tedge = items[0].tedge;
    const int gen = items[0].gen;
    const size_t o = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (o < kPad) {
        cbase[(size_t)pl.T * pl.Nv + o] = 0;
        cbase[pl.sb_off + (size_t)pl.T * pl.Nv + o] = 0;
    }
    if (o >= (size_t)pl.T * pl.Nv) return;
    const int2 q = idx[o];
    cbase[o] = coarse_base(q.x, q.y, pl);
    cbase[pl.sb_off + o] = super_base(q.x, q.y, pl);
    if (q.x - pl.win_x < 0 || q.y - pl.win_y < 0) tedge[o / pl.Nv] = gen;
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
// Copy n elements global -> LDS with the whole workgroup, loads issued in
// batches of 8 per thread before their stores (a plain strided loop waits one
// memory latency per element per thread).
template <class T>
__device__ __forceinline__ void stage_lds(T* dst, const T* __restrict__ src, int n)
{
    const int nt = blockDim.x;
    for (int v0 = threadIdx.x; v0 < n; v0 += 8 * nt) {
        T x[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int v = v0 + j * nt;
            if (v < n) x[j] = src[v];
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int v = v0 + j * nt;
            if (v < n) dst[v] = x[j];
        }
    }
}

// Block-wide row staging (stage_lds's replacement for lean items): the angle
// row of coarse bases / cells into LDS.
__device__ __forceinline__ void stage_cbase_row(int* dst, const MatchItem& it, int t, int n)
{
    if (!it.lean) {
        stage_lds(dst, it.cbase + (size_t)t * it.pl.Nv, n);
#ifdef LGS_CHECK_OFFSETS
        __syncthreads();
        for (int v = threadIdx.x; v < n; v += blockDim.x) LGS_CHK_COARSE(it.pl, dst[v], t, v);
#endif
        return;
    }
    for (int v = threadIdx.x; v < n; v += blockDim.x) {
        dst[v] = lean_coarse_base(it, t, v);
        LGS_CHK_COARSE(it.pl, dst[v], t, v);
    }
}
__device__ __forceinline__ void stage_idx_row(int2* dst, const MatchItem& it, int t, int n)
{
    if (!it.lean) {
        stage_lds(dst, it.idx + (size_t)t * it.pl.Nv, n);
        return;
    }
    for (int v = threadIdx.x; v < n; v += blockDim.x) dst[v] = lean_cell(it, t, v);
}


constexpr int kSB = 4;   // superblock = kSB x kSB coarse blocks
constexpr int kSeedCands = 4;   // k_seed_super workgroups (candidate superblocks)
constexpr int kSeedWide = 16;   // wide seed (batches): at most this many candidate superblocks' best members compared

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
// Phase-plane ("decimated") coarse map.  Coarse reads of one beam are at
// x = ix - winX + lr*jx, y = iy - winY + lr*jy: a stride-lr lattice.  Storing
// the coarse map as lr*lr planes D[ry][rx][qy][qx] = C[lr*qy+ry][lr*qx+rx]
// turns that lattice into a dense block of one plane, so the lanes of a wave
// (consecutive jx) gather consecutive doubles.  Cells past the map are 0.0,
// exactly what GridMap::Value returns out of bounds.
// --------------------------------------------------------------------------
// Writes the interior of the padded planes only (the margins are zeroed once
// per buffer and layout, planes_buffer).
__global__ __launch_bounds__(256) void k_decimate(const double* __restrict__ C, int W, int H, int lr,
                                                  int Wq, int M, int Wqp, long long pstride,
                                                  double* __restrict__ D)
{
    const int qx = blockIdx.x * blockDim.x + threadIdx.x;
    const int qy = blockIdx.y;
    const int plane = blockIdx.z;  // ry * lr + rx
    if (qx >= Wq) return;
    const int rx = plane % lr, ry = plane / lr;
    const int x = lr * qx + rx, y = lr * qy + ry;
    const double v = (x < W && y < H) ? C[(size_t)y * W + x] : 0.0;
    D[plane * pstride + (long long)(qy + M) * Wqp + qx + M] = v;
}

// Supplied coarse maps of a batch in one launch (r05: one k_decimate and one
// k_planes16 per map were 8 small launches per config-5 chunk): job
// blockIdx.z / lr^2, plane blockIdx.z % lr^2; the interior of the padded
// planes and, where the set has them, their fp16 round-up copies (the
// margins of both are zero from planes_buffer).
struct DecimJob {
    const double* C;        // the supplied coarse map (W x H)
    double* D;              // the set's padded phase planes
    unsigned short* D16;    // their fp16 copies (null: no superblock bounds)
    int* negflag;
    int pgen;
};
__global__ __launch_bounds__(256) void k_decimate_jobs(const DecimJob* __restrict__ jobs, int W, int H, int lr,
                                                       int Wq, int M, int Wqp, long long pstride)
{
    const int np = lr * lr;
    const DecimJob& j = jobs[blockIdx.z / np];
    const int plane = blockIdx.z % np;   // ry * lr + rx
    const int qx = blockIdx.x * blockDim.x + threadIdx.x;
    const int qy = blockIdx.y;
    if (qx >= Wq) return;
    const int rx = plane % lr, ry = plane / lr;
    const int x = lr * qx + rx, y = lr * qy + ry;
    const double v = (x < W && y < H) ? j.C[(size_t)y * W + x] : 0.0;
    const long long o = plane * pstride + (long long)(qy + M) * Wqp + qx + M;
    j.D[o] = v;
    if (j.D16) {
        j.D16[o] = half_round_up_bits(v);
        if (v < 0.0) *j.negflag = j.pgen;
    }
}

// --------------------------------------------------------------------------
// Sequential fp64 sum in beam order with the gathers software-pipelined:
// batch k+1's loads are issued before batch k's values are added, so two
// batches of loads are always in flight per lane while the add chain (the
// reference's order, :217-221) runs.  load(v) issues one gather; beam
// indices are wave-uniform (scalar loads).
// --------------------------------------------------------------------------

// load(v) must be safe for v < n + 2*kPipe (index arrays are padded) and must
// not branch: out-of-map lanes read a zero cell.  Adding 0.0 to the running
// sum is an exact no-op (the sum starts at +0.0 and can never become -0.0),
// and is exactly what GridMap::Value's default contributes for those cells.
// fetch(v): the beam's (wave-uniform) index record; addr(rec): this lane's
// cell address (or the zero cell).  Index records of a batch are fetched
// together (merged scalar loads) before any address is formed.
template <class Rec, class Fetch, class Addr>
__device__ __forceinline__ void issue_batch(int v0, Fetch& fetch, Addr& addr, double (&buf)[kPipe])
{
    Rec rc[kPipe];
#pragma unroll
    for (int j = 0; j < kPipe; ++j) rc[j] = fetch(v0 + j);
#pragma unroll
    for (int j = 0; j < kPipe; ++j) buf[j] = gload(addr(rc[j]));
}

__device__ __forceinline__ void add_batch(double& s, const double (&buf)[kPipe], int left)
{
    if (left >= kPipe) {
#pragma unroll
        for (int j = 0; j < kPipe; ++j) s += buf[j];
    } else {
        for (int j = 0; j < left; ++j) s += buf[j];
    }
}

// Two register buffers alternate roles (no copies), so while batch k is being
// added, batch k+1's gathers are in flight.  seq_sum_from continues a sum
// (the same additions, in order, as one longer seq_sum).
template <class Rec, class Fetch, class Addr>
__device__ __forceinline__ double seq_sum_from(double s, int n, Fetch fetch, Addr addr)
{
    double a[kPipe], b[kPipe];
    issue_batch<Rec>(0, fetch, addr, a);
    for (int v0 = 0; v0 < n; v0 += 2 * kPipe) {
        issue_batch<Rec>(v0 + kPipe, fetch, addr, b);
        add_batch(s, a, n - v0);
        if (v0 + kPipe >= n) break;
        issue_batch<Rec>(v0 + 2 * kPipe, fetch, addr, a);
        add_batch(s, b, n - v0 - kPipe);
    }
    return s;
}
template <class Rec, class Fetch, class Addr>
__device__ __forceinline__ double seq_sum(int n, Fetch fetch, Addr addr)
{
    double a[kPipe], b[kPipe];
    double s = 0.0;
    issue_batch<Rec>(0, fetch, addr, a);
    for (int v0 = 0; v0 < n; v0 += 2 * kPipe) {
        issue_batch<Rec>(v0 + kPipe, fetch, addr, b);
        add_batch(s, a, n - v0);
        if (v0 + kPipe >= n) break;
        issue_batch<Rec>(v0 + 2 * kPipe, fetch, addr, a);
        add_batch(s, b, n - v0 - kPipe);
    }
    return s;
}

// compile-time loop C = 0, STEP, 2*STEP, ... < MAXC; f returns false to stop
template <int C, int MAXC, int STEP, class F>
__device__ __forceinline__ void static_for_step(F&& f)
{
    if constexpr (C < MAXC) {
        if (!f(std::integral_constant<int, C>{})) return;
        static_for_step<C + STEP, MAXC, STEP>(f);
    }
}

// Four batches in flight (for kernels with few waves, where one wave's
// latency is the kernel's duration): look-ahead up to 4*kPipe entries.
template <class Rec, class Fetch, class Addr>
__device__ __forceinline__ double seq_sum4(int n, Fetch fetch, Addr addr)
{
    double a[kPipe], b[kPipe], c[kPipe], d[kPipe];
    double s = 0.0;
    issue_batch<Rec>(0, fetch, addr, a);
    issue_batch<Rec>(kPipe, fetch, addr, b);
    issue_batch<Rec>(2 * kPipe, fetch, addr, c);
    for (int v0 = 0; v0 < n; v0 += 4 * kPipe) {
        issue_batch<Rec>(v0 + 3 * kPipe, fetch, addr, d);
        add_batch(s, a, n - v0);
        if (v0 + kPipe >= n) break;
        issue_batch<Rec>(v0 + 4 * kPipe, fetch, addr, a);
        add_batch(s, b, n - v0 - kPipe);
        if (v0 + 2 * kPipe >= n) break;
        issue_batch<Rec>(v0 + 5 * kPipe, fetch, addr, b);
        add_batch(s, c, n - v0 - 2 * kPipe);
        if (v0 + 3 * kPipe >= n) break;
        issue_batch<Rec>(v0 + 6 * kPipe, fetch, addr, c);
        add_batch(s, d, n - v0 - 3 * kPipe);
    }
    return s;
}

// seq_sum4 continuing a sum (k_coarse_list_c's chunks, LGS_LIST_PIPE4)
template <class Rec, class Fetch, class Addr>
__device__ __forceinline__ double seq_sum_from4(double s, int n, Fetch fetch, Addr addr)
{
    double a[kPipe], b[kPipe], c[kPipe], d[kPipe];
    issue_batch<Rec>(0, fetch, addr, a);
    issue_batch<Rec>(kPipe, fetch, addr, b);
    issue_batch<Rec>(2 * kPipe, fetch, addr, c);
    for (int v0 = 0; v0 < n; v0 += 4 * kPipe) {
        issue_batch<Rec>(v0 + 3 * kPipe, fetch, addr, d);
        add_batch(s, a, n - v0);
        if (v0 + kPipe >= n) break;
        issue_batch<Rec>(v0 + 4 * kPipe, fetch, addr, a);
        add_batch(s, b, n - v0 - kPipe);
        if (v0 + 2 * kPipe >= n) break;
        issue_batch<Rec>(v0 + 5 * kPipe, fetch, addr, b);
        add_batch(s, c, n - v0 - 2 * kPipe);
        if (v0 + 3 * kPipe >= n) break;
        issue_batch<Rec>(v0 + 6 * kPipe, fetch, addr, c);
        add_batch(s, d, n - v0 - 3 * kPipe);
    }
    return s;
}

// --------------------------------------------------------------------------
// k_coarse: one lane per coarse block (t, jx, jy) of one search angle t per
// workgroup (blockDim = P rounded up to 64); lanes sweep jx fastest.  Each lane
// walks the beams in order: the reference's sequential fp64 sum.
//   PLANES = 1: phase-plane coarse map (k_decimate), lanes gather consecutive
//               doubles of one plane;
//   PLANES = 0: the coarse map as is (stride lr between lanes).
// --------------------------------------------------------------------------
__global__ __launch_bounds__(1024) void k_coarse(Items items, const double* __restrict__ zero)
{
    const MatchItem& it = items[blockIdx.z];
    const RtcsmPlan& pl = it.pl;
    if ((int)blockIdx.y >= pl.T) return;   // past this item's angles (uniform)
    const double* __restrict__ cmap = it.cmap;
    const int2* __restrict__ idx = it.idx;
    const int* __restrict__ cbase = it.cbase;
    const int* __restrict__ tedge = it.tedge;
    const int gen = it.gen;
    double* __restrict__ cscore = it.cscore;
    uint8_t* __restrict__ cflag = it.cflag;
    double* __restrict__ part_c = it.part_c;
    long long* __restrict__ part_k = it.part_k;
    __shared__ double sv[16];
    __shared__ long long sk[16];
    const int tt = blockIdx.y;
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    const bool active = p < pl.P;
    const int jx = active ? p % pl.ncx : 0;
    const int jy = active ? p / pl.ncx : 0;
    const int lr = pl.low_res;
    const int W = pl.W, H = pl.H;
    const size_t o = (size_t)tt * pl.Nv;
    const int2* __restrict__ id = idx + o;
    const int* __restrict__ cb = cbase + o;
#ifdef LGS_CHECK_OFFSETS
    if (blockIdx.x == 0)
        for (int v = threadIdx.x; v < pl.Nv; v += blockDim.x) LGS_CHK_COARSE(pl, cb[v], tt, v);
#endif

    const double* __restrict__ lane_base = cmap + (jy * pl.Wqp + jx);
    const double sum =
        seq_sum<int>(pl.Nv, [&](int v) { return cb[v]; }, [&](const int& c) { return lane_base + c; });
    // unsafe: some coarse read left of / below the map while the block's fine
    // reads can land inside (x, y >= -(lr-1)); rare, so a separate pass
    bool unsafe = false;
    if (tedge[tt] == gen) {
        const int lo = -(lr - 1);
        const int x0 = -pl.win_x + jx * lr, y0 = -pl.win_y + jy * lr;
        for (int v = 0; v < pl.Nv; ++v) {
            const int2 q = id[v];
            if (q.x - pl.win_x < 0 || q.y - pl.win_y < 0) {  // wave-uniform
                const int x = q.x + x0, y = q.y + y0;
                unsafe |= (x >= lo) & (x < W) & (y >= lo) & (y < H) & ((x < 0) | (y < 0));
            }
        }
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

// --------------------------------------------------------------------------
// Superblock pruning.  A superblock is kSB x kSB coarse
// blocks of one angle.  Its bound, for beam v, reads the super planes (the
// forward kSB x kSB max of the padded coarse planes) at the superblock's
// corner, which is >= the coarse value of every member block at that beam.
// fp64 addition is monotone, so the reference-order sum of the member's
// coarse values is <= the reference-order sum of these super values, which is
// <= (any-order sum) * (1 + 8 n eps) for n nonnegative terms: sbound =
// parallel sum * pl.sb_mult bounds every member's coarse score.  A safe block
// with c < L is never selected, so superblocks with sbound < L are skipped.
// --------------------------------------------------------------------------
// The bound needs nonnegative terms (occupancy probabilities are); a negative
// cell stamps *negflag with this build's generation (the precompute or
// k_planes16, which write the planes' fp16 round-ups) and k_super then keeps
// every superblock.  NaN cells round to +0 and so are skipped by the max: a
// block whose sum is NaN fails c > thr and is never selected anyway.
// k_super_planes: one workgroup per (tile of kSPX padded columns x kSPY
// padded rows, plane, set).  A tile spans a config-2 plane's whole width
// (Wqp = 240; 224-column tiles left a second tile per row with 16 columns).
//  1. vertical 4-max in registers: a thread owns one footprint column
//     (kSPX + 3 <= kSPThreads), loads its kSPY + 3 values (0 past the plane)
//     at once and writes the kSPY window maxima, already rounded toward +inf
//     to fp16, to LDS (round-up is monotone: the max of the rounded values is
//     the rounded max, so rounding before the horizontal max changes nothing
//     and quarters the LDS);
//  2. horizontal 4-max of the fp16 values from LDS, 8 consecutive superblocks
//     of one sub-phase row per thread, one 16-byte store (Wq4 is a multiple of
//     8, so sub-phase rows are 16-byte aligned).
constexpr int kSPX = 256, kSPY = 16;   // kSPX = 4 sub-phases x 64 (8 stores of 8)
constexpr int kSPThreads = (kSPX + 3 + 63) / 64 * 64;   // >= kSPX + kSB - 1 column loaders

// SPX: tile width (kSPX for a batch's sets; a lone set takes narrower tiles,
// more workgroups for its few hundred tiles: latency-bound, like the precompute)
constexpr int kSPXLone = 128;   // measured (lone config-2 set): 256: 12.9 us, 128: 11.3, 64: 11.2
template <int SPX>
__global__ __launch_bounds__((SPX + 3 + 63) / 64 * 64) void k_super_planes(const PlaneJob* __restrict__ jobs, int nplanes)
{
    constexpr int kSPX = SPX;
    constexpr int kSPThreads = (kSPX + 3 + 63) / 64 * 64;
    const Blk wg = xcd_block();
    const PlaneJob& job = jobs[wg.z / nplanes];
    const int plane = wg.z % nplanes;
    const RtcsmPlan& pl = job.pl;
    const unsigned short* __restrict__ P = job.planes16;
    SuperT* __restrict__ S = job.super;
    const int Wqp = pl.Wqp, Hqp = pl.Hqp;
    constexpr int TW = kSPX + kSB - 1, TH = kSPY + kSB - 1;
    static_assert(TW <= kSPThreads, "one loader per footprint column");
    __shared__ SuperT vm[kSPY][TW + 1];
    const int x0 = wg.x * kSPX, y0 = wg.y * kSPY;
    SuperT* __restrict__ out = S + plane * pl.pstride4;
    const int tid = threadIdx.x;
    // the strip left of / below the map (padded column / row M - 1 of the
    // planes rx >= 1 / ry >= 1: coarse x, y in [-(lr - 1), -1], whose fine
    // windows overlap the map) reads the map's first coarse column / row
    // C(0, y) / C(x, 0) >= every fine value of the overlap, so superblock
    // bounds also bound the FINE scores of unsafe blocks;
    // the coarse planes themselves keep the reference's zeros there
    const int lr = pl.low_res, M = pl.M;
    const int rx = plane % lr, ry = plane / lr;
    if (tid < TW) {
        const int x = x0 + tid;
        const bool cx = (x == M - 1) && rx > 0;
        const int sx = cx ? M : x;
        // global (not flat) loads: the plane pointer comes through a struct
        typedef const __attribute__((address_space(1))) unsigned short ghalf_t;
        ghalf_t* __restrict__ colp = (ghalf_t*)(P + (long long)(cx ? ry * lr : plane) * pl.pstride);   // plane (ry, 0)
        ghalf_t* __restrict__ rowp = (ghalf_t*)(P + (long long)(cx ? 0 : rx) * pl.pstride);           // plane (0, rx)
        unsigned short v[TH];
#pragma unroll
        for (int k = 0; k < TH; ++k) {
            const int y = y0 + k;
            const bool cy = (y == M - 1) && ry > 0;
            ghalf_t* __restrict__ src = cy ? rowp + (long long)M * Wqp : colp + (long long)y * Wqp;
            v[k] = (x < Wqp && y < Hqp) ? src[sx] : (unsigned short)0;   // 0 past the plane
        }
        // forward 4-max as two pair maxima of the fp16 round-ups (the values
        // are +0 or positive unless a negative cell disabled the bounds, so
        // their bit patterns order like the values; round-up is monotone, so
        // this is the round-up of the fp64 maximum)
        static_assert(kSB == 4, "pairwise forward 4-max");
        unsigned short m2[TH - 1];
#pragma unroll
        for (int k = 0; k < TH - 1; ++k) m2[k] = v[k] > v[k + 1] ? v[k] : v[k + 1];
#pragma unroll
        for (int r = 0; r < kSPY; ++r)
            vm[r][tid] = __builtin_bit_cast(SuperT, m2[r] > m2[r + 2] ? m2[r] : m2[r + 2]);
    }
    __syncthreads();
    // horizontal 4-max of the rounded values, lane = padded column, stored
    // sub-phase-major: hs[r][sx][X4] = S at column 4 X4 + sx
    constexpr int kQ = kSPX / 4;
    __shared__ __attribute__((aligned(16))) SuperT hs[kSPY][4][kQ];
    if (tid < kSPX) {
#pragma unroll
        for (int r = 0; r < kSPY; ++r) {
            // max of the bit patterns: the values are +0 or positive unless a
            // negative cell disabled the bounds (negflag)
            unsigned short m = __builtin_bit_cast(unsigned short, vm[r][tid]);
#pragma unroll
            for (int j = 1; j < kSB; ++j) {
                const unsigned short c = __builtin_bit_cast(unsigned short, vm[r][tid + j]);
                m = (m < c) ? c : m;
            }
            hs[r][tid & 3][tid >> 2] = __builtin_bit_cast(SuperT, m);
        }
    }
    __syncthreads();
    const int q0 = x0 >> 2;   // the tile's first superblock column (x0 is a multiple of 4)
    if (pl.oct) {
        // octet layout: the tile is kSPY / 16 quads (sub-phase rows 4 qt ..
        // 4 qt + 3, 16 padded rows each) of every sub-phase array; a quad's 4
        // rows at column X are the low half of unit (qt, X) and the high half
        // of (qt - 1, X)
        static_assert(kSPY % 16 == 0, "whole quads of sub-phase rows per tile");
        typedef unsigned long long u64;
        const int u8 = pl.unit8;   // 8-bit units: 2 dwords (8 rows) or 3 (12 rows), as k_super_hv
        unsigned* __restrict__ uo = (unsigned*)S + (long long)u8 * plane * pl.pstrideO;
        bool over = false;
        for (int k = tid; k < kSPY * kQ; k += blockDim.x) {   // (quad, sub-phase, column), column fastest
            const int h = k / (16 * kQ), sp = (k / kQ) % 16, X = k % kQ;
            const int qt = (y0 >> 4) + h;
            const int cy = sp >> 2, sx = sp & 3, Xg = q0 + X;
            if (Xg >= pl.Wq4) continue;
            u64 v = 0;
#pragma unroll
            for (int i = 0; i < 4; ++i)
                v |= (u64)__builtin_bit_cast(unsigned short, hs[16 * h + 4 * i + cy][sx][X]) << (16 * i);
            const unsigned b4 = quad_u8(v, over);
            const long long u = sp * pl.subO + (long long)qt * pl.Wq4 + Xg;
            gstore(uo + u8 * u, b4);                                          // rows 4 qt .. of unit qt
            if (qt > 0) gstore(uo + (u8 * (u - pl.Wq4) + 1), b4);             // .. of unit qt - 1
            if (u8 == 3 && qt > 1) gstore(uo + (3 * (u - 2 * pl.Wq4) + 2), b4);   // .. of unit qt - 2
        }
        if (over && job.negflag) gstore(job.negflag, job.pgen);
        return;
    }
    // one 16-byte store of 8 consecutive superblocks of a sub-phase row per
    // task (row, sub-phase, chunk), chunk fastest
    constexpr int kChunks = kQ / 8;
    typedef SuperT s8 __attribute__((ext_vector_type(8)));
    for (int k = tid; k < kSPY * 4 * kChunks; k += blockDim.x) {
        const int r = k / (4 * kChunks), rem = k % (4 * kChunks);
        const int sx = rem / kChunks, ch = rem % kChunks;
        const int y = y0 + r;
        const int xq = q0 + 8 * ch;
        if (y >= Hqp || xq >= pl.Wq4) continue;
        gstore((s8*)(out + ((y & 3) * 4 + sx) * pl.sub4 + (long long)(y >> 2) * pl.Wq4 + xq), *(const s8*)&hs[r][sx][8 * ch]);
    }
}

// --------------------------------------------------------------------------
// k_super_hv (r05): the octet superblock units straight from the planes'
// fp16 round-up copies, one thread per (plane, quad qt, unit column X4) with
// both 4-maxima in registers (r04's k_super_planes: one workgroup per 256 x 16
// tile, vertical max in registers, horizontal max through LDS).
//
// S(Y, X) = max_{i,j<4} V(Y + j, X + i) over the strip-clamped copies V:
// padded column M - 1 of a plane rx > 0 reads column M of plane (0, ry), row
// M - 1 of a plane ry > 0 reads row M of plane (rx, 0) (both: plane 0's (M,
// M)) -- the map's first coarse column / row, DESIGN.md §4.1b -- and 0 past
// the plane.  A thread loads rows 16 qt .. 16 qt + 18 at columns 4 X4 ..
// 4 X4 + 6 (two 8-byte loads per row: plane rows are a multiple of 4
// columns), forms the horizontal then the vertical max with packed u16 max
// (bit patterns of the nonnegative round-ups order like the values; a
// negative cell disables the bounds), and stores the 16 sub-phases' halves of
// rows 4 qt .. 4 qt + 3: the low half of unit qt, the high half of unit
// qt - 1 (24-byte units: the top third of qt - 2).  Threads are (quad, unit
// column) pairs, column fastest: no idle lanes, and a workgroup's quads are
// consecutive, so the two halves of a unit meet in one L2.  Same bits as
// k_super_planes.  Only units that can hold a nonzero value (padded rows /
// columns [M - 4, M + Hq / Wq)) are written; the others keep the zeros
// written when the buffer was allocated (planes_buffer).  (Measured and
// rejected: a thread walking a run of 4 unit rows down its column, carrying
// the halo rows and storing each unit whole -- 1.0 vs 0.18 ms per 64
// config-2 sets: the ring of the last quads' maxima went to scratch.)
struct SuperGeom {
    int M, Wqp, Wq4, unit8, Hqp;
    long long pstride, subO, pstrideO;
    int X4lo, ncol, qlo, nqt, lr;     // unit columns [X4lo, X4lo + ncol), quads [qlo, qlo + nqt)
};
// k_super_hv's grid (x): workgroups per plane
inline int hv_grid_x(const SuperGeom& g, int nq) { return (g.ncol * (g.nqt + nq - 1) + 255) / 256; }
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ unsigned pkmax(unsigned a, unsigned b)
{
    return __builtin_bit_cast(unsigned, __builtin_elementwise_max(__builtin_bit_cast(u16x2, a), __builtin_bit_cast(u16x2, b)));
}
// NQ quads per thread: NQ = 1 stores the quad's halves (two 8-byte stores
// per sub-phase, each unit's other half from the neighbouring quad's
// thread); NQ = 2 (16-byte units) computes quads qt and qt + 1 and stores
// unit qt whole (one 16-byte store per sub-phase, 64 consecutive units per
// wave instruction), every quad's maxima computed by two threads.
template <int NQ>
__global__ __launch_bounds__(256) void k_super_hv(const PlaneJob* __restrict__ jobs, int nplanes, SuperGeom g, DevTs dts)
{
    const DtsScope dts_scope(dts);
    const Blk wg = xcd_block();
    const PlaneJob& job = jobs[wg.z / nplanes];
    const int p = wg.z % nplanes;
    // (quad or unit, unit column), column fastest.  (Measured and rejected,
    // r05: workgroups as tiles of 256 / n quads x n unit columns, n = 8-32,
    // so that zero tiles would also cover empty columns: 0.145-0.165 vs
    // 0.106 ms per 64 config-2 sets.)
    const int tq = wg.x * 256 + threadIdx.x;
    const int qi = tq / g.ncol, c = tq - qi * g.ncol;
    // NQ = 2: units qlo - 1 .. qlo + nqt - 1 (unit u holds quads u, u + 1)
    const int qt0 = g.qlo + qi - (NQ - 1);
    const bool live = qi < g.nqt + NQ - 1 && qt0 >= 0 && c < g.ncol;
    // zero tiles (ZeroTiles): the workgroup's word says whether every unit
    // half it stores holds +0 from its previous build; threads past the
    // quads then load in-range rows and take part in the barrier only
    unsigned* zw = job.zt ? job.zt + ((long long)p * gridDim.x + wg.x) : nullptr;   // uniform
    if (!live && !zw) return;
    const int X4 = g.X4lo + min(c, g.ncol - 1), qt = min(max(qt0, 0), g.qlo + g.nqt - 1);
    const int rx = p % g.lr, ry = p / g.lr;
    typedef unsigned long long u64;
    typedef const __attribute__((address_space(1))) u64 gu64_t;
    typedef const __attribute__((address_space(1))) unsigned short gu16_t;
    const unsigned short* P = job.planes16;
    const long long rowM = (long long)g.M * g.Wqp;
    // the column strip: column 3 of unit column (M - 1) / 4 in planes rx > 0
    const bool cstrip = rx > 0 && 4 * X4 + 3 == g.M - 1;
    constexpr int NR = 16 * NQ + 3;
    // every load first, from always-valid addresses (rows past the plane
    // clamped to its last row, then zeroed; the strip column's value loaded
    // by every thread, from its own row where it is not the strip): a load
    // under a branch made the compiler wait for each row (19 round trips)
    u64 la[NR], lb[NR];
    unsigned short ls[NR];
#pragma unroll
    for (int k = 0; k < NR; ++k) {
        const int Y = min(16 * qt + k, g.Hqp - 1);
        const bool rs = (Y == g.M - 1) && ry > 0;            // the row strip
        const unsigned short* row = rs ? P + rx * g.pstride + rowM : P + p * g.pstride + (long long)Y * g.Wqp;
        // column M - 1 reads column M of plane (0, ry) (row strip: plane 0)
        const unsigned short* src = !cstrip ? row + 4 * X4
                                  : rs ? P + rowM + g.M : P + ry * g.lr * g.pstride + (long long)Y * g.Wqp + g.M;
        la[k] = *(gu64_t*)(row + 4 * X4);
        lb[k] = *(gu64_t*)(row + 4 * X4 + 4);
        ls[k] = *(gu16_t*)src;
    }
    u64 hm[NR];   // horizontal forward 4-max of columns 4 X4 + k, k < 4, per row
#pragma unroll
    for (int k = 0; k < NR; ++k) {
        const bool in = 16 * qt + k < g.Hqp;
        u64 a = in ? la[k] : 0ull;
        const u64 b = in ? lb[k] : 0ull;
        if (cstrip) a = (a & 0x0000FFFFFFFFFFFFull) | ((u64)(in ? ls[k] : 0) << 48);
        // columns 0..7 as packed pairs: a = (c0 c1)(c2 c3), b = (c4 c5)(c6 c7)
        const unsigned a0 = (unsigned)a, a1 = (unsigned)(a >> 32), b0 = (unsigned)b, b1 = (unsigned)(b >> 32);
        const unsigned m01 = pkmax(a0, (a0 >> 16) | (a1 << 16));   // (max c0c1, max c1c2)
        const unsigned m23 = pkmax(a1, (a1 >> 16) | (b0 << 16));   // (max c2c3, max c3c4)
        const unsigned m45 = pkmax(b0, (b0 >> 16) | (b1 << 16));   // (max c4c5, max c5c6)
        hm[k] = (u64)pkmax(m01, m23) | ((u64)pkmax(m23, m45) << 32);   // 4-max at columns 0, 1 | 2, 3
    }
    unsigned vlo[16 * NQ], vhi[16 * NQ];   // vertical forward 4-max
#pragma unroll
    for (int k = 0; k < 16 * NQ; ++k) {
        vlo[k] = pkmax(pkmax((unsigned)hm[k], (unsigned)hm[k + 1]), pkmax((unsigned)hm[k + 2], (unsigned)hm[k + 3]));
        vhi[k] = pkmax(pkmax((unsigned)(hm[k] >> 32), (unsigned)(hm[k + 1] >> 32)),
                       pkmax((unsigned)(hm[k + 2] >> 32), (unsigned)(hm[k + 3] >> 32)));
    }
    if (zw) {
        unsigned nzw = 0;
#pragma unroll
        for (int k = 0; k < 16 * NQ; ++k) nzw |= vlo[k] | vhi[k];
        const unsigned zprev = *zw;                            // read by every thread before the
        const int anynz = __syncthreads_or(live && nzw != 0);  // barrier, rewritten after it
        if (!anynz && zprev == 1u) return;
        if (threadIdx.x == 0 && zprev != (anynz ? 0u : 1u)) *zw = anynz ? 0u : 1u;
    }
    if (!live) return;
    // 8-bit units of unit8 dwords: a quad's 4 rows are dword 0 of unit qt,
    // dword 1 of unit qt - 1 (and dword 2 of unit qt - 2)
    unsigned* __restrict__ uo = (unsigned*)job.super + (long long)g.unit8 * p * g.pstrideO;
    const int u8 = g.unit8;
    bool over = false;
#pragma unroll
    for (int cy = 0; cy < 4; ++cy) {
#pragma unroll
        for (int cx = 0; cx < 4; ++cx) {
            unsigned h[NQ];
#pragma unroll
            for (int q = 0; q < NQ; ++q) {
                u64 hh = 0;
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const unsigned wv = (cx < 2) ? vlo[16 * q + 4 * i + cy] : vhi[16 * q + 4 * i + cy];
                    hh |= (u64)((cx & 1) ? (wv >> 16) : (wv & 0xFFFFu)) << (16 * i);
                }
                h[q] = quad_u8(hh, over);
            }
            const long long u = (cy * 4 + cx) * g.subO + (long long)qt * g.Wq4 + X4;
            if constexpr (NQ == 2) {   // unit qt whole (8-row units)
                gstore((u64*)(uo + 2 * u), (u64)h[0] | ((u64)h[1] << 32));
            } else {
                gstore(uo + u8 * u, h[0]);                                          // rows 4 qt .. of unit qt
                if (qt > 0) gstore(uo + (u8 * (u - g.Wq4) + 1), h[0]);              // .. of unit qt - 1
                if (u8 == 3 && qt > 1) gstore(uo + (3 * (u - 2 * g.Wq4) + 2), h[0]);   // .. of unit qt - 2
            }
        }
    }
    if (over && job.negflag) gstore(job.negflag, job.pgen);
}

// k_super: one workgroup (kSupWaves waves) per (chunk of superblocks, search
// angle); lane = superblock, wave w sums a quarter of the beams (any order:
// the bound absorbs the rounding; four batches of gathers in flight), LDS
// reduction over the waves.  PAIR (nsb2 <= 32): lanes 32..63 take the odd
// beams of the wave's range, so one gather instruction serves two beams (the
// texture-address rate per gather instruction, not bytes, is what this stage
// spends).  The angle's superblock base row is staged in LDS.  Also the
// chunk's best superblock for the seed (-inf in rows that may hold unsafe
// blocks).
constexpr int kSupWaves = 4;
template <int PAIR>
__global__ __launch_bounds__(64 * kSupWaves) void k_super(Items items, const double* __restrict__ zero)
{
    const Blk wg = xcd_block();
    const MatchItem& it = items[wg.z];
    const RtcsmPlan& pl = it.pl;
    if (wg.y >= pl.T) return;   // past this item's angles (uniform)
    const SuperT* __restrict__ sp = it.super;
    const SuperT* __restrict__ zf = (const SuperT*)zero;
    const int* __restrict__ cbase = it.cbase;
    const int* __restrict__ negflag = it.negflag;
    const int pgen = it.pgen;
    double* __restrict__ sbound = it.sbound;
    double* __restrict__ part_c = it.part_c;
    long long* __restrict__ part_k = it.part_k;
    extern __shared__ int srow[];   // [Nv]
    __shared__ double red[kSupWaves][64];
    constexpr int SPW = PAIR ? 32 : 64;   // superblocks per chunk
    const int t = wg.y;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int nsb2 = pl.nsbx * pl.nsby;
    const int h = PAIR ? (lane >> 5) : 0;
    const int sbi = wg.x * SPW + (lane & (SPW - 1));
    const bool act = sbi < nsb2;
    const int a = act ? sbi % pl.nsbx : 0, b = act ? sbi / pl.nsbx : 0;
    const SuperT* __restrict__ lb = sp + (b * pl.Wq4 + a);
    LGS_PROBE_DECL;
    LGS_PROBE_MARK();
    const int* __restrict__ cbrow = cbase + pl.sb_off + (size_t)t * pl.Nv;
    stage_lds(srow, cbrow, pl.Nv);
    __syncthreads();
#ifdef LGS_CHECK_OFFSETS
    for (int v = threadIdx.x; v < pl.Nv; v += blockDim.x) LGS_CHK_SUPER(pl, srow[v], t, v);
#endif
    LGS_PROBE_MARK();
    const int per = (pl.Nv + kSupWaves - 1) / kSupWaves;
    const int lo = min(w * per, pl.Nv), cnt = min(per, pl.Nv - lo);
    const int* row = srow + lo;
    double s;
    if constexpr (PAIR) {
        const int n2 = (cnt + 1) >> 1;
        s = seq_sum4<int>(n2, [&](int i) { const int v = 2 * i + h; return (v < cnt) ? row[v] : INT_MIN; },
                          [&](const int& c) { return (act && c != INT_MIN) ? lb + c : zf; });
        s += __shfl_xor(s, 32, 64);
    } else {
        s = seq_sum4<int>(cnt, [&](int v) { return (v < cnt) ? row[v] : INT_MIN; },
                          [&](const int& c) { return (act && c != INT_MIN) ? lb + c : zf; });
    }
    red[w][lane] = s;
    LGS_PROBE_MARK();
    __syncthreads();
    LGS_PROBE_MARK();
    if (w != 0) return;
    double tot = 0.0;
    for (int j = 0; j < kSupWaves; ++j) tot += red[j][lane];
    const double bound = (*negflag == pgen) ? INFINITY : tot * pl.sb_mult;
    const bool own = act && h == 0;
    if (own) sbound[(size_t)t * nsb2 + sbi] = bound;
    const bool seedable = own;   // k_seed_super skips unsafe members
    double bv = seedable ? bound : -INFINITY;
    long long bk = seedable ? (long long)t * nsb2 + sbi : LLONG_MAX;
    for (int off = 32; off > 0; off >>= 1) {
        const double ov = __shfl_xor(bv, off, 64);
        const long long ok = __shfl_xor(bk, off, 64);
        if (better(ov, ok, bv, bk)) {
            bv = ov;
            bk = ok;
        }
    }
    if (lane == 0) {
        const int part = t * gridDim.x + wg.x;
        part_c[part] = bv;
        part_k[part] = bk;
    }
    LGS_PROBE_MARK();
    LGS_PROBE_PRINT("super(stage, sum w0, barrier, tail)");
}

// k_super_oct (octet layout, nsbx, nsby <= 5): lane = (beam slot, window
// column a); one aligned 16-byte load per (beam, column) brings the column's 8
// sub-phase rows 4q .. 4q + 7, of which rows k .. k + 4 (k = the window's
// first row & 3) are the beam's 5 superblock rows -- a beam touches its 5
// columns' 80 contiguous bytes (1-2 cache lines) instead of 5 rows' lines.
// 64 / nsbx beams per wave instruction (12 for the config-2 window).  Slot
// partials meet in LDS; the bound is the any-order sum (the rounding slack
// sb_mult covers any order).
typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
#ifndef LGS_OCT_PIPE9
#define LGS_OCT_PIPE9 4   // load batches in flight per lane, 9-row windows (measured r04: 2-6: 0.280 ms per config-5 launch, 8: 0.304, 12: 0.376, 16: 0.445)
#endif
#ifndef LGS_OCT_PIPE5
#define LGS_OCT_PIPE5 8
#endif
template <int NR>
constexpr int oct_pipe() { return NR > 5 ? LGS_OCT_PIPE9 : LGS_OCT_PIPE5; }
// entries past the staged superblock-base row that k_super_oct's batched
// row reads may touch (64 beam slots x the deepest pipeline)
constexpr int kOctRowPad = 64 * (LGS_OCT_PIPE5 > LGS_OCT_PIPE9 ? LGS_OCT_PIPE5 : LGS_OCT_PIPE9);
// NR = the superblock rows a lane sums per beam: 5 (nsby <= 5: the beam's
// rows sit in one unit) or 9 (nsby <= 9: one unit + the high half of the next
// unit, rows 4q + 8 .. 4q + 11).
// U8: the unit size in 8-byte words (2: 16-byte units, 3: 24-byte units whose
// third word holds rows 4q + 8 .. 4q + 11, read with the first two at once)
template <int NR, int U8>
__global__ __launch_bounds__(64 * kSupWaves) void k_super_oct(Items items, const double* __restrict__ zero, DevTs dts)
{
    static_assert((NR == 5 && U8 == 2) || (NR == 9 && U8 == 3), "8-bit units: 8 rows for 5-row windows, 12 for 9");
    const DtsScope dts_scope(dts);
    const Blk wg = xcd_block();
    const MatchItem& it = items[wg.z];
    const RtcsmPlan& pl = it.pl;
    if (wg.y >= pl.T) return;   // past this item's angles (uniform)
    typedef unsigned long long u64;
    const unsigned* __restrict__ ub = (const unsigned*)it.super;   // 8-bit units of U8 dwords
    const unsigned* __restrict__ z4 = (const unsigned*)zero;
    extern __shared__ int srow[];   // [Nv + kOctRowPad]
    __shared__ int part[kSupWaves][64][NR];
    const int t = wg.y;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int nsbx = pl.nsbx, nsb2 = nsbx * pl.nsby;
    const int nb = 64 / nsbx;               // beam slots per wave instruction
    const int q = lane / nsbx, a = lane - nsbx * q;
    const bool act = q < nb;
    if (it.lean) {   // the row formed here (lean_super_row), k_project does not run
        lean_super_row(it, t, srow);
    } else {
        const int* __restrict__ cbrow = it.cbase + pl.sb_off + (size_t)t * pl.Nv;
        stage_lds(srow, cbrow, pl.Nv);
#ifdef LGS_CHECK_OFFSETS
        __syncthreads();
        for (int v = threadIdx.x; v < pl.Nv; v += blockDim.x) LGS_CHK_SUPER(pl, srow[v], t, v);
#endif
    }
    __syncthreads();
    const int per = (pl.Nv + kSupWaves - 1) / kSupWaves;
    const int lo = min(w * per, pl.Nv), cnt = min(per, pl.Nv - lo);
    const int* row = srow + lo;
    const int nq = (cnt + nb - 1) / nb;     // slot q takes beams nb i + q
    // exact integer sums of the 8-bit values, SWAR: two u64 of four 16-bit
    // fields, window rows (0, 2, 4, 6) and (1, 3, 5, 7), + row 8 (NR = 9).
    // A lane sums at most ceil(Nv / (kSupWaves nb)) <= 74 beams (Nv <= 2048 on
    // the pruned path, nb >= 7): <= 74 x 255 < 2^16, no field overflows.
    constexpr u64 kM = 0x00FF00FF00FF00FFull;
    u64 ae = 0, ao = 0;
    unsigned a8 = 0;
    constexpr int kOctPipe = oct_pipe<NR>();
    for (int i0 = 0; i0 < nq; i0 += kOctPipe) {
        u64 x[kOctPipe];
        unsigned y[kOctPipe];
        int sh[kOctPipe];
        // the batch's row entries first, unconditionally (the LDS row is
        // padded by kOctRowPad entries): one LDS wait per batch instead of
        // one per load (a masked read before each gather serialised them)
        int cv[kOctPipe];
#pragma unroll
        for (int j = 0; j < kOctPipe; ++j) cv[j] = row[nb * (i0 + j) + q];
#pragma unroll
        for (int j = 0; j < kOctPipe; ++j) {
            const int v = nb * (i0 + j) + q;
            const bool ok = act && v < cnt;
            const int c = ok ? cv[j] : 0;
            sh[j] = 8 * (c & 3);                      // the window's first row in the unit
            const unsigned* pu = ok ? ub + (size_t)U8 * (size_t)((c >> 2) + a) : z4;
            if constexpr (U8 == 2) {   // one 8-byte unit: rows 4q .. 4q + 7
                typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
                typedef const __attribute__((address_space(1))) u32x2 gu32x2_t;
                const u32x2 d = *(gu32x2_t*)pu;
                x[j] = (u64)d.x | ((u64)d.y << 32);
                y[j] = 0u;
            } else {                   // one 12-byte unit: rows 4q .. 4q + 11
                typedef unsigned u32x3 __attribute__((ext_vector_type(3), aligned(4)));
                typedef const __attribute__((address_space(1))) u32x3 gu32x3_t;
                const u32x3 d = *(gu32x3_t*)pu;
                x[j] = (u64)d.x | ((u64)d.y << 32);
                y[j] = d.z;
            }
        }
#pragma unroll
        for (int j = 0; j < kOctPipe; ++j) {
            const int k = sh[j];
            u64 wl;
            if constexpr (NR == 5) {
                wl = (x[j] >> k) & 0xFFFFFFFFFFull;   // rows 0..4 of the window
            } else {
                // rows 0..7 from bytes k/8 .. of (x, y); (y << (63 - k)) << 1 is
                // y << (64 - k) for k > 0 and 0 for k = 0: no branch on k
                wl = (x[j] >> k) | (((u64)y[j] << (63 - k)) << 1);
                a8 += (y[j] >> k) & 0xFFu;          // row 8
            }
            ae += wl & kM;
            ao += (wl >> 8) & kM;
        }
    }
#pragma unroll
    for (int r = 0; r < NR && r < 8; ++r) part[w][lane][r] = (int)(((r & 1) ? ao : ae) >> (16 * (r >> 1)) & 0xFFFFu);
    if constexpr (NR == 9) part[w][lane][8] = (int)a8;
    __syncthreads();
    if (w != 0) return;
    const int sbi = lane;
    const bool own = sbi < nsb2;
    int tot = 0;   // <= Nv x 255 (Nv <= 2048 on the pruned path): exact
    if (own) {
        const int ca = sbi % nsbx, rb = sbi / nsbx;
        for (int j = 0; j < kSupWaves; ++j)
            for (int s = 0; s < nb; ++s) tot += part[j][s * nsbx + ca][rb];
    }
    // the sum of the units / 255 >= the sum of the fp16 round-ups >= the sum
    // of the members' coarse values; the division's rounding (<= 2^-53
    // relative) is covered by 1 + 2^-50, the reference order by sb_mult
    const double bound =
        (*it.negflag == it.pgen) ? INFINITY : ((double)tot / 255.0) * (1.0 + 0x1p-50) * pl.sb_mult;
    if (own) it.sbound[(size_t)t * nsb2 + sbi] = bound;
    const bool seedable = own;   // k_seed_super skips unsafe members
    double bv = seedable ? bound : -INFINITY;
    long long bk = seedable ? (long long)t * nsb2 + sbi : LLONG_MAX;
    for (int off = 32; off > 0; off >>= 1) {
        const double ov = __shfl_xor(bv, off, 64);
        const long long ok = __shfl_xor(bk, off, 64);
        if (better(ov, ok, bv, bk)) {
            bv = ov;
            bk = ok;
        }
    }
    if (lane == 0) {
        it.part_c[t] = bv;
        it.part_k[t] = bk;
    }
}

// k_coarse_rows (superblock pruning): coarse scores of the blocks k_select
// could take; workgroup (angle t, patch row pr) of kRowWaves waves.  The
// angle's superblocks are kept when bound > thr and (bound >= L, or the angle
// may hold unsafe blocks); L = max of the seed candidates' fine lower bounds.
// Wave w scores patch row pr (4 blocks) of kept superblocks w, w + kRowWaves,
// ...: the four rows of a superblock run on four CUs, since a CU's
// outstanding cache-line misses, not its ALUs, pace a gather whose every beam
// touches another line.  Gathers and additions are transposed:
// global_load_lds (16 bytes = two neighbouring blocks' cells, no register
// destination) lands 32 beams x 4 blocks per wave instruction in an LDS ring
// of kRing slots, kRing instructions ahead of 4 adder lanes that walk the
// beams in order (the reference's sequential fp64 sum); counted vmcnt waits
// keep kRing - 1 gathers in flight, and each slot is refilled once read.
constexpr int kRowWaves = 1;   // waves per workgroup
constexpr int kRowSplit = 4;   // workgroups per (angle, patch row): kept superblocks e = z, z + 4, ...
// 1 KiB glds slots per wave; measured (lone config-2 scan): 12: 30.0 us, 14:
// 30.6, 16: 26.8, 18: 31.5, 20: 33.0, 24: 34.2, 32: 32.4
constexpr int kRing = 16;
typedef __attribute__((address_space(3))) void lds_void_t;
typedef const __attribute__((address_space(1))) void gbl_void_t;
// s_waitcnt immediates (gfx9 encoding: vmcnt[3:0] | expcnt[6:4] | lgkmcnt[11:8] | vmcnt[5:4] << 14)
constexpr unsigned waitcnt_imm(unsigned vm, unsigned lgkm)
{
    return (vm & 15u) | (7u << 4) | ((lgkm & 15u) << 8) | ((vm >> 4) << 14);
}
__global__ __launch_bounds__(64 * kRowWaves) void k_coarse_rows(Items items, const double* __restrict__ zero)
{
    // plain block order: the kept superblocks concentrate on few angles of
    // each item, and the XCD remap would put one item's busy workgroups on
    // one XCD (measured 0.59 -> 0.89 ms for 64 config-2 scans)
    const Blk wg = { (int)blockIdx.x, (int)blockIdx.y, (int)blockIdx.z };
    const MatchItem& it = items[wg.z / kRowSplit];
    const int split = wg.z % kRowSplit;   // kept superblocks e = split, split + kRowSplit, ...
    const RtcsmPlan& pl = it.pl;
    if (wg.x >= pl.T) return;   // past this item's angles (uniform)
    const double* __restrict__ cmap = it.cmap;
    const int2* __restrict__ idx = it.idx;
    const int* __restrict__ cbase = it.cbase;
    const int* __restrict__ tedge = it.tedge;
    const int gen = it.gen;
    const double* __restrict__ sbound = it.sbound;
    const double* __restrict__ Lc = it.Lc;
    double* __restrict__ Lp = it.Lp;
    double* __restrict__ cscore = it.cscore;
    uint8_t* __restrict__ cflag = it.cflag;
    RtcsmRecord* rec = it.rec;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    __shared__ int s_sb[64];
    __shared__ int s_cnt;
    const int t = wg.x, pr = wg.y;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int nsb2 = pl.nsbx * pl.nsby;
    const int Nv = pl.Nv;
    LGS_PROBE_DECL;
    LGS_PROBE_MARK();
    double L = -INFINITY;
#pragma unroll
    for (int b = 0; b < kSeedCands; ++b) L = fmax(L, Lc[b]);
    if (t == 0 && pr == 0 && split == 0 && tid == 0) *Lp = L;
    const bool te = tedge[t] == gen;
    // kept superblocks of this angle (nsb2 <= 64 on this path), in key order
    if (w == 0) {
        bool kp = false;
        if (lane < nsb2) {
            const double bnd = sbound[(size_t)t * nsb2 + lane];
            kp = (bnd > pl.thr) && bnd >= L;
        }
        const unsigned long long bal = __ballot(kp);
        if (kp) s_sb[__popcll(bal & ((1ull << lane) - 1ull))] = lane;
        if (lane == 0) {
            s_cnt = __popcll(bal);
            unsigned long long nb = 0;
            for (unsigned long long mm = bal; mm; mm &= mm - 1) {
                const int sb = __ffsll((long long)mm) - 1;
                const int a = sb % pl.nsbx, b = sb / pl.nsbx;
                nb += (unsigned long long)(min(kSB, pl.ncx - kSB * a) * min(kSB, pl.ncy - kSB * b));
            }
            if (nb && pr == 0 && split == 0) atomicAdd(&rec->coarse_evals, nb);
        }
    }
    __syncthreads();
    LGS_PROBE_MARK();
    const int cnt = s_cnt;
    if (cnt <= split * kRowWaves) return;   // no superblock for this workgroup
    int* srow = (int*)smem;                                   // [Nv]
    const size_t srow_bytes = (sizeof(int) * (size_t)Nv + 15) & ~(size_t)15;
    double* ring = (double*)(smem + srow_bytes) + (size_t)w * kRing * 128;   // [kRing][32 beams][4 blocks]
    stage_lds(srow, cbase + (size_t)t * Nv, Nv);
    __syncthreads();
#ifdef LGS_CHECK_OFFSETS
    for (int v = threadIdx.x; v < Nv; v += blockDim.x) LGS_CHK_COARSE(pl, srow[v], t, v);
#endif
    LGS_PROBE_MARK();
    // gather lane: beam lane / 2 of the instruction's 32, blocks 2 (lane % 2)
    // and + 1 of the patch row; adder lane c < 4: block c of the patch row
    const int gb = lane >> 1, gc = (lane & 1) * 2;
    const int ninstr = (Nv + 31) / 32;
    for (int e = split * kRowWaves + w; e < cnt; e += kRowWaves * kRowSplit) {
        const int sb = s_sb[e];
        const int jx0 = kSB * (sb % pl.nsbx), jy = kSB * (sb / pl.nsbx) + pr;
        const double* __restrict__ pb = cmap + (jy * pl.Wqp + jx0 + gc);
        auto offset_of = [&](int i) {   // unconditional LDS read (a branch would cost counted waits)
            const int v = 32 * i + gb;
            const int o = srow[min(v, Nv - 1)];
            return (v < Nv) ? o : -1;
        };
        auto issue = [&](int i, int off) {
            const double* g = (off >= 0) ? pb + off : zero;
            __builtin_amdgcn_global_load_lds((gbl_void_t*)g, (lds_void_t*)(ring + (i % kRing) * 128), 16, 0, 0);
        };
        for (int i = 0; i < kRing; ++i) issue(i, offset_of(i));   // past the scan: the zero cells
        const int jx = jx0 + (lane & 3);
        const bool active = lane < 4 && jx < pl.ncx && jy < pl.ncy;
        double acc = 0.0;
        // slot i + 1 -> nxt (LDS reads issued before slot i is added), then
        // slot i is refilled
        double ra[32], rb[32];
        auto read_slot = [&](int i, double (&x)[32]) {
            const double* slot = ring + (i % kRing) * 128 + (lane & 3);
#pragma unroll
            for (int bb = 0; bb < 32; ++bb) x[bb] = slot[bb * 4];
        };
        int offn = offset_of(kRing);
        auto step = [&](int i, double (&cur)[32], double (&nxt)[32]) {
            __builtin_amdgcn_s_waitcnt(waitcnt_imm(kRing - 2, 15));   // instruction i + 1 has landed
            read_slot(i + 1, nxt);   // past the scan: zero cells or unused slot contents
            const int oc = offn;
            offn = offset_of(i + kRing + 1);
            __builtin_amdgcn_sched_barrier(0);
            // beams past the scan read the zero cells: adding +0.0 to a sum that
            // starts at +0.0 is exact (as in seq_sum), so no tail predicate
            double s = acc;
#pragma unroll
            for (int bb = 0; bb < 32; ++bb) s += cur[bb];
            acc = s;
            __builtin_amdgcn_sched_barrier(0);
            __builtin_amdgcn_s_waitcnt(waitcnt_imm(63, 0));   // slot i + 1 is in registers
            issue(i + kRing, oc);                             // refill slot i
            __builtin_amdgcn_sched_barrier(0);
        };
        LGS_PROBE_MARK();
        __builtin_amdgcn_s_waitcnt(waitcnt_imm(kRing - 1, 15));   // instruction 0 has landed
        read_slot(0, ra);
        LGS_PROBE_MARK();
        for (int i = 0; i < ninstr; i += 2) {
            step(i, ra, rb);
            if (i + 1 >= ninstr) break;
            step(i + 1, rb, ra);
        }
        LGS_PROBE_MARK();
        __builtin_amdgcn_s_waitcnt(waitcnt_imm(0, 15));   // ring drained before its reuse
        // unsafe test (angles that may hold unsafe blocks only): lane (c, q)
        // checks beams q, q + 16, ..., OR-reduced over q
        // (+ ext: the strip reads' bound of the fine values, see strip_read)
        bool unsafe = false;
        double ext = 0.0;
        const int uc = lane & 3, uq = lane >> 2;
        const int ujx = jx0 + uc;
        if (te && ujx < pl.ncx && jy < pl.ncy) {
            const int2* __restrict__ id = idx + (size_t)t * Nv;
            const int lr = pl.low_res;
            const int x0 = -pl.win_x + ujx * lr, y0 = -pl.win_y + jy * lr;
            for (int v = uq; v < Nv; v += 16) {
                const int2 c = id[v];
                if (c.x - pl.win_x < 0 || c.y - pl.win_y < 0) unsafe |= strip_read(cmap, c.x + x0, c.y + y0, pl, ext);
            }
        }
#pragma unroll
        for (int off = 4; off < 64; off <<= 1) {
            unsafe |= __shfl_xor((int)unsafe, off, 64) != 0;
            ext += __shfl_xor(ext, off, 64);
        }
        if (active) {
            const long long k = (long long)t * pl.P + (long long)jx * pl.ncy + jy;
            cscore[k] = acc;
            // an unsafe block whose fine scores all stay below L can change
            // nothing: it is treated as safe (c <= bound < L)
            cflag[k] = (unsafe && (acc + ext) * pl.sb_mult >= L) ? 1 : 0;
        }
        LGS_PROBE_MARK();
    }
#ifdef LGS_PROBE
    if (tid == 0 && cnt >= 1 && pr == 0 && split == 0)
        printf("probe coarse_rows t=%d cnt=%d: select %.2f stage %.2f issue %.2f fill %.2f loop %.2f tail %.2f us\n",
               t, cnt, 0.01 * (double)(lgs_probe_t[1] - lgs_probe_t[0]),
               0.01 * (double)(lgs_probe_t[2] - lgs_probe_t[1]), 0.01 * (double)(lgs_probe_t[3] - lgs_probe_t[2]),
               0.01 * (double)(lgs_probe_t[4] - lgs_probe_t[3]), 0.01 * (double)(lgs_probe_t[5] - lgs_probe_t[4]),
               0.01 * (double)(lgs_probe_t[6] - lgs_probe_t[5]));
#endif
}

// The unsafe test of one angle (batched launches, k_unsafe_list): angles
// whose beams reach left of / below the map (tedge) need the unsafe test of
// every kept block over those beams; the workgroup first compacts the angle's
// edge beams (in beam order) into LDS, so each block walks only them instead
// of all Nv beams (the loop detector's local maps put most angles there).
// Lane = (kept superblock, member block), four superblocks per wave.
constexpr int kLaneWaves = 4;
constexpr int kEdgeMax = 1024;     // edge beams compacted in LDS (more: the full walk); 8 KB keeps
constexpr int kEdgeMaxNv = 4096;   // the occupancy of the kernel (measured: 32 KB cost config 2 30%)
// One angle t of item `it`: its kept superblocks (the selection ballot), the
// edge-beam compaction, then per kept block the unsafe test (the sum is
// already in cscore, written by k_coarse_list).  Called by a whole workgroup
// of kLaneWaves waves; the LDS arrays are reused when a workgroup takes
// several angles.
__device__ __forceinline__ void unsafe_angle(const MatchItem& it, int t)
{
    const RtcsmPlan& pl = it.pl;
    const double* __restrict__ cmap = it.cmap;
    const int2* __restrict__ idx = it.idx;
    const int gen = it.gen;
    __shared__ int s_sb[64];
    __shared__ int s_cnt;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int nsb2 = pl.nsbx * pl.nsby;
    double L = -INFINITY;
#pragma unroll
    for (int b = 0; b < kSeedCands; ++b) L = fmax(L, it.Lc[b]);
    const bool te = it.tedge[t] == gen;
    __syncthreads();   // the previous angle's LDS is read
    // kept superblocks of this angle (nsb2 <= 64 on this path), in key order
    if (w == 0) {
        bool kp = false;
        if (lane < nsb2) {
            const double bnd = it.sbound[(size_t)t * nsb2 + lane];
            kp = (bnd > pl.thr) && bnd >= L;
        }
        const unsigned long long bal = __ballot(kp);
        if (kp) s_sb[__popcll(bal & ((1ull << lane) - 1ull))] = lane;
        if (lane == 0) s_cnt = __popcll(bal);
    }
    __syncthreads();
    const int cnt = s_cnt;
    // edge beams of this angle: q = idx[t][v] with q.x - win_x < 0 or
    // q.y - win_y < 0, compacted in beam order (chunk counts, then offsets)
    __shared__ int2 s_edge[kEdgeMax];
    __shared__ int s_ccnt[kEdgeMaxNv / 64];
    int ne = -1;   // -1: walk every beam
    const int2* __restrict__ idr = idx + (size_t)t * pl.Nv;
    const bool lean = it.lean != 0;   // the cells formed here (lean_cell), not read
    if (te && cnt > 0 && pl.Nv <= kEdgeMaxNv) {
        const int nch = (pl.Nv + 63) / 64;
        for (int c = w; c < nch; c += kLaneWaves) {
            const int v = c * 64 + lane;
            const int2 q = v < pl.Nv ? (lean ? lean_cell(it, t, v) : idr[v]) : make_int2(pl.win_x, pl.win_y);
            const bool e = (q.x - pl.win_x < 0) | (q.y - pl.win_y < 0);
            const unsigned long long bal = __ballot(e);
            if (lane == 0) s_ccnt[c] = __popcll(bal);
        }
        __syncthreads();
        ne = 0;
        for (int k = 0; k < nch; ++k) ne += s_ccnt[k];
        for (int c = w; c < nch && ne <= kEdgeMax; c += kLaneWaves) {
            int off = 0;
            for (int k = 0; k < c; ++k) off += s_ccnt[k];
            const int v = c * 64 + lane;
            const int2 q = v < pl.Nv ? (lean ? lean_cell(it, t, v) : idr[v]) : make_int2(pl.win_x, pl.win_y);
            const bool e = (q.x - pl.win_x < 0) | (q.y - pl.win_y < 0);
            const unsigned long long bal = __ballot(e);
            if (e) s_edge[off + __popcll(bal & ((1ull << lane) - 1ull))] = q;
        }
        if (ne > kEdgeMax) ne = -1;
        __syncthreads();
    }
    for (int e0 = 4 * w; e0 < cnt; e0 += 4 * kLaneWaves) {   // wave-uniform
        const int e = e0 + (lane >> 4), m = lane & 15;
        const bool has = e < cnt;
        const int sb = has ? s_sb[e] : 0;
        const int jx = kSB * (sb % pl.nsbx) + (m & 3), jy = kSB * (sb / pl.nsbx) + (m >> 2);
        const bool active = has && jx < pl.ncx && jy < pl.ncy;
        const long long k = (long long)t * pl.P + (long long)jx * pl.ncy + jy;
        const double sum = active ? it.cscore[k] : 0.0;
        // unsafe: some coarse read left of / below the map while the block's
        // fine reads can land inside (x, y >= -(lr-1)); rare, so a separate pass
        // (+ ext: the strip reads' bound of the fine values, see strip_read)
        bool unsafe = false;
        double ext = 0.0;
        if (te && active) {
            const int lr = pl.low_res;
            const int x0 = -pl.win_x + jx * lr, y0 = -pl.win_y + jy * lr;
            if (ne >= 0) {
                for (int v = 0; v < ne; ++v) {
                    const int2 q = s_edge[v];
                    unsafe |= strip_read(cmap, q.x + x0, q.y + y0, pl, ext);
                }
            } else {
                for (int v = 0; v < pl.Nv; ++v) {
                    const int2 q = lean ? lean_cell(it, t, v) : idr[v];
                    if (q.x - pl.win_x < 0 || q.y - pl.win_y < 0)
                        unsafe |= strip_read(cmap, q.x + x0, q.y + y0, pl, ext);
                }
            }
        }
        if (active) {
            // an unsafe block whose fine scores all stay below L can change
            // nothing: it is treated as safe (c <= bound < L)
            it.cflag[k] = (unsafe && (sum + ext) * pl.sb_mult >= L) ? 1 : 0;
        }
    }
}

// Kept-superblock work list (every pruned batch; a lone match takes
// k_coarse_rows).  Most angles of a batch keep 0-3
// superblocks (loop closure: 76% keep none), so one workgroup per angle leaves
// most lanes idle.  k_keep lists every kept (angle, superblock) of each item
// -- the same selection, counted into the item's record -- and the angles
// with edge beams among them; k_coarse_list gives each wave four listed
// superblocks from any angles and items (16 lanes each), so the waves that
// walk the beams are full; k_unsafe_list then runs the unsafe test of the
// listed edge angles only.  The lists' order does not matter: every entry
// writes its own blocks.
// WorkList: cnt = 2 counters per item, 16 ints apart (zeroed by k_seed_super
// through MatchItem::keepc); sbl = per item `region` entries t << 6 | sb;
// al = per item Tmax edge angles.
struct WorkList {
    int* cnt;
    int* sbl;
    int* al;
    int region, tmax;
};
constexpr int kListMaxNv = 4096;   // work-list batches: Nv bound (the unsafe test stages an angle's edge beams)
// grid sizes measured (config 5 / config 2 stage ms): list 2048 + unsafe 1024: 0.272 / 0.373; 2048 + 4096:
// 0.241 / 0.375; 4096 + 4096: 0.226 / 0.364; 2304 + 4096: 0.226 / 0.365; 1024 + 4096: 0.288 / 0.528
#ifndef LGS_LIST_WAVES
#define LGS_LIST_WAVES 4096
#endif
constexpr int kListWaves = LGS_LIST_WAVES;   // k_coarse_list workgroups (one wave each, grid-stride)
#ifndef LGS_LIST_XCD
#define LGS_LIST_XCD 1
#endif
#ifndef LGS_XCD2
#define LGS_XCD2 1   // the same for k_fine_regs, and xcd_block() for the seed kernels
#endif
static_assert(kListWaves % 8 == 0, "whole workgroups per XCD");
constexpr int kUnsafeGroups = 4096;

__global__ __launch_bounds__(64) void k_keep(Items items, WorkList W, DevTs dts)
{
    const DtsScope dts_scope(dts);
    const int j = blockIdx.y;
    const MatchItem& it = items[j];
    const RtcsmPlan& pl = it.pl;
    const int t = blockIdx.x;
    if (t >= pl.T) return;   // past this item's angles (uniform)
    const int lane = threadIdx.x;
    const int nsb2 = pl.nsbx * pl.nsby;
    double L = -INFINITY;
#pragma unroll
    for (int b = 0; b < kSeedCands; ++b) L = fmax(L, it.Lc[b]);
    if (t == 0 && lane == 0) *it.Lp = L;
    bool kp = false;
    if (lane < nsb2) {
        const double bnd = it.sbound[(size_t)t * nsb2 + lane];
        kp = (bnd > pl.thr) && bnd >= L;
    }
    const unsigned long long bal = __ballot(kp);
    if (!bal) return;
    int base = 0;
    if (lane == 0) {
        unsigned long long nb = 0;
        for (unsigned long long mm = bal; mm; mm &= mm - 1) {
            const int sb = __ffsll((long long)mm) - 1;
            const int a = sb % pl.nsbx, b = sb / pl.nsbx;
            nb += (unsigned long long)(min(kSB, pl.ncx - kSB * a) * min(kSB, pl.ncy - kSB * b));
        }
        atomicAdd(&it.rec->coarse_evals, nb);
        base = atomicAdd(W.cnt + 16 * j, __popcll(bal));
        if (it.tedge[t] == it.gen) W.al[(size_t)j * W.tmax + atomicAdd(W.cnt + 16 * j + 1, 1)] = t;
    }
    base = __shfl(base, 0, 64);
    if (kp) W.sbl[(size_t)j * W.region + base + __popcll(bal & ((1ull << lane) - 1ull))] = t << 6 | lane;
}

// Inclusive prefix of the items' counters `which` over lanes 0..n-1 (every
// lane of the wave computes it); returns the total.
__device__ __forceinline__ int list_prefix(const WorkList& W, int which, int n, int& c)
{
    const int lane = threadIdx.x & 63;
    c = lane < n ? W.cnt[16 * lane + which] : 0;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const int u = __shfl_up(c, off, 64);
        if (lane >= off) c += u;
    }
    return __shfl(c, 63, 64);
}

// Four listed superblocks per wave (grid-stride over the list): lane =
// (superblock, member block), every lane walks the beams in order with
// pipelined gathers (seq_sum: the reference's sequential fp64 sum); cflag is
// 0 here, k_unsafe_list then redoes the edge angles' blocks.  The four beam
// rows are staged in chunks of kLC beams (4 KB of LDS per wave; r03's whole
// rows, 4 * Nv ints = 17 KB for config 2, capped the kernel at 9 waves per
// CU): the next chunk is loaded into registers while the current one is
// summed, then written to LDS; the sum carries over the chunks in beam order
// (seq_sum_from).
#ifndef LGS_LC
#define LGS_LC 256
#endif
#ifndef LGS_LIST_PIPE4
#define LGS_LIST_PIPE4 0   // 1: four gather batches in flight per lane (seq_sum_from4)
#endif
constexpr int kLC = LGS_LC;
constexpr int kLCPad = (LGS_LIST_PIPE4 ? 4 : 2) * kPipe;   // look-ahead entries past a staged chunk
static_assert(kLC % 64 == 0, "whole waves per chunk row");
__global__ __launch_bounds__(64) void k_coarse_list_c(Items items, WorkList W, int n, const double* __restrict__ zero, DevTs dts)
{
    const DtsScope dts_scope(dts);
    __shared__ int s_cb[4][kLC + kLCPad];
    const int lane = threadIdx.x, g4 = lane >> 4, m = lane & 15;
    int c;
    const int total = list_prefix(W, 0, n, c);
    const bool lean = items[0].lean != 0;   // the batch's items all run lean or none
    constexpr int kOff = -(1 << 30);
    constexpr int PER = kLC / 64;
#if LGS_LIST_XCD
    // XCD-aware split (r06): workgroups go to the 8 XCDs round-robin, so
    // consecutive quads -- one item's superblocks -- landed on every XCD and
    // each XCD's L2 held every item's planes; XCD x now takes the x-th eighth
    // of the list (items contiguous), its workgroups grid-striding over it
    const int nq = (total + 3) >> 2, xcd = blockIdx.x & 7, per = gridDim.x >> 3;
    const int qe = (int)(((long long)nq * (xcd + 1)) >> 3);
    for (int qd = (int)(((long long)nq * xcd) >> 3) + (int)(blockIdx.x >> 3); qd < qe; qd += per) {
        const int e0 = 4 * qd;   // wave-uniform
#else
    for (int e0 = 4 * blockIdx.x; e0 < total; e0 += 4 * gridDim.x) {   // wave-uniform
#endif
        const int e = e0 + g4;
        const bool has = e < total;
        int j = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int jq = __popcll(__ballot(lane < n && c <= e0 + q));
            if (g4 == q) j = jq;
        }
        if (!has) j = 0;
        const int cprev = __shfl(c, max(j - 1, 0), 64);
        const int before = j > 0 ? cprev : 0;
        const MatchItem& it = items[j];
        const RtcsmPlan& pl = it.pl;
        const int ent = has ? W.sbl[(size_t)j * W.region + (e - before)] : 0;
        const int t = ent >> 6, sb = ent & 63;
        const int Nv = has ? pl.Nv : 0;
        const int* __restrict__ cbr = it.cbase + (size_t)t * pl.Nv;
        int nmax = Nv;
#pragma unroll
        for (int off = 16; off < 64; off <<= 1) nmax = max(nmax, __shfl_xor(nmax, off, 64));
        const int nsbx = max(pl.nsbx, 1);
        const int jx = kSB * (sb % nsbx) + (m & 3), jy = kSB * (sb / nsbx) + (m >> 2);
        const bool active = has && jx < pl.ncx && jy < pl.ncy;
        const double* __restrict__ lane_base = it.cmap + (active ? jy * pl.Wqp + jx : 0);
        int pre[4][PER];
        auto fetch_chunk = [&](int v0) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int nq = __shfl(Nv, 16 * q, 64);
                if (lean) {   // the group's row formed here (lean_cell), its item and angle wave-uniform
                    const int jq = __builtin_amdgcn_readfirstlane(__shfl(j, 16 * q, 64));
                    const int tq = __builtin_amdgcn_readfirstlane(__shfl(t, 16 * q, 64));
                    const MatchItem& iq = items[jq];
#pragma unroll
                    for (int i = 0; i < PER; ++i) {
                        const int v = v0 + lane + 64 * i;
                        pre[q][i] = v < nq ? lean_coarse_base(iq, tq, v) : kOff;
                    }
                    continue;
                }
                const int* row = (const int*)__shfl((unsigned long long)cbr, 16 * q, 64);
#pragma unroll
                for (int i = 0; i < PER; ++i) {
                    const int v = v0 + lane + 64 * i;
                    pre[q][i] = v < nq ? gload(row + v) : kOff;   // past a row: the zero cell
                }
            }
#ifdef LGS_CHECK_OFFSETS
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int jq = __builtin_amdgcn_readfirstlane(__shfl(j, 16 * q, 64));
                const int tq = __builtin_amdgcn_readfirstlane(__shfl(t, 16 * q, 64));
                const int nq = __shfl(Nv, 16 * q, 64);
#pragma unroll
                for (int i = 0; i < PER; ++i) {
                    const int v = v0 + lane + 64 * i;
                    if (v < nq) LGS_CHK_COARSE(items[jq].pl, pre[q][i], tq, v);
                }
            }
#endif
        };
        fetch_chunk(0);
        double sum = 0.0;
        for (int v0 = 0; v0 < nmax; v0 += kLC) {   // wave-uniform
            // one wave: its LDS operations run in order, so the previous
            // chunk's reads are done before these writes
#pragma unroll
            for (int q = 0; q < 4; ++q) {
#pragma unroll
                for (int i = 0; i < PER; ++i) s_cb[q][lane + 64 * i] = pre[q][i];
                if (lane < kLCPad) s_cb[q][kLC + lane] = kOff;   // seq_sum's look-ahead
            }
            if (v0 + kLC < nmax) fetch_chunk(v0 + kLC);
            const int cnt = min(kLC, nmax - v0);
            const int* __restrict__ my = s_cb[g4];
#if LGS_LIST_PIPE4
            sum = seq_sum_from4<int>(sum, cnt, [&](int v) { return my[v]; },
                                     [&](const int& cc) { return (active && cc != kOff) ? lane_base + cc : zero; });
#else
            sum = seq_sum_from<int>(sum, cnt, [&](int v) { return my[v]; },
                                    [&](const int& cc) { return (active && cc != kOff) ? lane_base + cc : zero; });
#endif
        }
        if (active) {
            const long long k = (long long)t * pl.P + (long long)jx * pl.ncy + jy;
            it.cscore[k] = sum;
            it.cflag[k] = 0;
        }
    }
}

// The unsafe test of the listed edge angles (k_keep), one angle at a time per
// workgroup (grid-stride).
__global__ __launch_bounds__(64 * kLaneWaves) void k_unsafe_list(Items items, WorkList W, int n,
                                                                 const double* __restrict__ zero, DevTs dts)
{
    const DtsScope dts_scope(dts);
    const int lane = threadIdx.x & 63;
    int c;
    const int total = list_prefix(W, 1, n, c);
    for (int a = blockIdx.x; a < total; a += gridDim.x) {   // workgroup-uniform
        const int j = __popcll(__ballot(lane < n && c <= a));
        const int cprev = __shfl(c, max(j - 1, 0), 64);
        const int before = j > 0 ? cprev : 0;
        unsafe_angle(items[j], W.al[(size_t)j * W.tmax + (a - before)]);
    }
}

// Fine scores of one block by one wave: lane q owns pose (xo = q % lr,
// yo = q / lr) and runs the pipelined sequential sum over the beams.  The
// reference visits x outer, y inner (:239-240), so its order index is
// o = xo*lr + yo; ties resolve to the smallest o.  The block's angle row of
// beam indices is staged in LDS first (sidx, Nv + 2*kPipe entries), so the
// per-batch index fetch is an LDS broadcast instead of a scalar-cache miss.
// The workgroup is this one wave.
__device__ void eval_block(const RtcsmPlan& pl, const double* __restrict__ grid,
                           const int2* __restrict__ idx, const double* __restrict__ zero,
                           long long k, int2* sidx, double& f, int& pos)
{
    const int tt = (int)(k / pl.P);
    const int rem = (int)(k % pl.P);
    const int jx = rem / pl.ncy, jy = rem % pl.ncy;
    const int lr = pl.low_res;
    const int npose = lr * lr;
    const int W = pl.W, H = pl.H;
    const int2* __restrict__ id = idx + (size_t)tt * pl.Nv;
    const int lane = threadIdx.x & 63;
    __syncthreads();
    stage_lds(sidx, id, pl.Nv);
    for (int v = pl.Nv + lane; v < pl.Nv + 2 * kPipe; v += 64) sidx[v] = make_int2(-(1 << 28), -(1 << 28));
    __syncthreads();
    double bv = -1.0;
    long long bo = LLONG_MAX;
    for (int q = lane; q - lane < npose; q += 64) {   // wave-uniform trip count
        const bool act = q < npose;
        const int xo = q % lr, yo = q / lr;
        const int xf = -pl.win_x + jx * lr + xo, yf = -pl.win_y + jy * lr + yo;
        const double s = seq_sum<int2>(pl.Nv, [&](int v) { return sidx[v]; }, [&](const int2& c) {
            const int x = c.x + xf, y = c.y + yf;
            const bool inb = act & ((unsigned)x < (unsigned)W) & ((unsigned)y < (unsigned)H);
            const unsigned off = (unsigned)(y * W + x);
            return inb ? grid + off : zero;
        });
        const long long o = (long long)xo * lr + yo;
        if (act && better(s, o, bv, bo)) {
            bv = s;
            bo = o;
        }
    }
    for (int off = 32; off > 0; off >>= 1) {
        const double ov = __shfl_xor(bv, off, 64);
        const long long ok = __shfl_xor(bo, off, 64);
        if (better(ov, ok, bv, bo)) {
            bv = ov;
            bo = ok;
        }
    }
    f = bv;
    pos = (int)bo;
}

// Transposed block evaluation for a compile-time window LR (LR <= 16): the
// workgroup has LR waves, wave w owns block row yo = w (poses xo = 0..LR-1).
// lane = beam of a 64-beam chunk: it gathers the LR cells of its beam in the
// wave's row (independent loads), stores them to LDS row xo, and lanes
// xo < LR then add their row in beam order (the reference's sequential sum).
// Two chunks of gathers are kept in flight ahead of the adds (ping-pong, no
// register copies).  Beam indices of the angle row are staged in LDS first.
// Ties resolve to the smallest reference order index o = xo*LR + yo.
constexpr int kMaxChunks = 32;   // transposed evaluator handles Nv <= 2048
typedef double d2a8 __attribute__((ext_vector_type(2), aligned(8)));


// row >= 0 (row split): the workgroup is one wave that evaluates block row
// yo = row only; (f, pos) is then that row's best, and the caller combines the
// LR rows (k_replay).
template <int LR, int DEPTH = 2>
__device__ void eval_block_t(const RtcsmPlan& pl, const double* __restrict__ grid,
                             const int2* __restrict__ idx, const double* __restrict__ zero,
                             long long k, char* smem, double* sv, long long* sk, double& f,
                             int& pos, int row = -1)
{
    constexpr int LD = 65;
    const int tt = (int)(k / pl.P);
    const int rem = (int)(k % pl.P);
    const int jx = rem / pl.ncy, jy = rem % pl.ncy;
    const int wave = row >= 0 ? row : (int)(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int xc = -pl.win_x + jx * LR, yr = -pl.win_y + jy * LR + wave;
    const int W = pl.W, H = pl.H, Nv = pl.Nv;
    const int2* __restrict__ id = idx + (size_t)tt * Nv;
    int2* sidx = (int2*)smem;                                        // [Nv]
    double* bufs = (double*)(smem + sizeof(int2) * (size_t)((Nv + 1) & ~1)) + (row >= 0 ? 0 : wave) * 2 * LR * LD;
    const int nchunk = (Nv + 63) / 64;

    __syncthreads();
    stage_lds(sidx, id, Nv);
    __syncthreads();


    // chunks of gathers in flight: 2 for the LR-wave block evaluation (depth 4
    // there made k_fine slower, 36 vs 27 us: register pressure at LR waves per
    // workgroup); the one-wave row split affords more
    constexpr int kDepth = DEPTH;
    double r[DEPTH][LR];
    // A lane's LR cells are consecutive doubles of one row: when the whole
    // run is inside the map (all but the border beams) it is fetched with
    // 16-byte loads (8-byte aligned, which gfx950 global loads accept), i.e.
    // 3 instead of 5 memory instructions for LR = 5 -- the per-CU cache
    // lookups, not the bytes, bound this gather.
    auto gather = [&](int c, double (&r)[LR]) {
        const int b = c * 64 + lane;
        const int2 ij = sidx[min(b, Nv - 1)];
        const bool bv = b < Nv;
        const int x0 = ij.x + xc, y = ij.y + yr;
        bool full = false;
        // 16-byte loads for the inner runs (LR waves, depth 2: fewer memory
        // instructions per CU); the row split (depth > 2) keeps every lane's
        // instruction sequence identical, so the waits count exactly
        if constexpr (LR == 5 && DEPTH == 2) full = bv & ((unsigned)y < (unsigned)H) & (x0 >= 0) & (x0 + LR - 1 < W);
        if (full) {
            const double* p = grid + (unsigned)(y * W + x0);
            typedef const __attribute__((address_space(1))) d2a8 gd2a8_t;
            const d2a8 a = *(gd2a8_t*)p;
            const d2a8 e = *(gd2a8_t*)(p + 2);
            r[0] = a.x;
            r[1] = a.y;
            r[2] = e.x;
            r[3] = e.y;
            r[LR - 1] = gload(p + 4);
        } else {
#pragma unroll
            for (int q = 0; q < LR; ++q) {
                const int x = x0 + q;
                const bool inb = bv & ((unsigned)x < (unsigned)W) & ((unsigned)y < (unsigned)H);
                const unsigned off = (unsigned)(y * W + x);
                r[q] = gload(inb ? grid + off : zero);
            }
        }
    };
    auto store = [&](const double (&r)[LR], double* buf) {
#pragma unroll
        for (int q = 0; q < LR; ++q) buf[q * LD + lane] = r[q];
        // no fence: a wave's LDS operations execute in order, and a release
        // fence here would also wait for the prefetch gathers in flight
        __builtin_amdgcn_wave_barrier();
    };
    double acc = 0.0;
    auto add_chunk = [&](int c, const double* buf) {
        if (lane < LR) {
            const double* row = buf + lane * LD;
            const int cnt = min(64, Nv - c * 64);
            double s = acc;
            if (cnt == 64) {
#pragma unroll 16
                for (int b = 0; b < 64; ++b) s += row[b];
            } else {
                for (int b = 0; b < cnt; ++b) s += row[b];
            }
            acc = s;
        }
    };
    // kDepth chunks of gathers in flight ahead of the adds (alternating register
    // sets), fully unrolled over at most kMaxChunks chunks: without a loop
    // header there are no phi copies of in-flight registers, so each store
    // waits only for the oldest batch; sched_barrier keeps each batch's
    // gathers contiguous and in program order.  The in-order LDS of a wave
    // makes two row buffers enough (a store never overtakes the previous
    // chunk's reads).
    static_for_step<0, DEPTH, 1>([&](auto dd) {
        gather(decltype(dd)::value, r[decltype(dd)::value]);
        __builtin_amdgcn_sched_barrier(0);
        return true;
    });
    auto stage = [&](int c, double (&x)[LR], double* buf) {
        store(x, buf);
        __builtin_amdgcn_sched_barrier(0);
        gather(c + kDepth, x);
        __builtin_amdgcn_sched_barrier(0);
        add_chunk(c, buf);
    };
    static_for_step<0, kMaxChunks, kDepth>([&](auto cc) {
        constexpr int c = decltype(cc)::value;
        bool go = true;
        static_for_step<0, DEPTH, 1>([&](auto dd) {
            constexpr int d = decltype(dd)::value;
            if (c + d >= nchunk) {
                go = false;
                return false;
            }
            stage(c + d, r[d], bufs + (d & 1) * LR * LD);
            return true;
        });
        return go;
    });
    double bv = -1.0;
    long long bo = LLONG_MAX;
    if (lane < LR) {
        bv = acc;
        bo = (long long)lane * LR + wave;
    }
    if (row >= 0) {
        for (int off = 32; off > 0; off >>= 1) {
            const double ov = __shfl_xor(bv, off, 64);
            const long long ok = __shfl_xor(bo, off, 64);
            if (better(ov, ok, bv, bo)) {
                bv = ov;
                bo = ok;
            }
        }
    } else {
        block_argmax(bv, bo, sv, sk);
    }
    f = bv;
    pos = (int)bo;
}

template <int LR>
constexpr size_t eval_t_smem(int Nv)
{
    return sizeof(int2) * (size_t)((Nv + 1) & ~1) + sizeof(double) * 2 * LR * LR * 65;
}

// k_seed: best safe coarse block -> its fine max is a lower bound of the
// final score (every safe block's fine max is <= the reference's final score).
// LR > 0: transposed evaluation with LR waves; LR == 0: generic one-wave path.
template <int LR>
__global__ __launch_bounds__(LR > 0 ? 64 * LR : 64) void k_seed(Items items, const double* __restrict__ zero,
                                                                 int force_dense)
{
    const MatchItem& it = items[blockIdx.y];
    const RtcsmPlan& pl = it.pl;
    const double* __restrict__ grid = it.grid;
    const int2* __restrict__ idx = it.idx;
    const double* __restrict__ part_c = it.part_c;
    const long long* __restrict__ part_k = it.part_k;
    const int nparts = it.nparts;
    double* __restrict__ Lout = it.Lp;
    extern __shared__ char smem[];
    __shared__ double sv[16];
    __shared__ long long sk[16];
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
    if constexpr (LR > 0)
        eval_block_t<LR>(pl, grid, idx, zero, bk, smem, sv, sk, f, pos);
    else
        eval_block(pl, grid, idx, zero, bk, (int2*)smem, f, pos);
    if (threadIdx.x == 0) *Lout = f;
}

// k_seed_super (superblock pruning): kSeedCands workgroups of 1024 threads.
//  1. every workgroup picks the same kSeedCands best superblocks above thr
//     among k_super's per-chunk bests (rows that may hold unsafe blocks are
//     excluded there); workgroup b takes candidate b;
//  2. its 16 members' coarse scores summed in any order (they only choose
//     which block to refine: any safe block's fine max is a valid L);
//  3. the best member's lr x lr fine scores, also summed in any order, each
//     lowered by its rounding bound (4 (Nv + 2) eps sum|x| >= the gap to the
//     reference-order sum), so L_b <= that block's exact fine max <= the
//     reference's final score;
//  4. L_b goes to Lc[b] (-inf without a candidate); k_coarse_rows and
//     k_select use L = max_b L_b.
// Loads are issued in independent batches of 16 (one workgroup per
// candidate: each one's duration is its latency chain).
constexpr int kSeedMaxNv = 2048;   // LDS: the candidate row (Nv ints / int2)
constexpr int kSeedRegParts = 4;   // parts held in registers per thread
// gathers per batch (one memory round trip each) in the member and fine
// stages: a 1081-beam scan needs 17 per thread in the member stage and 34 in
// the fine stage (25 poses padded to 32 lanes)
constexpr int kSeedB1 = 24, kSeedB2 = 36;

// k_seed_super step 3: the fine scores of block mk (coarse score cmk, sum of
// magnitudes cma) over its lr x lr poses, any order, rounding-bounded; returns
// L_b = min(fine max, cmk), both lowered by their rounding bounds (uniform
// over the workgroup).  sidx: the block's angle's beam cells in LDS.
__device__ __forceinline__ double seed_fine(const RtcsmPlan& pl, const double* __restrict__ grid, const double* __restrict__ zero,
                            const int2* sidx, long long mk, double cmk, double cma, double* red, double* reda,
                            double* sv)
{
    const int tid = threadIdx.x;
    const int Nv = pl.Nv;
    // 3. fine scores of block mk, any order, rounding-bounded
    const int rem = (int)(mk % pl.P);
    const int bjx = rem / pl.ncy, bjy = rem % pl.ncy;
    const int lr = pl.low_res, npose = lr * lr;
    int QP = 1;
    while (QP < npose) QP <<= 1;   // npose <= 1024
    const int G = (int)blockDim.x / QP;
    const int q = tid % QP, gq = tid / QP;
    double fs = 0.0, fa = 0.0;
    if (q < npose) {
        const int xo = q % lr, yo = q / lr;
        const int xf = -pl.win_x + bjx * lr + xo, yf = -pl.win_y + bjy * lr + yo;
        const int W = pl.W, H = pl.H;
        const int cnt = (gq < Nv) ? (Nv - gq + G - 1) / G : 0;   // beams gq, gq + G, ...
        for (int i0 = 0; i0 < cnt; i0 += kSeedB2) {
            double buf[kSeedB2];
#pragma unroll
            for (int j = 0; j < kSeedB2; ++j) {
                const int2 c = sidx[gq + G * min(i0 + j, cnt - 1)];
                const int x = c.x + xf, y = c.y + yf;
                const bool inb = (i0 + j < cnt) & ((unsigned)x < (unsigned)W) & ((unsigned)y < (unsigned)H);
                buf[j] = gload(inb ? grid + (unsigned)(y * W + x) : zero);
            }
#pragma unroll
            for (int j = 0; j < kSeedB2; ++j) {
                fs += buf[j];
                fa += fabs(buf[j]);
            }
        }
    }
    __syncthreads();
    // pose totals: lanes of a wave with equal q (QP < 64) by shuffles,
    // then the waves through LDS
    for (int off = QP; off < 64; off <<= 1) {
        fs += __shfl_xor(fs, off, 64);
        fa += __shfl_xor(fa, off, 64);
    }
    const int wq = min(QP, 64);
    if ((tid & 63) < wq) {
        red[(tid >> 6) * wq + (tid & 63)] = fs;
        reda[(tid >> 6) * wq + (tid & 63)] = fa;
    }
    __syncthreads();
    if (tid < 64) {
        double lv = -INFINITY;
        // poses q: this lane's q (QP <= 64) or q = tid + 64 j (QP > 64)
        for (int q0 = tid; q0 < npose; q0 += 64) {
            double ts = 0.0, ta = 0.0;
            if (QP <= 64) {
                for (int j = 0; j < (int)(blockDim.x >> 6); ++j) {
                    ts += red[j * wq + q0];
                    ta += reda[j * wq + q0];
                }
            } else {   // QP > 64: a wave holds 64 poses of one group
                for (int j = 0; j < (int)(blockDim.x >> 6); ++j)
                    if (((j * 64) % QP) == (q0 / 64) * 64) {
                        ts += red[j * wq + (q0 & 63)];
                        ta += reda[j * wq + (q0 & 63)];
                    }
            }
            lv = fmax(lv, ts - (4.0 * (double)(Nv + 2) * 0x1p-53) * ta);
        }
        for (int off = 32; off > 0; off >>= 1) lv = fmax(lv, __shfl_xor(lv, off, 64));
        if (tid == 0) sv[0] = lv;
    }
    __syncthreads();
    // s_final >= f_mk if the reference refines block mk, else >= c_mk
    // (it skips the block only when c_mk <= scoreMax), so min(f, c) is a
    // lower bound of the result for ANY block, unsafe ones included
    // (their f may exceed c); both terms rounding-bounded from below
    return fmin(sv[0], cmk - (4.0 * (double)(Nv + 2) * 0x1p-53) * cma);
}

// Wide seed for batches (r05, LGS_OPT_SEED_WIDE): k_seed_members, one
// 256-thread workgroup per candidate superblock b < kSeedWide, runs steps 1-2
// (the candidate as the b-th best of k_super's per-chunk bests by rank, the
// parts staged in LDS) and publishes its best member (coarse score, block,
// sum of magnitudes) to it.seedm; then k_seed_super MODE 2, kSeedCands
// workgroups, takes the b-th best of those members by coarse score and runs
// steps 3-4 on it (MODE 0: steps 1-4 as above).  The final best block was its
// superblock's best member in every config-2 query measured, and that
// superblock ranked 2-12 by bound where the four candidates missed it
// (tools/diag_seed.py): a third of the queries then scored ~4.5x the coarse
// blocks.  Sixteen candidates cost member sums, not fine scores.
constexpr int kSeedMembersThreads = 256;
#ifndef LGS_SEED2_THREADS
#define LGS_SEED2_THREADS 1024   // k_seed_super<2> workgroup (MODE 2 takes any multiple of 64 up to 1024)
#endif
constexpr int kSeedWideMaxParts = 1024;   // parts held in one wave's registers (larger searches: block rounds)
// Candidate b of the seed, by one whole wave: the parts in registers (16 per
// lane), b + 1 rounds of a wave argmax, each taking the best part out (the
// seed's order: bound, then block order); a candidate needs a bound above
// thr.  LLONG_MAX: no candidate b.  (r05: the block-wide argmax rounds, two
// barriers each, were the seed's longest chain for its last workgroups.)
__device__ __forceinline__ long long seed_pick_wave(const MatchItem& it, const RtcsmPlan& pl, int b)
{
    const int lane = (int)__lane_id();
    const int nparts = it.nparts;
    constexpr int R = kSeedWideMaxParts / 64;
    double v[R];
    long long k[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int i = lane + 64 * r;
        v[r] = (i < nparts) ? it.part_c[i] : -INFINITY;
        k[r] = (i < nparts) ? it.part_k[i] : LLONG_MAX;
    }
    long long pick = LLONG_MAX;
    for (int round = 0; round <= b; ++round) {
        double bv = -INFINITY;
        long long bk = LLONG_MAX;
#pragma unroll
        for (int r = 0; r < R; ++r)
            if (better(v[r], k[r], bv, bk)) {
                bv = v[r];
                bk = k[r];
            }
        for (int off = 32; off > 0; off >>= 1) {
            const double ov = __shfl_xor(bv, off, 64);
            const long long ok = __shfl_xor(bk, off, 64);
            if (better(ov, ok, bv, bk)) {
                bv = ov;
                bk = ok;
            }
        }
        if (bk == LLONG_MAX || bv == -INFINITY || !(bv > pl.thr)) break;   // uniform: no candidate b
        if (round == b) pick = bk;
#pragma unroll
        for (int r = 0; r < R; ++r)
            if (k[r] == bk) v[r] = -INFINITY, k[r] = LLONG_MAX;
    }
    return pick;
}
__global__ __launch_bounds__(kSeedMembersThreads) void k_seed_members(Items items, DevTs dts)
{
#if LGS_XCD2
    const Blk sbk = xcd_block();   // an item's workgroups on one XCD (its planes in one L2)
#else
    const Blk sbk{ (int)blockIdx.x, (int)blockIdx.y, (int)blockIdx.z };
#endif
    const DtsScope dts_scope(dts);
    const MatchItem& it = items[sbk.y];
    const RtcsmPlan& pl = it.pl;
    const double* __restrict__ cmap = it.cmap;
    if (sbk.x == 0 && threadIdx.x < 2 && it.keepc) it.keepc[threadIdx.x] = 0;   // before k_keep
    extern __shared__ char smem[];
    __shared__ double red[2][kSeedMembersThreads / 64][16];
    __shared__ long long s_cand;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int nsb2 = pl.nsbx * pl.nsby;
    const int Nv = pl.Nv;
    // 1. candidate b by wave 0 (seed_pick_wave)
    if (w == 0) {
        const long long pick = seed_pick_wave(it, pl, (int)sbk.x);
        if (lane == 0) s_cand = pick;
    }
    __syncthreads();
    double* out = it.seedm + 3 * sbk.x;
    const long long ck = s_cand;
    if (ck == LLONG_MAX) {   // no candidate b: an empty member
        if (tid == 0) {
            out[0] = -INFINITY;
            out[1] = __builtin_bit_cast(double, (long long)LLONG_MAX);
            out[2] = 0.0;
        }
        return;
    }
    const int ct = (int)(ck / nsb2), csb = (int)(ck % nsb2);
    // 2. member sums: member m = tid % 16, beam group g = tid / 16 (16 groups)
    int* srow = (int*)smem;   // [Nv]
    stage_cbase_row(srow, it, ct, Nv);
    __syncthreads();
    constexpr int G = kSeedMembersThreads / 16;
    const int m = tid & 15, g = tid >> 4;
    const int jx = kSB * (csb % pl.nsbx) + (m & 3);
    const int jy = kSB * (csb / pl.nsbx) + (m >> 2);
    const bool valid = jx < pl.ncx && jy < pl.ncy;
    double s = 0.0, sa = 0.0;   // member sum and its sum of magnitudes (any order)
    if (valid) {
        const double* __restrict__ lb = cmap + (jy * pl.Wqp + jx);
        const int cnt = (g < Nv) ? (Nv - g + G - 1) / G : 0;   // beams g, g + G, ...
        double acc[4] = { 0.0, 0.0, 0.0, 0.0 };
        for (int i0 = 0; i0 < cnt; i0 += kSeedB1) {
            double buf[kSeedB1];
#pragma unroll
            for (int j = 0; j < kSeedB1; ++j) {
                const int i = min(i0 + j, cnt - 1);
                buf[j] = (i0 + j < cnt) ? gload(lb + srow[g + G * i]) : 0.0;
            }
#pragma unroll
            for (int j = 0; j < kSeedB1; ++j) {
                acc[j & 3] += buf[j];
                sa += fabs(buf[j]);
            }
        }
        s = (acc[0] + acc[1]) + (acc[2] + acc[3]);
    }
    // member totals: the wave's 4 groups by shuffles, then the waves
    s += __shfl_xor(s, 16, 64);
    s += __shfl_xor(s, 32, 64);
    sa += __shfl_xor(sa, 16, 64);
    sa += __shfl_xor(sa, 32, 64);
    if (lane < 16) {
        red[0][w][m] = s;
        red[1][w][m] = sa;
    }
    __syncthreads();
    if (tid < 64) {
        double mv = -1.0, ma = 0.0;
        long long mk = LLONG_MAX;
        if (tid < 16 && valid) {
            double tot = 0.0, tota = 0.0;
#pragma unroll
            for (int j = 0; j < kSeedMembersThreads / 64; ++j) {
                tot += red[0][j][tid];
                tota += red[1][j][tid];
            }
            mv = tot;
            ma = tota;
            mk = (long long)ct * pl.P + (long long)jx * pl.ncy + jy;
        }
        for (int off = 32; off > 0; off >>= 1) {
            const double ov = __shfl_xor(mv, off, 64);
            const double oa = __shfl_xor(ma, off, 64);
            const long long ok = __shfl_xor(mk, off, 64);
            if (better(ov, ok, mv, mk)) {
                mv = ov;
                ma = oa;
                mk = ok;
            }
        }
        if (tid == 0) {
            out[0] = mv;
            out[1] = __builtin_bit_cast(double, mk);
            out[2] = ma;
        }
    }
}

template <int MODE>
__global__ __launch_bounds__(1024) void k_seed_super(Items items, const double* __restrict__ zero, DevTs dts)
{
#if LGS_XCD2
    const Blk sbk = xcd_block();   // an item's workgroups on one XCD (its planes in one L2)
#else
    const Blk sbk{ (int)blockIdx.x, (int)blockIdx.y, (int)blockIdx.z };
#endif
    const DtsScope dts_scope(dts);
    const MatchItem& it = items[sbk.y];
    const RtcsmPlan& pl = it.pl;
    const double* __restrict__ grid = it.grid;
    const double* __restrict__ cmap = it.cmap;
    const double* __restrict__ part_c = it.part_c;
    const long long* __restrict__ part_k = it.part_k;
    const int nparts = it.nparts;
    double* __restrict__ Lc = it.Lc;
    RtcsmRecord* rec = it.rec;
    if (MODE == 0 && sbk.x == 0 && threadIdx.x < 2 && it.keepc) it.keepc[threadIdx.x] = 0;   // before k_keep
    extern __shared__ char smem[];
    __shared__ double sv[16];
    __shared__ long long sk[16];
    __shared__ long long cand[kSeedCands];
    __shared__ double red[1024];
    __shared__ double reda[1024];
    const int tid = threadIdx.x;
    const int nsb2 = pl.nsbx * pl.nsby;
    const int Nv = pl.Nv;
    LGS_PROBE_DECL;
    LGS_PROBE_MARK();
    double Lmine = -INFINITY;
    if constexpr (MODE == 2) {
        // the b-th best published member (coarse score, then block order)
        if (tid < 64) {
            const bool ok = tid < it.nseedm;
            const double mv = ok ? it.seedm[3 * tid] : -INFINITY;
            const long long mk = ok ? __builtin_bit_cast(long long, it.seedm[3 * tid + 1]) : LLONG_MAX;
            const double ma = ok ? it.seedm[3 * tid + 2] : 0.0;
            const bool valid = ok && mk != LLONG_MAX && mv > -INFINITY;
            int rank = 0;
            for (int j = 0; j < it.nseedm; ++j) {
                const double ov = __shfl(mv, j, 64);
                const long long okk = __shfl(mk, j, 64);
                const bool ovalid = __shfl((int)valid, j, 64) != 0;
                rank += (ovalid && j != tid && better(ov, okk, mv, mk)) ? 1 : 0;
            }
            if (tid == 0) sk[0] = LLONG_MAX;
            __builtin_amdgcn_wave_barrier();
            if (valid && rank == (int)sbk.x) {
                sk[0] = mk;
                sv[1] = mv;
                sv[2] = ma;
            }
        }
        __syncthreads();
        if (sk[0] != LLONG_MAX) {
            const int ct = (int)(sk[0] / pl.P);
            int2* sidx = (int2*)(smem + ((sizeof(int) * (size_t)Nv + 15) & ~(size_t)15));   // [Nv]
            stage_idx_row(sidx, it, ct, Nv);
            __syncthreads();
            Lmine = seed_fine(pl, grid, zero, sidx, sk[0], sv[1], sv[2], red, reda, sv);
        }
        if (tid == 0) {
            Lc[sbk.x] = Lmine;
            if (sbk.x == 0) rec->coarse_evals = 0ull;   // k_coarse_rows counts
        }
        return;
    }
    int nc = 0;
    if (nparts <= kSeedWideMaxParts) {   // candidate b by one wave
        __shared__ int s_nc;
        if (tid < 64) {
            const long long pick = seed_pick_wave(it, pl, (int)sbk.x);
            if (tid == 0) {
                cand[sbk.x] = pick;
                s_nc = (pick != LLONG_MAX) ? (int)sbk.x + 1 : 0;
            }
        }
        __syncthreads();
        nc = s_nc;
    } else {
        double pv[kSeedRegParts];
        long long pk[kSeedRegParts];
#pragma unroll
        for (int j = 0; j < kSeedRegParts; ++j) {
            const int i = tid + j * 1024;
            pv[j] = (i < nparts) ? part_c[i] : -INFINITY;
            pk[j] = (i < nparts) ? part_k[i] : LLONG_MAX;
        }
        for (; nc <= (int)sbk.x; ++nc) {   // candidates 0..sbk.x
            double bv = -INFINITY;
            long long bk = LLONG_MAX;
#pragma unroll
            for (int j = 0; j < kSeedRegParts; ++j)
                if (better(pv[j], pk[j], bv, bk)) {
                    bv = pv[j];
                    bk = pk[j];
                }
            for (int i = tid + kSeedRegParts * 1024; i < nparts; i += 1024) {   // large searches only
                bool taken = false;
                for (int j = 0; j < nc; ++j) taken |= cand[j] == part_k[i];
                if (!taken && better(part_c[i], part_k[i], bv, bk)) {
                    bv = part_c[i];
                    bk = part_k[i];
                }
            }
            block_argmax(bv, bk, sv, sk);
            if (bk == LLONG_MAX || bv == -INFINITY || !(bv > pl.thr)) break;   // uniform
            if (tid == 0) cand[nc] = bk;
#pragma unroll
            for (int j = 0; j < kSeedRegParts; ++j)
                if (pk[j] == bk) pv[j] = -INFINITY, pk[j] = LLONG_MAX;
            __syncthreads();
        }
    }
    LGS_PROBE_MARK();
    if (nc > (int)sbk.x) {
        const long long ck = cand[sbk.x];
        const int ct = (int)(ck / nsb2), csb = (int)(ck % nsb2);
        // 2. member sums: member m = tid % 16, beam group tid / 16 (64 groups);
        // the fine stage's beam row is staged together with the coarse one
        // (one memory round trip less on this latency chain)
        int* srow = (int*)smem;   // [Nv]
        int2* sidx = (int2*)(smem + ((sizeof(int) * (size_t)Nv + 15) & ~(size_t)15));   // [Nv]
        stage_cbase_row(srow, it, ct, Nv);
        stage_idx_row(sidx, it, ct, Nv);
        __syncthreads();
        const int m = tid & 15, g = tid >> 4;
        const int jx = kSB * (csb % pl.nsbx) + (m & 3);
        const int jy = kSB * (csb / pl.nsbx) + (m >> 2);
        const bool valid = jx < pl.ncx && jy < pl.ncy;
        double s = 0.0, sa = 0.0;   // member sum and its sum of magnitudes
        if (valid) {
            const double* __restrict__ lb = cmap + (jy * pl.Wqp + jx);
            const int cnt = (g < Nv) ? (Nv - g + 63) / 64 : 0;   // beams g, g + 64, ...
            double acc[4] = { 0.0, 0.0, 0.0, 0.0 };
            for (int i0 = 0; i0 < cnt; i0 += kSeedB1) {
                double buf[kSeedB1];
#pragma unroll
                for (int j = 0; j < kSeedB1; ++j) {
                    const int i = min(i0 + j, cnt - 1);
                    buf[j] = (i0 + j < cnt) ? gload(lb + srow[g + 64 * i]) : 0.0;
                }
#pragma unroll
                for (int j = 0; j < kSeedB1; ++j) {
                    acc[j & 3] += buf[j];
                    sa += fabs(buf[j]);
                }
            }
            s = (acc[0] + acc[1]) + (acc[2] + acc[3]);
        }
        // member totals: the wave's 4 groups by shuffles, then the 16 waves
        s += __shfl_xor(s, 16, 64);
        s += __shfl_xor(s, 32, 64);
        sa += __shfl_xor(sa, 16, 64);
        sa += __shfl_xor(sa, 32, 64);
        if ((tid & 63) < 16) {
            red[(tid >> 6) * 16 + m] = s;
            reda[(tid >> 6) * 16 + m] = sa;
        }
        __syncthreads();
        LGS_PROBE_MARK();
        if (tid < 64) {
            double mv = -1.0, ma = 0.0;
            long long mk = LLONG_MAX;
            if (tid < 16) {
                double tot = 0.0, tota = 0.0;
                for (int j = 0; j < (int)(blockDim.x >> 6); ++j) {
                    tot += red[j * 16 + tid];
                    tota += reda[j * 16 + tid];
                }
                if (valid) {
                    mv = tot;
                    ma = tota;
                    mk = (long long)ct * pl.P + (long long)jx * pl.ncy + jy;
                }
            }
            for (int off = 32; off > 0; off >>= 1) {
                const double ov = __shfl_xor(mv, off, 64);
                const double oa = __shfl_xor(ma, off, 64);
                const long long ok = __shfl_xor(mk, off, 64);
                if (better(ov, ok, mv, mk)) {
                    mv = ov;
                    ma = oa;
                    mk = ok;
                }
            }
            if (tid == 0) {
                sk[0] = mk;
                sv[1] = mv;
                sv[2] = ma;
            }
        }
        __syncthreads();
        Lmine = seed_fine(pl, grid, zero, sidx, sk[0], sv[1], sv[2], red, reda, sv);
        LGS_PROBE_MARK();
    }
    // 4. publish
    if (tid == 0) {
        Lc[sbk.x] = Lmine;
        if (sbk.x == 0) rec->coarse_evals = 0ull;   // k_coarse_rows counts
    }
    LGS_PROBE_MARK();
    LGS_PROBE_PRINT("seed(b0: cand, members, argmax, stage, fine, reduce, publish)");
}

// k_select: one workgroup per segment of kSelSeg consecutive blocks.  The
// selected blocks of a segment are written in block order to
// list[seg * kSelSeg + rank] (wave ballots + an LDS prefix over the 16
// waves) and their number to segcnt[seg]; consumers rebuild the exclusive
// prefix over segments in LDS (seg_prefix), which gives every selected block
// its position in the reference's block order.
constexpr int kSelSeg = 1024;

// sbound (superblock pruning, else nullptr): blocks of superblocks
// k_coarse_rows did not keep were never scored and are never taken (the
// same keep rule, evaluated again here).
// kSelThreads threads per segment, kSelSeg / kSelThreads keys each: the
// segment's keys in chunks of kSelThreads, each chunk compacted in key order
// after the previous ones (fewer, fuller waves than one key per thread: the
// kernel was launch-bound on ~120k mostly idle waves per batch)
// (batches: 256 threads, 36.4 -> 26.7 us per 64 scans; a lone scan keeps one
// key per thread, 6.4 vs 8.3 us: its ~120 segments do not fill the GPU)
template <int kSelThreads>
__global__ __launch_bounds__(kSelThreads) void k_select(Items items, int use_sbound, DevTs dts)
{
    const DtsScope dts_scope(dts);
    static_assert(kSelSeg % kSelThreads == 0 && kSelThreads % 64 == 0, "whole chunks of whole waves");
    const MatchItem& it = items[blockIdx.y];
    if ((int)blockIdx.x >= it.nseg) return;   // past this item's segments (uniform)
    const RtcsmPlan& pl = it.pl;
    const double* __restrict__ cscore = it.cscore;
    const uint8_t* __restrict__ cflag = it.cflag;
    const double* __restrict__ sbound = use_sbound ? it.sbound : nullptr;
    int* __restrict__ list = it.list;
    int* __restrict__ segcnt = it.segcnt;
    constexpr int kW = kSelThreads / 64, kChunks = kSelSeg / kSelThreads;
    __shared__ int s_w[kChunks][kW];
    const double L = *it.Lp;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    bool f[kChunks];
#pragma unroll
    for (int j = 0; j < kChunks; ++j) {
        const long long k = (long long)blockIdx.x * kSelSeg + j * kSelThreads + threadIdx.x;
        f[j] = false;
        if (k < pl.K) {
            bool kp = true;
            if (sbound) {
                const int t = (int)(k / pl.P), rem = (int)(k % pl.P);
                const int jx = rem / pl.ncy, jy = rem % pl.ncy;
                const double bnd = sbound[(size_t)t * pl.nsbx * pl.nsby + (jy / kSB) * pl.nsbx + jx / kSB];
                kp = (bnd > pl.thr) && bnd >= L;
            }
            if (kp) {
                const double c = cscore[k];
                f[j] = (c > pl.thr) && (cflag[k] || c >= L);
            }
        }
        const unsigned long long bal = __ballot(f[j]);
        if (lane == 0) s_w[j][wid] = __popcll(bal);
    }
    __syncthreads();
    int off = 0;   // keys of the earlier chunks, then of the earlier waves of this chunk
#pragma unroll
    for (int j = 0; j < kChunks; ++j) {
        const unsigned long long bal = __ballot(f[j]);
        int o = off;
        for (int w = 0; w < wid; ++w) o += s_w[j][w];
        if (f[j]) list[(size_t)blockIdx.x * kSelSeg + o + __popcll(bal & ((1ull << lane) - 1ull))] =
            (int)((long long)blockIdx.x * kSelSeg + j * kSelThreads + threadIdx.x);
        for (int w = 0; w < kW; ++w) off += s_w[j][w];
    }
    if (threadIdx.x == 0) segcnt[blockIdx.x] = off;
}

// pref[0..nseg] = exclusive prefix of segcnt, built in LDS by the whole
// workgroup (chunk per thread, wave scans, one LDS pass over the waves).
// ws: >= 16 ints of LDS scratch.  Ends with a barrier.
__device__ void seg_prefix(const int* __restrict__ segcnt, int nseg, int* pref, int* ws)
{
    const int nt = blockDim.x, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int chunk = (nseg + nt - 1) / nt;
    const int lo = min(tid * chunk, nseg), hi = min(lo + chunk, nseg);
    int c = 0;
    for (int i = lo; i < hi; ++i) c += segcnt[i];
    int incl = c;
    for (int off = 1; off < 64; off <<= 1) {
        const int t = __shfl_up(incl, off, 64);
        if (lane >= off) incl += t;
    }
    const int last = min(63, nt - 1 - wid * 64);
    if (lane == last) ws[wid] = incl;
    __syncthreads();
    int run = incl - c;
    for (int j = 0; j < wid; ++j) run += ws[j];
    for (int i = lo; i < hi; ++i) {
        pref[i] = run;
        run += segcnt[i];
    }
    if (tid == nt - 1) pref[nseg] = run;
    __syncthreads();
}

// segment holding dense position b: pref[lo] <= b < pref[lo + 1]
__device__ __forceinline__ int seg_of(const int* pref, int nseg, int b)
{
    int lo = 0, hi = nseg;
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (pref[mid] <= b) lo = mid;
        else hi = mid;
    }
    return lo;
}

// k_fine: the listed blocks, dense position b.  LR > 0: one single-wave
// workgroup per (block, block row) item b * LR + row = blockIdx.x,
// +gridDim.x, ... (a block's LR rows on LR CUs: the gathers of one CU's
// memory pipeline are what a block evaluation waits on); fval/fpos are
// indexed by item and k_replay combines a block's rows.  LR == 0: one wave
// per block, indexed by dense position.
constexpr int kFineDepth = 6;   // measured (lone config-2 scan): 4: 33.7 us, 5: 34.2, 6: 23.8, 7: 24.0, 8: 34.1
template <int LR>
__global__ __launch_bounds__(64) void k_fine(Items items, const double* __restrict__ zero, unsigned eval_smem)
{
    const Blk wg = { (int)blockIdx.x, (int)blockIdx.y, (int)blockIdx.z };   // (as k_coarse_rows: uneven work)
    const MatchItem& it_ = items[wg.y];
    const RtcsmPlan& pl = it_.pl;
    const double* __restrict__ grid = it_.grid;
    const int2* __restrict__ idx = it_.idx;
    const int* __restrict__ list = it_.list;
    const int* __restrict__ segcnt = it_.segcnt;
    const int nseg = it_.nseg;
    double* __restrict__ fval = it_.fval;
    int* __restrict__ fpos = it_.fpos;
    extern __shared__ char smem[];
    __shared__ double sv[16];
    __shared__ long long sk[16];
    __shared__ int ws[16];
    int* pref = (int*)(smem + eval_smem);
    LGS_PROBE_DECL;
    LGS_PROBE_MARK();
    seg_prefix(segcnt, nseg, pref, ws);
    LGS_PROBE_MARK();
    const int n = pref[nseg];
    constexpr int R = LR > 0 ? LR : 1;
    for (int it = wg.x; it < n * R; it += gridDim.x) {
        const int b = it / R;
        const int sg = seg_of(pref, nseg, b);
        const long long k = list[(size_t)sg * kSelSeg + (b - pref[sg])];
        double f;
        int pos;
        if constexpr (LR > 0)
            eval_block_t<LR, kFineDepth>(pl, grid, idx, zero, k, smem, sv, sk, f, pos, it % R);
        else
            eval_block(pl, grid, idx, zero, k, (int2*)smem, f, pos);
        if (threadIdx.x == 0) {
            fval[it] = f;
            fpos[it] = pos;
        }
        LGS_PROBE_MARK();
    }
    LGS_PROBE_PRINT("fine(seg_prefix, item0[, item1])");
}

// k_compact: one workgroup per item writes the item's selected blocks (the
// per-segment lists of k_select) dense in block order, dlist[0..n), and n.
// Wave w copies segments w, w + 4, ...
__global__ __launch_bounds__(256) void k_compact(Items items)
{
    const MatchItem& it = items[blockIdx.x];
    extern __shared__ int pref[];   // nseg + 1
    __shared__ int ws[16];
    seg_prefix(it.segcnt, it.nseg, pref, ws);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int sg = w; sg < it.nseg; sg += 4) {
        const int c = pref[sg + 1] - pref[sg];
        const int* __restrict__ src = it.list + (size_t)sg * kSelSeg;
        int* __restrict__ dst = it.dlist + pref[sg];
        for (int i = lane; i < c; i += 64) dst[i] = src[i];
    }
    if (threadIdx.x == 0) *it.nsel = pref[it.nseg];
}

// k_fine_lanes: EvaluateHighResolutionMap (:227-256) for every selected block
// of the batch, one wave per block and one LANE per fine pose (lr * lr <= 64
// lanes): each lane walks the beams in order with pipelined gathers (seq_sum:
// the reference's sequential fp64 sum), so the add chains of all poses run
// side by side -- the transposed evaluator (eval_block_t) ran one block row
// per wave with LR adding lanes.  The batch's blocks form one global index
// space (items' counts prefix-summed in LDS), so a scan with thousands of
// selected blocks (tie-heavy maps) spreads over the whole GPU instead of
// loading its own workgroups.  Block max and its first position in the
// reference's (x outer, y inner) order: lane q = xo * lr + yo, ties to the
// smallest q.  Writes fval[b], fpos[b] (frows = 1).
constexpr int kFineLanesWaves = 1;   // one wave per workgroup: its LDS holds the block's index row
constexpr int kFineLanesMaxNv = 2048;
__global__ __launch_bounds__(64 * kFineLanesWaves) void k_fine_lanes(Items items, int n,
                                                                    const double* __restrict__ zero)
{
    __shared__ int ipref[kMaxBatchItems + 1];
    extern __shared__ int2 sidx[];   // [Nv + 4 * kPipe] the block's angle row
    if (threadIdx.x < 64) {   // inclusive scan of the items' counts (n <= 64)
        const int j = threadIdx.x;
        const int c = (j < n) ? *items[j].nsel : 0;
        int incl = c;
        for (int off = 1; off < 64; off <<= 1) {
            const int t = __shfl_up(incl, off, 64);
            if (j >= off) incl += t;
        }
        if (j < n) ipref[j + 1] = incl;
        if (j == 0) ipref[0] = 0;
    }
    __syncthreads();
    const int total = ipref[n];
    const int lane = threadIdx.x & 63;
    for (int g = blockIdx.x; g < total; g += gridDim.x) {   // workgroup-uniform
        int lo = 0, hi = n - 1;   // item of block g: last j with ipref[j] <= g
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (ipref[mid] <= g) lo = mid;
            else hi = mid - 1;
        }
        // the item and block are uniform: SGPRs, so the descriptor fields are
        // scalar loads
        const int j = __builtin_amdgcn_readfirstlane(lo);
        const MatchItem& it = items[j];
        const RtcsmPlan& pl = it.pl;
        const int b = __builtin_amdgcn_readfirstlane(g - ipref[j]);
        const int k = it.dlist[b];
        const int tt = k / pl.P, rem = k % pl.P;
        const int jx = rem / pl.ncy, jy = rem % pl.ncy;
        const int lr = pl.low_res, npose = lr * lr;
        const bool act = lane < npose;
        const int xo = lane / lr, yo = lane - (lane / lr) * lr;
        const int xf = -pl.win_x + jx * lr + xo, yf = -pl.win_y + jy * lr + yo;
        const int W = pl.W, H = pl.H, Nv = pl.Nv;
        const double* __restrict__ grid = it.grid;
        // the angle row of beam cells staged in LDS (8 loads in flight per
        // lane), then read back as broadcasts: the gathers of a batch then wait
        // on LDS, not on a global index load
        __syncthreads();
        stage_lds(sidx, it.idx + (size_t)tt * Nv, Nv);
        for (int v = Nv + lane; v < Nv + 4 * kPipe; v += 64) sidx[v] = make_int2(-(1 << 28), -(1 << 28));
        __syncthreads();
        // four batches of gathers in flight (seq_sum4): the kernel's duration
        // is one wave's latency chain over the beams
        const double s = seq_sum4<int2>(Nv, [&](int v) { return sidx[v]; }, [&](const int2& c) {
            const int x = c.x + xf, y = c.y + yf;
            const bool inb = act & ((unsigned)x < (unsigned)W) & ((unsigned)y < (unsigned)H);
            return inb ? grid + (unsigned)(y * W + x) : zero;
        });
        double bv = act ? s : -INFINITY;
        long long bo = act ? (long long)lane : LLONG_MAX;
        for (int off = 32; off > 0; off >>= 1) {
            const double ov = __shfl_xor(bv, off, 64);
            const long long ok = __shfl_xor(bo, off, 64);
            if (better(ov, ok, bv, bo)) {
                bv = ov;
                bo = ok;
            }
        }
        if (lane == 0) {
            it.fval[b] = bv;
            it.fpos[b] = (int)bo;
        }
    }
}

// k_fine_regs (LowRes 5, W even, 16-byte aligned grid, at most 8192 cells per
// side): k_fine_lanes with each beam's 5 x 5 window staged through LDS
// instead of one 25-lane gather per beam.  The gather made ~34 L1 tag
// accesses per instruction (its 25 addresses spread over 5 rows,
// profiles/raw/r03_v7_k1_pipeline_counters.csv) and was bound by that rate.
// Here 16 lanes per beam each load one aligned 16-byte segment -- row yo
// (0..4), segment s (0..2) of columns X0 .. X0 + 5, X0 = the window's first
// column rounded down to even, so a segment never straddles the map's x = 0
// or x = W edge (W is even); the 16th lane idles -- 4 beams per load
// instruction, two batches of kFrI instructions in flight in registers.  Each
// segment is written to LDS shifted by the window's column parity (a pose
// lane then reads column xo + 1 of its row whatever the window's start), and
// pose lane (xo, yo) adds the batch's beams in beam order (the reference's
// sequential fp64 sum).  Segments outside the map load the zero cells, what
// the per-beam gather reads there.  The beam index row is staged packed (x,
// y as int16).  Measured (config 2, 64 scans, one stream): 0.147 ms
// (k_fine_lanes) -> 0.084 ms with kFrI = 4 (2: 0.092, 6: 0.103, 8: 0.118);
// the same staging by global_load_lds (LDS DMA, a ring of 4-16 slots) ran
// 0.094-0.158 ms.
#ifndef LGS_FR_I
#define LGS_FR_I 4
#endif
constexpr int kFrI = LGS_FR_I;            // load instructions per batch (4 beams each)
constexpr int kFrRow = 13;                // doubles per staged row (bank-conflict-free reads of 5 x 5)
constexpr int kFrBeam = 5 * kFrRow;       // doubles per staged beam
constexpr int kFrPad = 4 * kFrI + 4;      // sentinel entries past the row (the last batch's tail)
__device__ __forceinline__ int2 unpack16(unsigned u)
{
    return make_int2((int)(short)(u & 0xFFFFu), (int)(short)(u >> 16));
}
__global__ __launch_bounds__(64) void k_fine_regs(Items items, int n, const double* __restrict__ zero, DevTs dts)
{
    const DtsScope dts_scope(dts);
    __shared__ int ipref[kMaxBatchItems + 1];
    __shared__ double stage[4 * kFrI * kFrBeam];
    extern __shared__ unsigned pidx[];   // [Nv + kFrPad] packed (x, y)
    {
        const int j = threadIdx.x;
        const int c = (j < n) ? *items[j].nsel : 0;
        int incl = c;
        for (int off = 1; off < 64; off <<= 1) {
            const int t = __shfl_up(incl, off, 64);
            if (j >= off) incl += t;
        }
        if (j < n) ipref[j + 1] = incl;
        if (j == 0) ipref[0] = 0;
    }
    __syncthreads();
    const int total = ipref[n];
    const int lane = threadIdx.x & 63;
    constexpr int LR = 5;
    const int lb = lane >> 4, ls = lane & 15;
    const int lrow = ls / 3, lseg = ls - 3 * (ls / 3);
    const bool act = lane < LR * LR;
    const int xo = lane / LR, yo = lane - (lane / LR) * LR;
    typedef double d2v __attribute__((ext_vector_type(2)));
#if LGS_XCD2
    // XCD-aware split of the list (as k_coarse_list_c): XCD x takes the x-th
    // eighth, items contiguous, so an item's map rows stay in one XCD's L2
    const int xcd = blockIdx.x & 7, per = gridDim.x >> 3;
    const int ge = (int)(((long long)total * (xcd + 1)) >> 3);
    for (int g = (int)(((long long)total * xcd) >> 3) + (int)(blockIdx.x >> 3); g < ge; g += per) {
#else
    for (int g = blockIdx.x; g < total; g += gridDim.x) {   // workgroup-uniform
#endif
        int lo = 0, hi = n - 1;
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (ipref[mid] <= g) lo = mid;
            else hi = mid - 1;
        }
        const int j = __builtin_amdgcn_readfirstlane(lo);
        const MatchItem& it = items[j];
        const RtcsmPlan& pl = it.pl;
        const int b = __builtin_amdgcn_readfirstlane(g - ipref[j]);
        const int k = it.dlist[b];
        const int tt = k / pl.P, rem = k % pl.P;
        const int jx = rem / pl.ncy, jy = rem % pl.ncy;
        const int xf0 = -pl.win_x + jx * LR, yf0 = -pl.win_y + jy * LR;
        const int W = pl.W, H = pl.H, Nv = pl.Nv;
        const double* __restrict__ grid = it.grid;
        const int2* __restrict__ src_idx = it.idx + (size_t)tt * Nv;
        __syncthreads();   // the previous block's row is read
        const bool lean = it.lean != 0;
        for (int v = lane; v < Nv + kFrPad; v += 64) {
            int2 c = v < Nv ? (lean ? lean_cell(it, tt, v) : src_idx[v]) : make_int2(-(1 << 28), -(1 << 28));
            c.x = min(max(c.x, -16384), 16383);   // far outside the map either way (W, H <= 8192)
            c.y = min(max(c.y, -16384), 16383);
            pidx[v] = (unsigned)(c.x & 0xFFFF) | ((unsigned)c.y << 16);
        }
        __syncthreads();
        const int nb = (Nv + 4 * kFrI - 1) / (4 * kFrI);   // batches
        auto load = [&](int bt, d2v (&r)[kFrI], int (&dx)[kFrI]) {
#pragma unroll
            for (int q = 0; q < kFrI; ++q) {
                const int2 c = unpack16(pidx[(bt * kFrI + q) * 4 + lb]);
                const int x = c.x + xf0;
                const int X = (x & ~1) + 2 * lseg, y = c.y + yf0 + lrow;
                dx[q] = x & 1;
                const bool in = ls < 15 && (unsigned)y < (unsigned)H && X >= 0 && X < W;
                typedef const __attribute__((address_space(1))) d2v gd2v_t;
                r[q] = *(gd2v_t*)(in ? grid + ((size_t)y * W + X) : zero);
            }
        };
        auto put = [&](const d2v (&r)[kFrI], const int (&dx)[kFrI]) {
            if (ls < 15) {
#pragma unroll
                for (int q = 0; q < kFrI; ++q) {
                    double* row = stage + (q * 4 + lb) * kFrBeam + lrow * kFrRow + 1 + 2 * lseg - dx[q];
                    row[0] = r[q].x;
                    row[1] = r[q].y;
                }
            }
        };
        d2v ra[kFrI], rb[kFrI];
        int da[kFrI], db[kFrI];
        load(0, ra, da);
        load(1, rb, db);
        double acc = 0.0;
        const int pose_off = yo * kFrRow + 1 + xo;
        auto consume = [&](d2v (&r)[kFrI], int (&dx)[kFrI], int next) {
            put(r, dx);   // LDS ops of a wave run in order: the reads below see these writes
            double v[4 * kFrI];
#pragma unroll
            for (int q = 0; q < 4 * kFrI; ++q) v[q] = stage[q * kFrBeam + pose_off];
            __builtin_amdgcn_s_waitcnt(waitcnt_imm(63, 0));
            __builtin_amdgcn_sched_barrier(0);
            if (next < nb) load(next, r, dx);   // refill (the last batch's tail: sentinel beams, zero cells)
            __builtin_amdgcn_sched_barrier(0);
            double s = acc;
#pragma unroll
            for (int q = 0; q < 4 * kFrI; ++q) s += v[q];   // beams past the row add +0.0: exact
            acc = s;
        };
        for (int bt = 0; bt < nb; bt += 2) {
            consume(ra, da, bt + 2);
            if (bt + 1 >= nb) break;
            consume(rb, db, bt + 3);
        }
        __builtin_amdgcn_s_waitcnt(0);
        double bv = act ? acc : -INFINITY;
        long long bo = act ? (long long)lane : LLONG_MAX;
        for (int off = 32; off > 0; off >>= 1) {
            const double ov = __shfl_xor(bv, off, 64);
            const long long ok = __shfl_xor(bo, off, 64);
            if (better(ov, ok, bv, bo)) {
                bv = ov;
                bo = ok;
            }
        }
        if (lane == 0) {
            it.fval[b] = bv;
            it.fpos[b] = (int)bo;
        }
    }
}

// k_replay (one wave): the reference's sequential acceptance (:98-114 with the
// strict update of :246) over the selected blocks in block order.  Lanes load
// 64 consecutive entries at once; the acceptance itself walks them in lane
// order with wave-uniform shuffles.  Then the 7 cost poses.
__global__ __launch_bounds__(64) void k_replay(Items items, DevTs dts)
{
    const DtsScope dts_scope(dts);
    const MatchItem& it = items[blockIdx.x];
    const RtcsmPlan& pl = it.pl;
    const double* __restrict__ cscore = it.cscore;
    const uint8_t* __restrict__ cflag = it.cflag;
    const int* __restrict__ list = it.list;
    const int* __restrict__ segcnt = it.segcnt;
    const int nseg = it.nseg;
    const double* __restrict__ fval = it.fval;
    const int* __restrict__ fpos = it.fpos;
    const int frows = it.frows;
    const double* __restrict__ Lp = it.Lp;
    RtcsmRecord* rec = it.rec;
    double* __restrict__ poses7 = it.poses7;
    extern __shared__ int pref[];   // nseg + 1
    __shared__ int ws[16];
    seg_prefix(segcnt, nseg, pref, ws);
    const int n = pref[nseg];
    const double L = *Lp;
    const int lane = threadIdx.x;
    double s = pl.thr;
    long long bestk = -1;
    int bestpos = 0;
    bool dangerous = false;
    for (int b0 = 0; b0 < n; b0 += 64) {
        const int b = b0 + lane;
        double c = -INFINITY, f = -INFINITY;
        long long k = -1;
        int pos = 0;
        if (b < n) {
            const int sg = seg_of(pref, nseg, b);
            k = list[(size_t)sg * kSelSeg + (b - pref[sg])];
            c = cscore[k];
            // k_fine's frows row results of the block: max, ties to the
            // smallest order index (the reference's x-outer, y-inner walk)
            const size_t fi = (size_t)b * frows;
            f = fval[fi];
            pos = fpos[fi];
            for (int r = 1; r < frows; ++r) {
                const double fr = fval[fi + r];
                const int pr = fpos[fi + r];
                if (fr > f || (fr == f && pr < pos)) {
                    f = fr;
                    pos = pr;
                }
            }
            if (cflag[k] && c < L && f >= L) dangerous = true;
        }
        // the sequential rule in as many steps as it accepts blocks: the
        // first lane (from `from` on) whose block passes under the current s
        // is the next one the walk would accept; the lanes before it fail
        // under this s and are passed over exactly as the walk does
        const int cnt = min(64, n - b0);
        for (int from = 0;;) {   // wave-uniform
            const bool cand = lane >= from && lane < cnt && c > s && f > s;
            const unsigned long long m = __ballot(cand);
            if (m == 0ull) break;
            const int j = __ffsll((long long)m) - 1;
            s = __shfl(f, j, 64);
            bestk = __shfl(k, j, 64);
            bestpos = __shfl(pos, j, 64);
            from = j + 1;
        }
    }
    dangerous = __ballot(dangerous) != 0ull;
    if (lane != 0) return;
    int bx = -pl.win_x, by = -pl.win_y, bt = -pl.win_t;
    if (bestk >= 0) {
        const int tt = (int)(bestk / pl.P);
        const int rem = (int)(bestk % pl.P);
        const int jx = rem / pl.ncy, jy = rem % pl.ncy;
        bx = -pl.win_x + jx * pl.low_res + bestpos / pl.low_res;
        by = -pl.win_y + jy * pl.low_res + bestpos % pl.low_res;
        bt = tt - pl.win_t;
    }
    rec->status = dangerous ? REC_DANGEROUS : 0;
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
// greedy-endpoint cost, one workgroup per pose: every thread computes the
// cells and the exp() term of its beams into LDS, then lane 0 performs the
// reference's `costValue -= exp(..)` in beam order (filtered beams add an
// exact -0.0 no-op), and `costValue *= scale`.
// --------------------------------------------------------------------------
constexpr int kCostThreads = 1024;
constexpr int kCostLdsTerms = 8192;
// dynamic LDS of a k_cost launch: the terms of its largest item (r06: a
// static 64 KB array held two workgroups per CU and made the 7 x n
// workgroups wait for whole CUs under other streams' work)
template <class V>
inline size_t cost_lds(const V& items)
{
    int n = 1;
    for (const auto& it : items) n = std::max(n, it.cp.N);
    return sizeof(double) * (size_t)std::min(n, kCostLdsTerms);
}

__device__ __forceinline__ double gval(const CostPlan& cp, const double* __restrict__ g, int x,
                                       int y)
{
    const bool inb = ((unsigned)x < (unsigned)cp.W) & ((unsigned)y < (unsigned)cp.H);
    const size_t off = inb ? (size_t)y * cp.W + x : 0;
    const double v = gload(g + off);
    return inb ? v : 0.0;
}

// The kernel-window search of CostGreedyEndpoint::Cost (:69-99) for one beam:
// min squared distance to a cell with hit >= occThr and miss <= occThr (both
// known).  KS > 0: compile-time kernel size, every cell value loaded before
// any test (the loads of a beam are independent); KS == 0: runtime size.
template <int KS>
__device__ __forceinline__ double min_sq_dist(const CostPlan& cp, const double* __restrict__ grid, int4 c,
                                              double minSq0)
{
    double minSq = minSq0;
    if constexpr (KS > 0) {
        constexpr int D = 2 * KS + 1;
        double hv[D * D], mv[D * D];
#pragma unroll
        for (int q = 0; q < D * D; ++q) {
            hv[q] = gval(cp, grid, c.x + q % D - KS, c.y + q / D - KS);
            mv[q] = gval(cp, grid, c.z + q % D - KS, c.w + q / D - KS);
        }
#pragma unroll
        for (int q = 0; q < D * D; ++q) {
            const int kx = q % D - KS, ky = q / D - KS;
            if (hv[q] == 0.0 || mv[q] == 0.0) continue;
            if (hv[q] < cp.occupancy_threshold || mv[q] > cp.occupancy_threshold) continue;
            const double dX = kx * cp.res;
            const double dY = ky * cp.res;
            const double sq = dX * dX + dY * dY;
            minSq = (minSq < sq) ? minSq : sq;
        }
    } else {
        const int K = cp.kernel_size;
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
    }
    return minSq;
}

// mode 0: compute cells (+ guard records) and store them in cidx;
// mode 1: read cells from cidx (after host patches).
template <int KS>
__global__ __launch_bounds__(kCostThreads) void k_cost(Items items, int guard_cap, double guard_eps, int inject,
                                                       int mode, DevTs dts)
{
    const DtsScope dts_scope(dts);
    const MatchItem& it = items[blockIdx.y];
    const CostPlan& cp = it.cp;
    const double* __restrict__ grid = it.grid;
    const double* __restrict__ ranges = it.ranges;
    const double* __restrict__ angles = it.angles;
    const double* __restrict__ poses = it.poses7;
    int4* __restrict__ cidx = it.cidx;
    double* __restrict__ gterms = it.terms;
    RtcsmRecord* rec = it.rec;
    const int gen = it.gen;
    extern __shared__ double lterms[];   // [min(max N of the launch, kCostLdsTerms)] (cost_lds)
    const int pi = blockIdx.x;
    const bool in_lds = cp.N <= kCostLdsTerms;
    double* __restrict__ tm = in_lds ? lterms : gterms + (size_t)pi * cp.N;
    const double px = poses[3 * pi], py = poses[3 * pi + 1], pt = poses[3 * pi + 2];
    const double lim = (cp.kernel_size + 1) * cp.res;
    const double minSq0 = lim * lim + lim * lim;
    // the cells of beam i (mode 0: computed + guard records; mode 1: read);
    // every active lane calls it (the guard slots are taken per wave)
    auto cells_of = [&](int i, bool have) -> int4 {
        if (mode != 0) return have ? cidx[(size_t)pi * cp.N + i] : make_int4(INT_MIN, 0, 0, 0);
        const double r = have ? ranges[i] : 0.0;
        const bool valid = have && !(r >= cp.max_range || r <= cp.min_range);
        double q[4] = { 0.0, 0.0, 0.0, 0.0 };
        if (valid) {
            const double cs = cos(pt + angles[i]);
            const double sn = sin(pt + angles[i]);
            q[0] = (px + r * cs - cp.min_x) / cp.res;
            q[1] = (py + r * sn - cp.min_y) / cp.res;
            q[2] = (px + (r - cp.hit_and_missed_dist) * cs - cp.min_x) / cp.res;
            q[3] = (py + (r - cp.hit_and_missed_dist) * sn - cp.min_y) / cp.res;
        }
        int cell[4];
        for (int j = 0; j < 4; ++j) {
            cell[j] = (int)floor(q[j]);
            const bool guarded = valid && near_boundary(q[j], guard_eps);
            const int slot = tagged_slot_wave(&rec->cost_guard_word, (unsigned)gen, guarded);
            if (guarded) {
                cell[j] += inject;
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
        const int4 c = valid ? make_int4(cell[0], cell[1], cell[2], cell[3]) : make_int4(INT_MIN, 0, 0, 0);
        if (have) cidx[(size_t)pi * cp.N + i] = c;
        return c;
    };
    // two beams per thread and pass (i, i + blockDim): a 1081-beam scan is one
    // latency chain per thread instead of a second pass for its last 57 beams
    for (int i0 = threadIdx.x; i0 < cp.N; i0 += 2 * blockDim.x) {
        const int i1 = i0 + (int)blockDim.x;
        const bool h1 = i1 < cp.N;
        const int4 c0 = cells_of(i0, true);
        const int4 c1 = cells_of(i1, h1);
        const double t0 = (c0.x != INT_MIN) ? exp(-0.5 * min_sq_dist<KS>(cp, grid, c0, minSq0) / cp.variance) : 0.0;
        const double t1 = (c1.x != INT_MIN) ? exp(-0.5 * min_sq_dist<KS>(cp, grid, c1, minSq0) / cp.variance) : 0.0;
        tm[i0] = t0;
        if (h1) tm[i1] = t1;
    }
    __syncthreads();
    // costValue -= exp(..) (C/mapping/cost_function_greedy_endpoint.cpp): the
    // cost feeds the normalized cost and the covariance, both held to 1e-5
    // (north_star), so the terms are summed as a tree (the reference's
    // beam-order chain differs in the last bits only)
    __shared__ double wsum[kCostThreads / 64];
    double part = 0.0;
    for (int i = threadIdx.x; i < cp.N; i += blockDim.x) part += tm[i];
    for (int off = 32; off > 0; off >>= 1) part += __shfl_xor(part, off, 64);
    if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = part;
    __syncthreads();
    if (threadIdx.x == 0) {
        double tot = 0.0;
        for (int j = 0; j < (int)(blockDim.x >> 6); ++j) tot += wsum[j];
        rec->costs[pi] = (0.0 - tot) * cp.scaling_factor;
    }
}

// kernel size 1 (the launcher JSON's) gets the unrolled instantiation
#define KCOST(ks) ((ks) == 1 ? k_cost<1> : k_cost<0>)

// --------------------------------------------------------------------------
// Small windows: the whole search of a window whose coarse
// lattice holds ONE block per angle (2 winX < lr and 2 winY < lr: the launcher
// JSON frontend window, +-0.1 m at 5 cm with LowRes 5) in one launch, one
// workgroup of LR waves per (angle, item):
//  1. ComputeScanIndices of the angle (:179-200) with k_project's arithmetic
//     and boundary guard, into LDS (and the item's index rows, which the
//     host's guard fix-ups patch; mode 1 reruns read those rows back);
//  2. the block's LR x LR fine scores and its coarse score in ONE pass over
//     the beams: wave w gathers fine row yo = w of 64 beams at a time (LR
//     cells each), lanes 0..LR-1 of every wave add their (xo, yo) row in beam
//     order.  The precomputed map's value at a beam's lattice start
//     (PrecomputeGridMap, C/mapping/grid_map_builder.cpp:518-536) is the max
//     of exactly those LR x LR cells when the window lies in the map (edge
//     beams: SlidingWindowMax's clamped last window, H/util.hpp:247-250, or 0
//     outside the map); wave 0 takes it from the waves' row maxima after a
//     workgroup barrier and its lane LR adds it in beam order.  No coarse map
//     is built;
//  3. the item's last workgroup to finish (a wrap-around device-scope
//     counter) walks the angles in the reference's order (:88-112) over the
//     published (coarse, fine max, first argmax) triples: a block is refined
//     when !(coarse <= scoreMax), accepted when its fine max > scoreMax; the
//     record, the refined-block count and the 7 cost poses are written there.
// Every score is the reference's sequential beam-order fp64 sum (bit-exact);
// nothing is pruned, so no rounding bound is involved.
// --------------------------------------------------------------------------
constexpr int kSmallMaxNv = 64 * kMaxChunks;   // fully unrolled chunk loop
constexpr int kSmallDepth = 4;                 // chunks of gathers in flight per wave

// Precomputed-map value at (bx, by) read directly from the fine map: 0 (the
// unknown value) outside the map, else the max of the window SlidingWindowMax
// assigns to that cell (its start clamped to the last full window, zero
// padding when the map is narrower than the window).
__device__ __forceinline__ double small_cval(const double* __restrict__ grid, int bx, int by, int W, int H, int lr)
{
    if (bx < 0 || by < 0 || bx >= W || by >= H) return 0.0;
    const int sx = min(bx, max(W - lr, 0)), sy = min(by, max(H - lr, 0));
    const int ex = min(sx + lr, W), ey = min(sy + lr, H);
    double m = (W < lr || H < lr) ? 0.0 : -INFINITY;
    for (int y = sy; y < ey; ++y)
        for (int x = sx; x < ex; ++x) m = fmax(m, gload(grid + (size_t)y * W + x));
    return m;
}

constexpr int kSmallRing = 3;   // chunk buffers between the row waves and the adder wave
template <int LR>
constexpr size_t small_buf_doubles()
{
    // the ring of chunk buffers (LR * LR pose rows of 65 doubles), then the
    // coarse column [kSmallMaxNv], then the ready counters and the consumed count
    return (size_t)kSmallRing * LR * LR * 65 + (size_t)kSmallMaxNv + kMaxChunks / 2 + 1;
}

// Workgroup of LR + 1 waves: row wave w < LR gathers fine row yo = w of 64
// beams at a time and writes its cells of every pose (xo, w) into the chunk's
// ring buffer and its row maxima into the coarse column (ds_max_f64); the
// adder wave's lane k adds pose k's row, lane LR * LR the coarse column, each
// in beam order.  No workgroup barrier inside the chunk loop: the row waves
// bump the chunk's ready counter after their LDS writes (a wave's LDS
// operations execute in order), the adder posts the chunks it is done with.
// One adder wave for every chain: r04's first layout (each row wave adding
// its own LR poses, a seventh wave the coarse column) ran the chains on waves
// that shared SIMDs with the gather work (16 us of chunk loop + 5 us waiting
// for the slowest wave per config-4 angle).  LowRes <= 7 (LR * LR + 1 <= 64 lanes).
template <int LR>
// mode 0: project; 2: project, then the host's guard patches (t, v, ix, iy);
// 1: read the index rows the host uploaded (a full host projection).  The
// projected rows are not written back: dirty lines would make the device-scope
// release before the angle count write back that much more L2.
__global__ __launch_bounds__(64 * (LR + 1)) void k_match_small(Items items, int mode, int guard_cap,
                                                               double guard_eps, int inject,
                                                               const double* __restrict__ zero,
                                                               const int4* __restrict__ patches, int npatch, DevTs dts)
{
    const DtsScope dts_scope(dts);
    constexpr int NT = 64 * (LR + 1), LD = 65;
    const MatchItem& it = items[blockIdx.y];
    const RtcsmPlan& pl = it.pl;
    const int tt = blockIdx.x;
    if (tt >= pl.T) return;   // past this item's angles (uniform)
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int Nv = pl.Nv, W = pl.W, H = pl.H;
    const double* __restrict__ grid = it.grid;
    RtcsmRecord* rec = it.rec;
    const int gen = it.gen;
    extern __shared__ char smem[];
    int2* sidx = (int2*)smem;   // [Nv]
    double* bufs = (double*)(smem + sizeof(int2) * (size_t)((Nv + 1) & ~1));   // [kSmallRing][LR * LR rows][LD]
    double* cmax = bufs + (size_t)kSmallRing * LR * LR * LD;   // [Nv] coarse values (interior beams: max of the rows)
    int* ready = (int*)(cmax + kSmallMaxNv);             // [kMaxChunks] row waves done with the chunk
    int* consumed = ready + kMaxChunks;                  // chunks the adder wave is done with
    __shared__ int s_wsum[LR + 1];
    __shared__ double s_trig[2];
    __shared__ int s_last;
    LGS_PROBE_DECL;
    LGS_PROBE_MARK();

    // 1. the angle's scan indices
    if (mode != 1) {
        const double* __restrict__ ranges = it.ranges;
        const double* __restrict__ angles = it.angles;
        int* smap = (int*)bufs;   // valid beam v -> beam index (the value buffers are not in use yet)
        if (tid == 0) {
            // currentSensorPose.mTheta = sensorPose.mTheta + stepTheta * t (:90-91)
            const double th = pl.st + pl.step_t * (double)(tt - pl.win_t);
            double sn, cs;
            sincos(th, &sn, &cs);
            s_trig[0] = cs;
            s_trig[1] = sn;
        }
        const int chunk = (pl.N + NT - 1) / NT;
        const int lo = min(tid * chunk, pl.N), hi = min(lo + chunk, pl.N);
        int nvalid = 0;
        for (int i = lo; i < hi; ++i) nvalid += !(ranges[i] >= pl.rmax);
        int incl = nvalid;
        for (int off = 1; off < 64; off <<= 1) {
            const int t = __shfl_up(incl, off, 64);
            if (lane >= off) incl += t;
        }
        if (lane == 63) s_wsum[wave] = incl;
        __syncthreads();
        int pos = incl - nvalid;
        for (int j = 0; j < wave; ++j) pos += s_wsum[j];
        for (int i = lo; i < hi; ++i)
            if (!(ranges[i] >= pl.rmax)) smap[pos++] = i;
        __syncthreads();
        const double ct = s_trig[0], st = s_trig[1];
        const double inv_res = 1.0 / pl.res;
        for (int v0 = 0; v0 < Nv; v0 += NT) {   // uniform trip count: tagged_slot_wave needs every lane
            const int v = v0 + tid;
            const bool act = v < Nv;
            int ix = 0, iy = 0;
            bool guarded = false;
            if (act) {
                // the arithmetic of k_project (HitPoint by rotation, x * (1 / res))
                const int i = smap[v];
                const double r = ranges[i];
                double sa, ca;
                sincos(angles[i], &sa, &ca);
                const double c = ct * ca - st * sa;
                const double s = st * ca + ct * sa;
                const double hx = pl.sx + r * c;
                const double hy = pl.sy + r * s;
                const double qx = (hx - pl.min_x) * inv_res;
                const double qy = (hy - pl.min_y) * inv_res;
                ix = (int)floor(qx);
                iy = (int)floor(qy);
                guarded = near_boundary(qx, guard_eps) || near_boundary(qy, guard_eps);
            }
            const int slot = tagged_slot_wave(&rec->guard_word, (unsigned)gen, guarded);
            if (guarded) {
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
            if (act) sidx[v] = make_int2(ix, iy);
        }
        __syncthreads();   // the beam map is dead from here on
        if (mode == 2) {
            for (int k = tid; k < npatch; k += NT) {
                const int4 pq = patches[k];
                if (pq.x == tt) sidx[pq.y] = make_int2(pq.z, pq.w);
            }
            __syncthreads();
        }
    } else {
        stage_lds(sidx, it.idx + (size_t)tt * Nv, Nv);
        __syncthreads();
    }
    LGS_PROBE_MARK();

    // 2. fine rows + coarse values, beam order
    const int nchunk = (Nv + 63) / 64;
    const int xc = -pl.win_x, yr = -pl.win_y + wave;
    const bool fine = wave < LR;
    // Every fine lane loads a row run of LR cells with 16-byte loads from the
    // run's start clamped into the map (W >= LR: always a valid address); a
    // run that leaves the map then holds every in-map cell the lane needs, at
    // index k = x - xs, and the cells outside are 0 -- selected in registers.
    // No load sits under a run-time branch inside the loop: the compiler
    // keeps kSmallDepth chunks of gathers in flight (a branch drained them).
    double r[kSmallDepth][LR];
    int sh[kSmallDepth];   // x0 - xs, or LR (every cell masked: no beam, or a row outside the map)
    bool inr[kSmallDepth]; // an interior beam of the chunk (its coarse value is the max of its rows)
    auto gather = [&](int c, double (&x)[LR], int& shift, bool& interior) {
        const int b = c * 64 + lane;
        const int2 ij = sidx[max(min(b, Nv - 1), 0)];
        const int x0 = ij.x + xc, y = ij.y + yr;
        const int xs = min(max(x0, 0), W - LR);
        typedef const __attribute__((address_space(1))) d2a8 gd2a8_t;
        const double* p = grid + (unsigned)(min(max(y, 0), H - 1) * W + xs);
#pragma unroll
        for (int q = 0; q + 1 < LR; q += 2) {
            const d2a8 a = *(gd2a8_t*)(p + q);
            x[q] = a.x;
            x[q + 1] = a.y;
        }
        if constexpr (LR & 1) x[LR - 1] = gload(p + LR - 1);
        shift = ((b < Nv) & ((unsigned)y < (unsigned)H)) ? x0 - xs : LR;
        const int by = y - wave;   // the beam's lattice start (x0, by)
        interior = (b < Nv) & (x0 >= 0) & (by >= 0) & (x0 <= W - LR) & (by <= H - LR);
#ifdef LGS_SMALL_NOGATHER   // diagnostics (timing only): no loads
        for (int q = 0; q < LR; ++q) x[q] = (double)(x0 + q);
#endif
    };
    // one adder lane's beam-order sum of a chunk row: the 64 values loaded
    // first, then the dependent chain
    auto add_row = [&](const double* row, int cnt, double& acc) {
        double s = acc;
        if (cnt == 64) {
            double v[64];
#pragma unroll
            for (int b = 0; b < 64; ++b) v[b] = row[b];
#pragma unroll
            for (int b = 0; b < 64; ++b) s += v[b];
        } else {
            for (int b = 0; b < cnt; ++b) s += row[b];
        }
        acc = s;
    };
    if (fine) {
        static_for_step<0, kSmallDepth, 1>([&](auto dd) {
            constexpr int d = decltype(dd)::value;
            gather(d, r[d], sh[d], inr[d]);
            __builtin_amdgcn_sched_barrier(0);
            return true;
        });
    }
    // the coarse column: the edge beams' values (lattice start outside
    // [0, W - LR] x [0, H - LR]) ahead of the chunk loop, which then holds no
    // load under a branch; -inf for the interior beams, whose value the row
    // waves' maxima build (ds_max_f64)
    for (int v = tid; v < Nv; v += NT) {
        const int2 ij = sidx[v];
        const int bx = ij.x - pl.win_x, by = ij.y - pl.win_y;
        const bool interior = (bx >= 0) & (by >= 0) & (bx <= W - LR) & (by <= H - LR);
        cmax[v] = interior ? -INFINITY : small_cval(grid, bx, by, W, H, LR);
    }
    for (int c = tid; c < kMaxChunks; c += NT) ready[c] = 0;
    if (tid == 0) *consumed = 0;
    __syncthreads();
    LGS_PROBE_MARK();
    constexpr int ROWS = LR * LR;   // pose rows of a chunk buffer, row = order index xo * LR + yo
    if (fine) {
        // a row wave: its cells of every pose (xo = 0..LR-1, yo = wave) into
        // the chunk's ring buffer, its row maxima into the coarse column
        static_for_step<0, kMaxChunks, 1>([&](auto cc) {
            constexpr int c = decltype(cc)::value;
            if (c >= nchunk) return false;
            if constexpr (c >= kSmallRing) {   // the adder is done with the buffer's previous chunk
                while (__hip_atomic_load(consumed, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) <
                       c - kSmallRing + 1) {
                }
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
            }
            double* cur = bufs + (size_t)(c % kSmallRing) * ROWS * LD;
            {
                constexpr int d = c % kSmallDepth;
                const int k0 = sh[d];
                double m = -INFINITY;
#pragma unroll
                for (int q = 0; q < LR; ++q) {
                    const int k = k0 + q;   // cell x0 + q in the run (in the map iff 0 <= k < LR)
                    double v = 0.0;
#pragma unroll
                    for (int j = 0; j < LR; ++j) v = (k == j) ? r[d][j] : v;
                    cur[(q * LR + wave) * LD + lane] = v;
                    m = fmax(m, v);
                }
                if (inr[d]) __hip_atomic_fetch_max(cmax + c * 64 + lane, m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (c + kSmallDepth < kMaxChunks)
                gather(c + kSmallDepth, r[c % kSmallDepth], sh[c % kSmallDepth], inr[c % kSmallDepth]);
            __builtin_amdgcn_sched_barrier(0);
            // after this wave's rows and maxima of the chunk: the release
            // fence orders them before the counter (lgkmcnt(0), not left to
            // the compiler's scheduling or the LDS unit's in-order issue)
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
            if (lane == 0) __hip_atomic_fetch_add(ready + c, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            return true;
        });
        return;
    }
    // the adder wave: lane k < ROWS adds pose k's row, lane ROWS the coarse
    // column, each in beam order, chunk by chunk as the row waves post them
    double acc = 0.0;
    for (int c = 0; c < nchunk; ++c) {
        while (__hip_atomic_load(ready + c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < LR) {
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
        const double* row = lane < ROWS ? bufs + (size_t)(c % kSmallRing) * ROWS * LD + lane * LD : cmax + c * 64;
#ifdef LGS_SMALL_NOSUM   // diagnostics (timing only): no sequential sums
        if (lane <= ROWS && c == 0) add_row(row, min(64, Nv - c * 64), acc);
#else
        if (lane <= ROWS) add_row(row, min(64, Nv - c * 64), acc);
#endif
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");   // the chunk's reads are done
        if (lane == 0) __hip_atomic_store(consumed, c + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    LGS_PROBE_MARK();
    LGS_PROBE_MARK();
    const double cval = __shfl(acc, ROWS, 64);
    double fv = lane < ROWS ? acc : -INFINITY;
    long long fk = lane < LR * LR ? lane : LLONG_MAX;
    for (int off = 32; off > 0; off >>= 1) {
        const double ov = __shfl_xor(fv, off, 64);
        const long long ok = __shfl_xor(fk, off, 64);
        if (better(ov, ok, fv, fk)) {
            fv = ov;
            fk = ok;
        }
    }
    typedef __attribute__((address_space(1))) double gdbl_t;
    typedef __attribute__((address_space(1))) int gint_t;
    LGS_PROBE_MARK();
    if (lane == 0) {
        ((gdbl_t*)it.cscore)[tt] = cval;
        ((gdbl_t*)it.fval)[tt] = fv;
        ((gint_t*)it.fpos)[tt] = (int)fk;
        __threadfence();   // release (device scope): the triple before the count
        const unsigned old = atomicInc((unsigned*)it.keepc, (unsigned)(pl.T - 1));   // wraps to 0 after T
        s_last = old == (unsigned)(pl.T - 1);
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
    LGS_PROBE_MARK();
    LGS_PROBE_PRINT("match_small(b0: project, edge pass, chunks, sync, argmax, publish)");
    if (!s_last) return;
    __threadfence();   // acquire: every angle's triple

    // 3. the reference's walk over the angles
    const double* cs = it.cscore;
    const double* fvs = it.fval;
    const int* fps = it.fpos;
    const int T = pl.T;
    double s = pl.thr;
    int bt = -1, bpos = 0;
    long long neval = 0;
    for (int b0 = 0; b0 < T; b0 += 64) {
        const int t = b0 + lane;
        const bool in = t < T;
        const double c = in ? __builtin_nontemporal_load(cs + t) : 0.0;
        const double f = in ? __builtin_nontemporal_load(fvs + t) : 0.0;
        const int p = in ? __builtin_nontemporal_load(fps + t) : 0;
        for (int from = 0;;) {   // wave-uniform
            const unsigned long long am = __ballot(in && lane >= from && !(c <= s) && f > s);
            const int j = am ? __ffsll((long long)am) - 1 : 64;
            // blocks from..j (j when accepted) are refined if !(score <= scoreMax) (:103-104)
            neval += __popcll(__ballot(in && lane >= from && lane <= j && !(c <= s)));
            if (!am) break;
            s = __shfl(f, j, 64);
            bt = b0 + j;
            bpos = __shfl(p, j, 64);
            from = j + 1;
        }
    }
    if (lane != 0) return;
    int bx = -pl.win_x, by = -pl.win_y, bth = -pl.win_t;
    if (bt >= 0) {
        bx = -pl.win_x + bpos / LR;
        by = -pl.win_y + bpos % LR;
        bth = bt - pl.win_t;
    }
    rec->status = 0;
    rec->found = s > pl.thr;
    rec->n_eval = neval;
    rec->best[0] = bx;
    rec->best[1] = by;
    rec->best[2] = bth;
    rec->score_max = s;
    rec->L = -INFINITY;
    rec->coarse_evals = (unsigned long long)pl.K;
    // bestSensorPose (:122-125) and the central-difference poses (as k_replay)
    const double x = pl.sx + bx * pl.step_x;
    const double y = pl.sy + by * pl.step_y;
    const double th = pl.st + bth * pl.step_t;
    const double dl = pl.res, da = 1e-2;
    const double P7[7][3] = {
        { x, y, th },
        { x + dl, y + 0.0, th + 0.0 }, { x - dl, y - 0.0, th - 0.0 },
        { x + 0.0, y + dl, th + 0.0 }, { x - 0.0, y - dl, th - 0.0 },
        { x + 0.0, y + 0.0, th + da }, { x - 0.0, y - 0.0, th - da },
    };
    for (int i = 0; i < 7; ++i)
        for (int j = 0; j < 3; ++j) ((gdbl_t*)it.poses7)[3 * i + j] = P7[i][j];
}

// --------------------------------------------------------------------------
// k_post (LGS_OPT_POST_RECORDS): the batch's records straight into the pinned
// (coherent) host copy, then the completion flag.  Every thread's loads are
// issued before its stores (r05: one wave copying 16-byte words in a loop
// waited a device round trip per word -- ~60 us for a 64-record chunk, 7% of
// a config-5 batch); each thread's system-scope release orders its record
// stores, the barrier puts all of them before the flag store.
// --------------------------------------------------------------------------
constexpr int kPostThreads = 256;
// A second segment (n2 words, LGS_OPT_DEVICE_TIMING: the chunk's timing
// words) is copied the same way.
__device__ __forceinline__ void post_copy(const uint4* __restrict__ src, uint4* __restrict__ dst, int n16)
{
    const int nt = blockDim.x;
    for (int i0 = threadIdx.x; i0 < n16; i0 += 4 * nt) {
        uint4 x[4];
#pragma unroll
        for (int j = 0; j < 4; ++j)
            if (i0 + j * nt < n16) x[j] = src[i0 + j * nt];
#pragma unroll
        for (int j = 0; j < 4; ++j)
            if (i0 + j * nt < n16) dst[i0 + j * nt] = x[j];
    }
}
__global__ __launch_bounds__(kPostThreads) void k_post(const uint4* __restrict__ src, uint4* __restrict__ dst, int n16,
                                                       unsigned* flag, unsigned gen, const uint4* __restrict__ src2,
                                                       uint4* __restrict__ dst2, int n2)
{
    post_copy(src, dst, n16);
    if (n2) post_copy(src2, dst2, n2);
    __threadfence_system();
    __syncthreads();
    if (threadIdx.x == 0) *(volatile unsigned*)flag = gen;
}

// --------------------------------------------------------------------------
// dense diagnostics: every fine score of the window (one lane per pose)
// --------------------------------------------------------------------------
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
void set_plane_layout(RtcsmPlan& pl)
{
    pl.Wq = (pl.W + pl.low_res - 1) / pl.low_res;
    pl.Hq = (pl.H + pl.low_res - 1) / pl.low_res;
    // margins also cover the superblock reads (kSB * nsb coarse blocks per axis)
    pl.nsbx = (pl.ncx + kSB - 1) / kSB;
    pl.nsby = (pl.ncy + kSB - 1) / kSB;
    pl.M = std::max(kSB * pl.nsbx, kSB * pl.nsby);
    // a multiple of 4: 16-byte aligned fp64 plane rows (k_precompute_planes'
    // paired stores), 8-byte aligned fp16 rows (k_super_hv's 4-column loads)
    pl.Wqp = (pl.Wq + 2 * pl.M + 3) & ~3;
    pl.Hqp = pl.Hq + 2 * pl.M;
    pl.pstride = (long long)pl.Wqp * pl.Hqp;
    pl.Wq4 = (((pl.Wqp + 3) / 4) + 7) & ~7;   // 16-byte aligned fp16 sub-phase rows (k_super_planes' stores)
    pl.Hq4 = (pl.Hqp + 3) / 4;
    pl.sub4 = (long long)pl.Wq4 * pl.Hq4;
    pl.pstride4 = 16 * pl.sub4;
    LGS_REQUIRE((long long)pl.low_res * pl.low_res * pl.pstride4 < (1LL << 31),
                "coarse map too large for 32-bit plane offsets");
    // octet layout (8-bit units, r06): unit (q, X) holds sub-phase rows 4q ..
    // 4q + 4 unit8 - 1 of column X, one byte each: 8 rows (unit8 = 2) hold
    // the 5 superblock rows of a window with nsby <= 5 at any of the 4 row
    // offsets, 12 rows (unit8 = 3) the 9 rows of nsby <= 9
    pl.oct = pl.nsbx <= 9 && pl.nsby <= 9 && pl.nsbx * pl.nsby <= 64;
    pl.unit8 = (pl.oct && pl.nsby > 5) ? 3 : 2;
    pl.Qo = (pl.Hq4 + 3) / 4 + 1;
    pl.subO = (long long)pl.Qo * pl.Wq4;
    pl.pstrideO = 16 * pl.subO;
    LGS_REQUIRE(!pl.oct || (long long)pl.low_res * pl.low_res * pl.pstrideO < (1LL << 29),
                "coarse map too large for 32-bit superblock unit offsets");
}

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
    pl.rmax = p->scan_range_max;
    set_plane_layout(pl);
    pl.sb_mult = 1.0 + 4.0 * (double)(nv + 1) * 0x1p-53;
    pl.sb_off = (long long)pl.T * std::max(nv, 1) + kPad;   // == ensure_workspace's nidx
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

// k_fine's items per block: LR rows on the transposed path (LowRes 5), 1 otherwise
inline bool lr5_path(int nv_max, int low_res) { return nv_max <= 64 * kMaxChunks && low_res == 5; }

inline size_t sidx_bytes(int nv) { return sizeof(int2) * (size_t)(nv + 2 * kPipe); }

inline int coarse_block(const RtcsmPlan& pl) { return std::min(1024, ((pl.P + 63) / 64) * 64); }

inline size_t align256(size_t b) { return (b + 255) & ~(size_t)255; }

// Shape of one batched launch sequence: every item shares the search
// parameters; T and Nv (and K = T * P) differ per scan, so the launch grids
// and dynamic LDS use the maxima.
struct BatchShape {
    int n = 0;
    int Tmax = 0, NvMax = 0, nsegMax = 0, nparts_max = 0;
    int P = 0, nsb2 = 0, chunks = 0, low_res = 0, cb = 0;
    bool pair = false;
    bool oct = false;       // k_super_oct (octet layout of the plan, nsbx, nsby <= 9; chunks == 1)
    int unit8 = 2;          // its unit size in 8-byte words (3: 24-byte units for 6-9 rows)
    int nsby = 0;
    bool pruned = false;    // superblock pruning
    bool small = false;     // k_match_small: one coarse block per angle, no coarse map (§4.1c)
    bool lr5 = false;       // transposed LR = 5 evaluators
    bool fine_lanes = false;   // k_compact + k_fine_lanes (lr * lr <= 64)
    bool fine_staged = false;  // ... as k_fine_regs (LowRes 5, every map W even, <= 8192, 16-byte aligned)
    int frows = 1;
    int kernel_size = 0;
    WorkList wl{};          // kept-superblock work list (wl.cnt null: k_coarse_rows)
};

// per-(chunk|tile, angle) best entries the seed kernel scans: k_super's
// chunks (pruned) or k_coarse's block tiles
inline int item_nparts(const BatchShape& B, const RtcsmPlan& pl, bool pruned)
{
    return pruned ? B.chunks * pl.T : ((B.P + B.cb - 1) / B.cb) * pl.T;
}

// superblock pruning applies (else k_coarse scores every block)
inline bool uses_super(const lgs_ctx* ctx, int nv_max, int nsb2, bool dense)
{
    // k_coarse_rows: one ballot over an angle's superblocks, Nv <= 2048
    return !(dense || ctx->force_dense) && ctx->super_prune && nv_max <= kSeedMaxNv &&
           nsb2 <= 64 && nsb2 >= ctx->prune_min_super;
}

// Per-item workspace: one contiguous region per item carved from S_BATCH_WS
// (sized for the batch's largest plan), field offsets below.
struct ItemLayout {
    size_t idx, cbase, cscore, cflag, list, segcnt, dlist, fval, fpos, part_c, part_k, sbound, poses7, cidx,
        terms, count, btab, atab, total;
};
ItemLayout item_layout(int Tmax, int NvMax, int P, int nsb2, int chunks, int cb, int frows, int Nmax)
{
    ItemLayout L{};
    size_t o = 0;
    auto take = [&](size_t bytes) {
        const size_t r = o;
        o += align256(std::max<size_t>(bytes, 16));
        return r;
    };
    const size_t K = (size_t)Tmax * P;
    const size_t nidx = (size_t)Tmax * std::max(NvMax, 1) + kPad;   // seq_sum's look-ahead padding
    const size_t nseg = (K + kSelSeg - 1) / kSelSeg;
    const size_t nparts = std::max<size_t>((size_t)((P + cb - 1) / cb) * Tmax, (size_t)chunks * Tmax);
    L.idx = take(sizeof(int2) * nidx);
    L.cbase = take(sizeof(int) * 2 * nidx);   // coarse bases, then superblock bases
    L.cscore = take(sizeof(double) * K);
    L.cflag = take(K);
    L.list = take(sizeof(int) * nseg * kSelSeg);
    L.segcnt = take(sizeof(int) * nseg);
    L.dlist = take(sizeof(int) * K);
    L.fval = take(sizeof(double) * K * frows);
    L.fpos = take(sizeof(int) * K * frows);
    L.part_c = take(sizeof(double) * nparts);
    L.part_k = take(sizeof(long long) * nparts);
    L.sbound = take(sizeof(double) * (size_t)Tmax * std::max(nsb2, 1));
    L.poses7 = take(sizeof(double) * 21);
    L.cidx = take(sizeof(int4) * 7 * (size_t)Nmax);
    L.terms = take(sizeof(double) * 7 * (size_t)Nmax);
    L.count = take(128 + 24 * kSeedWide);   // Lp, Lc[kSeedCands], nsel | wide-seed members
    L.btab = take(sizeof(double4) * (size_t)std::max(NvMax, 1));
    L.atab = take(sizeof(double2) * (size_t)std::max(Tmax, 1));
    L.total = o;
    return L;
}

void bind_workspace(MatchItem& it, char* base, const ItemLayout& L, int frows)
{
    it.idx = (int2*)(base + L.idx);
    it.cbase = (int*)(base + L.cbase);
    it.cscore = (double*)(base + L.cscore);
    it.cflag = (uint8_t*)(base + L.cflag);
    it.list = (int*)(base + L.list);
    it.segcnt = (int*)(base + L.segcnt);
    it.fval = (double*)(base + L.fval);
    it.fpos = (int*)(base + L.fpos);
    it.part_c = (double*)(base + L.part_c);
    it.part_k = (long long*)(base + L.part_k);
    it.sbound = (double*)(base + L.sbound);
    it.poses7 = (double*)(base + L.poses7);
    it.cidx = (int4*)(base + L.cidx);
    it.terms = (double*)(base + L.terms);
    it.Lp = (double*)(base + L.count);
    it.Lc = (double*)(base + L.count + 64);
    it.nsel = (int*)(base + L.count + 64 + 8 * kSeedCands);
    it.seedm = (double*)(base + L.count + 128);
    it.dlist = (int*)(base + L.dlist);
    it.btab = (double4*)(base + L.btab);
    it.atab = (double2*)(base + L.atab);
    static_assert(64 + 8 * kSeedCands + 4 <= 128, "count block layout");
    it.frows = frows;
    it.nseg = (int)((it.pl.K + kSelSeg - 1) / kSelSeg);
}

// Padded phase-plane buffers of nsets coarse maps (S_DECIM, set s at
// s * plane_bytes); their zero margins are written once per (buffer, layout,
// set count) -- the kernels only ever write the interiors.
inline size_t plane_bytes(const RtcsmPlan& pl)
{
    return align256(sizeof(double) * (size_t)pl.low_res * pl.low_res * (size_t)pl.pstride);
}
// the planes' fp16 round-up copies (the superblock pass's input), right after
// each set's fp64 planes: a fixed place per set, so their zero margins stay zero
inline size_t plane16_bytes(const RtcsmPlan& pl)
{
    // (+256: k_super_hv's 8-column loads of the last row may reach 8 bytes past it)
    return align256(sizeof(unsigned short) * (size_t)pl.low_res * pl.low_res * (size_t)pl.pstride) + 256;
}
inline size_t set_bytes(const RtcsmPlan& pl) { return plane_bytes(pl) + plane16_bytes(pl); }
inline size_t super_bytes(const RtcsmPlan& pl)
{
    if (pl.oct) return align256(4 * (size_t)pl.unit8 * pl.low_res * pl.low_res * (size_t)pl.pstrideO);
    return align256(sizeof(SuperT) * (size_t)pl.low_res * pl.low_res * (size_t)pl.pstride4);
}
double* planes_buffer(lgs_ctx* ctx, const RtcsmPlan& pl, int nsets, bool with_super)
{
    const int b = ctx->bank;
    const size_t bytes = set_bytes(pl) * (size_t)nsets;
    double* D = (double*)ctx->ensure(ctx->banked(S_DECIM), bytes);
    // (k_super_planes writes every superblock-plane value; they are zeroed
    // with the planes only so that no stale value is ever read)
    const size_t sbytes = super_bytes(pl) * (size_t)nsets;
    SuperT* S = with_super ? (SuperT*)ctx->ensure(ctx->banked(S_SUPER), sbytes) : nullptr;
    // (the unit layout too: k_super_hv leaves the all-zero units alone)
    const long long key[4] = { pl.low_res, pl.Wq, pl.Hq, pl.M * 16 + pl.oct * 4 + pl.unit8 };
    if (D != ctx->planes_ptr[b] || std::memcmp(key, ctx->planes_key[b], sizeof(key)) != 0 ||
        nsets > ctx->planes_sets[b] || (with_super && (S != ctx->super_ptr[b] || nsets > ctx->super_sets[b]))) {
        LGS_HIP_CHECK(hipMemsetAsync(D, 0, bytes, ctx->stream));
        ctx->planes_ptr[b] = D;
        ctx->planes_sets[b] = nsets;
        std::memcpy(ctx->planes_key[b], key, sizeof(key));
        ctx->super_ptr[b] = nullptr;
        ctx->super_sets[b] = 0;
        if (with_super) {
            LGS_HIP_CHECK(hipMemsetAsync(S, 0, sbytes, ctx->stream));
            ctx->super_ptr[b] = S;
            ctx->super_sets[b] = nsets;
        }
    }
    return D;
}

// One coarse map of a batch: where its planes live and how they are built.
struct PlaneSet {
    const lgs_grid* fine = nullptr;     // precompute from this fine map (OptimizePose(query))
    const lgs_grid* coarse = nullptr;   // or decimate this caller-supplied coarse map
    const double* cmap = nullptr;       // what k_coarse / k_seed_super read
    const SuperT* super = nullptr;
    const int* negflag = nullptr;
    int pgen = 0;
    bool half_copy = false;             // the fp16 copy comes from k_planes16 (not the precompute)
    unsigned short* planes16 = nullptr;
};

// Build the coarse maps of every set: batched precompute straight into the
// padded phase planes (query path) or a phase-plane copy of a supplied coarse
// map, then the superblock planes of all sets in one launch.
struct SetJobs {
    size_t jobs_off = 0, njobs = 0, pj_off = 0, npj = 0, dj_off = 0, ndj = 0;
    bool hv = false;   // k_super_hv (else k_super_planes)
};

// k_super_hv applies: octet unit layout (else k_super_planes)
inline bool hv_mode(const lgs_ctx* ctx, const RtcsmPlan& lp) { return ctx->fused_planes && lp.oct; }
SuperGeom super_geom(const RtcsmPlan& lp)
{
    SuperGeom g{};
    g.M = lp.M;
    g.Wqp = lp.Wqp;
    g.Wq4 = lp.Wq4;
    g.unit8 = lp.unit8;
    g.Hqp = lp.Hqp;
    g.pstride = lp.pstride;
    g.subO = lp.subO;
    g.pstrideO = lp.pstrideO;
    // units that can hold a nonzero value: padded rows / columns [M - 4, M + Hq / Wq)
    g.X4lo = (lp.M - kSB) >> 2;
    g.ncol = ((lp.M + lp.Wq - 1) >> 2) - g.X4lo + 1;
    g.qlo = (lp.M - kSB) >> 4;
    g.nqt = ((lp.M + lp.Hq - 1) >> 4) - g.qlo + 1;
    g.lr = lp.low_res;
    return g;
}

// Zero tiles.  A map is mostly unknown space (+0 cells: the config-2 bench
// map's room covers 23% of its 1000 x 1000 cells), and the per-map passes
// write every plane, fp16 copy and superblock unit of it again for each
// query.  k_precompute_planes (the launch's tiling: 16-row tiles, a lone
// map's shorter ones) and k_super_hv keep one
// word per tile / workgroup and set: 1 = the outputs it stores were built
// from all-(+0) inputs, so they hold +0; a tile whose inputs are still all +0
// then stores nothing -- the same bits, without the writes.  The words are
// kept valid here, per bank: a change of the plane layout, of a launch grid
// or of a buffer clears them all (0 = build the tile), and a set whose planes
// or units another path writes is marked stale, its words cleared before
// their next use.  (Only writers that keep the words write the tiles they
// cover; the zeroing of a whole buffer keeps them true.)
void zero_tiles(lgs_ctx* ctx, const RtcsmPlan& lp, const std::vector<PlaneSet>& sets, std::vector<PrecompJob>& jobs,
                const std::vector<int>& job_set, std::vector<PlaneJob>& pj, double* D, SuperT* S, bool need_super)
{
    const int b = ctx->bank, ns = (int)sets.size(), lr = lp.low_res;
    std::vector<unsigned char>& pre_ok = ctx->zt_pre[b];
    std::vector<unsigned char>& hv_ok = ctx->zt_hv[b];
    if ((int)pre_ok.size() < ns) pre_ok.resize(ns, 0);
    if ((int)hv_ok.size() < ns) hv_ok.resize(ns, 0);
    const bool want = ctx->zero_tiles && need_super && lr <= 8 && hv_mode(ctx, lp);
    const bool use_pre = want && !jobs.empty();
    const bool use_hv = want;
    // every set of this call is rewritten: stale unless a word-keeping pass covers it
    std::vector<unsigned char> pre_now(ns, 0), hv_now(ns, 0);
    int maxW = 0, maxH = 0;   // as launch_sets sizes the precompute's grid
    for (auto& ps : sets)
        if (ps.fine) {
            maxW = std::max(maxW, ps.fine->w);
            maxH = std::max(maxH, ps.fine->h);
        }
    int pgx = 0, pgy = 0, prows = 0;   // the launch's tiling (a lone map: its own, shorter tiles)
    if (use_pre) precompute_tile_grid(maxW, maxH, lr, (int)jobs.size(), &pgx, &pgy, &prows);
    const SuperGeom g = super_geom(lp);
    const int nq = ctx->hv_full && lp.unit8 == 2 ? 2 : 1;
    const int hgx = hv_grid_x(g, nq);
    const long long pre_words = use_pre ? (long long)pgx * pgy : 0;
    const long long hv_words = use_hv ? (long long)lr * lr * hgx : 0;
    const long long per_set = pre_words + hv_words;
    if (per_set > 0) {
        unsigned* Z = (unsigned*)ctx->ensure(ctx->banked(S_ZTILE), sizeof(unsigned) * (size_t)(per_set * ns));
        const long long key[12] = { (long long)(uintptr_t)D, (long long)(uintptr_t)S, (long long)(uintptr_t)Z,
                                    lr, lp.Wq, lp.Hq, lp.M * 16 + lp.oct * 4 + lp.unit8, lp.pstride,
                                    pgx, (long long)pgy << 8 | prows, hgx, nq };
        if (std::memcmp(key, ctx->zt_key[b], sizeof(key)) != 0) {
            std::memcpy(ctx->zt_key[b], key, sizeof(key));
            std::fill(pre_ok.begin(), pre_ok.end(), 0);
            std::fill(hv_ok.begin(), hv_ok.end(), 0);
        }
        bool clear = false;
        for (size_t k = 0; k < jobs.size() && use_pre; ++k) {
            const int s = job_set[k];
            // the word says "+0 outputs" for the tiles of this map size only
            const bool ok = pre_ok[s] && ctx->zt_dims[b].size() > (size_t)s &&
                            ctx->zt_dims[b][s] == ((long long)jobs[k].W << 32 | jobs[k].H);
            clear |= !ok;
            jobs[k].zt = Z + per_set * s;
            pre_now[s] = 1;
        }
        for (int s = 0; s < ns && use_hv; ++s) {
            clear |= !hv_ok[s];
            pj[s].zt = Z + per_set * s + pre_words;
            hv_now[s] = 1;
        }
        // (a cleared word only makes its tile build once more)
        if (clear) LGS_HIP_CHECK(hipMemsetAsync(Z, 0, sizeof(unsigned) * (size_t)(per_set * ns), ctx->stream));
        if (clear) {
            std::fill(pre_ok.begin(), pre_ok.end(), 0);
            std::fill(hv_ok.begin(), hv_ok.end(), 0);
        }
    }
    if ((int)ctx->zt_dims[b].size() < ns) ctx->zt_dims[b].resize(ns, -1);
    for (int s = 0; s < ns; ++s) {
        pre_ok[s] = pre_now[s];
        // units untouched when this call builds none (no superblock pass)
        if (need_super) hv_ok[s] = hv_now[s];
    }
    for (size_t k = 0; k < jobs.size(); ++k)
        ctx->zt_dims[b][job_set[k]] = ((long long)jobs[k].W << 32 | jobs[k].H);
}

void launch_decimate(const double* coarse, const RtcsmPlan& pl, double* D, hipStream_t st);
SetJobs build_sets(lgs_ctx* ctx, const RtcsmPlan& lp, std::vector<PlaneSet>& sets, bool need_super, Upload& up)
{
    const int ns = (int)sets.size();
    hipStream_t st = ctx->stream;
    const int lr = lp.low_res;
    double* D = planes_buffer(ctx, lp, ns, need_super);
    SuperT* S = need_super ? (SuperT*)ctx->ensure(ctx->banked(S_SUPER), super_bytes(lp) * (size_t)ns) : nullptr;
    int* neg = need_super ? (int*)ctx->ensure(ctx->banked(S_NEGFLAG), sizeof(int) * (size_t)ns) : nullptr;
    const size_t pb = plane_bytes(lp) / sizeof(double), sbb = super_bytes(lp) / sizeof(SuperT);
    const size_t ssz = set_bytes(lp) / sizeof(double);   // one set: fp64 planes, then their fp16 copies
    // fine maps with W, H multiples of LowRes: the precompute writes the
    // planes directly (one batched launch); other maps go through a plain
    // scratch map and the phase-plane copy, and supplied coarse maps through
    // the copy; then the superblock planes of every set (one batched launch).
    // (A fused planes + superblock-planes pass from the fine map was measured
    // slower: 1.08-1.19 ms vs 0.40 + 0.56 ms for 64 config-2 maps in r01, and
    // again in r05 as one streaming workgroup per 2 x 16 padded rows of units:
    // 0.61 ms vs 0.23 + 0.21 ms -- the 15-row halo of the vertical max and
    // the serial strips of a workgroup; r05 keeps two passes and moves the
    // horizontal max into the precompute, sh mode.)
    std::vector<PrecompJob> jobs;
    std::vector<int> job_set;
    std::vector<PlaneJob> pj;
    std::vector<DecimJob> djobs;
    for (int s = 0; s < ns; ++s) {
        PlaneSet& ps = sets[s];
        ps.cmap = D + ssz * (size_t)s;
        PlaneJob j{};
        j.pl = lp;
        ps.half_copy = need_super;
        if (need_super) {
            ps.planes16 = (unsigned short*)(D + ssz * (size_t)s + pb);
            j.planes16 = ps.planes16;
            j.super = S + sbb * (size_t)s;
            ps.super = j.super;
            ps.negflag = neg + s;
            ps.pgen = ctx->next_stamp();
            j.negflag = neg + s;
            j.pgen = ps.pgen;
        }
        if (ps.fine && precompute_planes_ok(ps.fine, lr)) {
            PrecompJob q{};
            q.in = ps.fine->d;
            q.out = D + ssz * (size_t)s;
            q.W = ps.fine->w;
            q.H = ps.fine->h;
            q.pg = PlaneGeom{ lp.M, lp.Wqp, lp.pstride };
            if (need_super && lr <= 8) {   // k_precompute_planes writes the fp16 copy itself
                q.out16 = ps.planes16;
                q.negflag = neg + s;
                q.pgen = ps.pgen;
                ps.half_copy = false;
            }
            jobs.push_back(q);
            job_set.push_back(s);
        } else if (ps.fine) {
            // rare (odd map sizes): one set at a time through the shared scratch
            const size_t cells = (size_t)lp.W * lp.H;
            double* plain = (double*)ctx->ensure(S_COARSE_GRID, sizeof(double) * std::max<size_t>(1, cells));
            launch_precompute(ctx, ps.fine, lr, plain, nullptr);
            launch_decimate(plain, lp, D + ssz * (size_t)s, st);
        } else {
            DecimJob dj{ ps.coarse->d, D + ssz * (size_t)s, need_super ? ps.planes16 : nullptr,
                         need_super ? neg + s : nullptr, ps.pgen };
            djobs.push_back(dj);
            ps.half_copy = false;   // k_decimate_jobs writes the copy
        }
        if (need_super) pj.push_back(j);
    }
    zero_tiles(ctx, lp, sets, jobs, job_set, pj, D, S, need_super);
    // the descriptors of this step go up with the batch's items (one copy):
    // the caller flushes before calling launch_sets
    SetJobs sj;
    sj.njobs = jobs.size();
    sj.jobs_off = jobs.empty() ? 0 : up.append(jobs.data(), jobs.size());
    sj.npj = pj.size();
    sj.pj_off = pj.empty() ? 0 : up.append(pj.data(), pj.size());
    sj.ndj = djobs.size();
    sj.dj_off = djobs.empty() ? 0 : up.append(djobs.data(), djobs.size());
    sj.hv = hv_mode(ctx, lp);
    return sj;
}

// Launch the set builds staged by build_sets (after the upload's flush).
void launch_sets(lgs_ctx* ctx, const RtcsmPlan& lp, const std::vector<PlaneSet>& sets, const SetJobs& sj,
                 const Upload& up)
{
    int maxW = 0, maxH = 0;
    for (auto& s : sets)
        if (s.fine) {
            maxW = std::max(maxW, s.fine->w);
            maxH = std::max(maxH, s.fine->h);
        }
    if (sj.njobs)
        launch_precompute_jobs(ctx, up.at<PrecompJob>(sj.jobs_off), (int)sj.njobs, maxW, maxH, lp.low_res);
    if (sj.ndj) {   // supplied coarse maps (all of the plan's size)
        const int np = lp.low_res * lp.low_res;
        hipLaunchKernelGGL(k_decimate_jobs, dim3((lp.Wq + 255) / 256, lp.Hq, np * (int)sj.ndj), dim3(256), 0,
                           ctx->stream, up.at<DecimJob>(sj.dj_off), lp.W, lp.H, lp.low_res, lp.Wq, lp.M, lp.Wqp,
                           lp.pstride);
        LGS_HIP_CHECK(hipGetLastError());
    }
    for (const auto& s : sets)
        if (s.half_copy) {   // planes the batched precompute did not write: their fp16 copy here
            const long long n = (long long)lp.low_res * lp.low_res * lp.pstride;
            hipLaunchKernelGGL(k_planes16, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, ctx->stream, s.cmap,
                               s.planes16, n, const_cast<int*>(s.negflag), s.pgen);
            LGS_HIP_CHECK(hipGetLastError());
        }
    if (sj.npj && sj.hv) {
        const int np = lp.low_res * lp.low_res;
        const SuperGeom g = super_geom(lp);
        const int nq = ctx->hv_full && lp.unit8 == 2 ? 2 : 1;   // threads per column: nqt quads or nqt + 1 units
        dim3 grid(hv_grid_x(g, nq), 1, np * (int)sj.npj);
        // algorithmic bytes: the copies read once (2 B per padded cell of the
        // quads' rows and the units' columns) + the unit halves written (8 B x
        // 16 sub-phases x unit8 copies per quad and column)
        const double cq = (double)np * g.ncol * g.nqt * sj.npj;
        const int tok = ctx->timing_begin(K_SUPER_PLANES, cq * (16.0 * 4.0 * 2.0 + 16.0 * 8.0 * g.unit8));
        if (!ctx->skipped(K_SUPER_PLANES))
        {
            if (nq == 2)
                hipLaunchKernelGGL(HIP_KERNEL_NAME(k_super_hv<2>), grid, dim3(256), 0, ctx->stream,
                                   up.at<PlaneJob>(sj.pj_off), np, g, ctx->dts(tok));
            else
                hipLaunchKernelGGL(HIP_KERNEL_NAME(k_super_hv<1>), grid, dim3(256), 0, ctx->stream,
                                   up.at<PlaneJob>(sj.pj_off), np, g, ctx->dts(tok));
        }
        ctx->timing_end(tok);
        LGS_HIP_CHECK(hipGetLastError());
    } else if (sj.npj) {
        const int np = lp.low_res * lp.low_res;
        const bool lone = sj.npj == 1;
        const int spx = lone ? kSPXLone : kSPX;
        dim3 g((lp.Wqp + spx - 1) / spx, (lp.Hqp + kSPY - 1) / kSPY, np * (int)sj.npj);
        const int tok = ctx->timing_begin(K_SUPER_PLANES, 8.0 * 2.0 * (double)np * lp.pstride * sj.npj);
        if (!ctx->skipped(K_SUPER_PLANES)) {
            if (lone)
                hipLaunchKernelGGL(HIP_KERNEL_NAME(k_super_planes<kSPXLone>), g,
                                   dim3((kSPXLone + 3 + 63) / 64 * 64), 0, ctx->stream, up.at<PlaneJob>(sj.pj_off), np);
            else
                hipLaunchKernelGGL(HIP_KERNEL_NAME(k_super_planes<kSPX>), g, dim3(kSPThreads), 0, ctx->stream,
                                   up.at<PlaneJob>(sj.pj_off), np);
        }
        ctx->timing_end(tok);
        LGS_HIP_CHECK(hipGetLastError());
    }
}

// Phase-plane copy of a plain coarse map into planes D.
void launch_decimate(const double* coarse, const RtcsmPlan& pl, double* D, hipStream_t st)
{
    dim3 gd((pl.Wq + 255) / 256, pl.Hq, pl.low_res * pl.low_res);
    hipLaunchKernelGGL(k_decimate, gd, dim3(256), 0, st, coarse, pl.W, pl.H, pl.low_res, pl.Wq, pl.M, pl.Wqp,
                       pl.pstride, D);
    LGS_HIP_CHECK(hipGetLastError());
}

// k_fine's grid per item: single-wave workgroups looping over the item's
// selected (block, row) items (the count is known only on the device; idle
// workgroups still hold wave slots, so the per-item grid shrinks with the batch)
inline int fine_grid(int n) { return std::max(64, std::min(1024, 8192 / std::max(n, 1))); }
// dynamic LDS: the evaluator's buffers, then the segment prefix (nseg + 1 ints)
inline size_t pref_bytes(int nseg) { return sizeof(int) * (size_t)(nseg + 1); }

struct ScanOptions {
    bool dense = false;
    const std::vector<int4>* patches = nullptr;    // projection patches (t, v, ix, iy)
    const std::vector<int2>* host_idx = nullptr;   // full host projection [T*Nv]
    const std::vector<int4>* cost_patches = nullptr;
    // the search result is already exact: only the cost terms are redone from
    // the previous run's cells with cost_patches applied
    bool cost_only = false;
};

// Host-patched cost cells (cidx[key.x] = cells, computed on the host with
// glibc) and the cost terms recomputed from them (k_cost mode 1).
void enqueue_cost_patches(lgs_ctx* ctx, const BatchShape& B, Items d_items, const std::vector<MatchItem>& items,
                          const std::vector<int4>& cost_patches)
{
    hipStream_t st = ctx->stream;
    const int np = (int)(cost_patches.size() / 2);
    int4* dp = (int4*)ctx->ensure(S_PATCH, sizeof(int4) * cost_patches.size());
    LGS_HIP_CHECK(hipMemcpyAsync(dp, cost_patches.data(), sizeof(int4) * cost_patches.size(),
                                 hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(k_cost_patch, dim3((np + 255) / 256), dim3(256), 0, st, items[0].cidx, dp, np);
    LGS_HIP_CHECK(hipGetLastError());
    hipLaunchKernelGGL(KCOST(B.kernel_size), dim3(7, 1), dim3(kCostThreads), cost_lds(items), st, d_items,
                       ctx->guard_cap, ctx->guard_eps, 0, 1, DevTs{});
    LGS_HIP_CHECK(hipGetLastError());
}

// Enqueue the whole device pipeline of a batch of matches on ctx->stream: one
// launch per stage for all items (d_items: the uploaded descriptors).
// Options (reruns) apply to single-item batches only.
void enqueue_items(lgs_ctx* ctx, const BatchShape& B, Items d_items, const std::vector<MatchItem>& items,
                   const ScanOptions& opt)
{
    if (opt.cost_only) {
        if (opt.cost_patches && !opt.cost_patches->empty())
            enqueue_cost_patches(ctx, B, d_items, items, *opt.cost_patches);
        return;
    }
    hipStream_t st = ctx->stream;
    const int n = B.n;
    const int inject = ctx->inject_index ? 1 : 0;
    const double* zero = ctx->zero;
    double beams_T = 0.0, beams_K = 0.0;   // sum over items of T*Nv, K*Nv (algorithmic bytes)
    for (auto& it : items) {
        beams_T += (double)it.pl.T * it.pl.Nv;
        beams_K += (double)it.pl.K * it.pl.Nv;
    }
    if (B.small) {
        // k_match_small (§4.1c): mode 0 projects, 2 projects and applies the
        // host's guard patches, 1 reads the rows of a full host projection
        int mode = 0;
        if (opt.host_idx) {
            const MatchItem& it = items[0];
            LGS_HIP_CHECK(hipMemcpyAsync(it.idx, opt.host_idx->data(), sizeof(int2) * opt.host_idx->size(),
                                         hipMemcpyHostToDevice, st));
            mode = 1;
        }
        const int4* dp = nullptr;
        int np = 0;
        if (!opt.host_idx && opt.patches && !opt.patches->empty()) {
            dp = (const int4*)ctx->ensure(S_PATCH, sizeof(int4) * opt.patches->size());
            LGS_HIP_CHECK(hipMemcpyAsync((void*)dp, opt.patches->data(), sizeof(int4) * opt.patches->size(),
                                         hipMemcpyHostToDevice, st));
            np = (int)opt.patches->size();
            mode = 2;
        }
        const int lr = B.low_res;
        const int tok = ctx->timing_begin(K_MATCH_SMALL, 8.0 * (lr * lr) * beams_T);
        const dim3 g((unsigned)B.Tmax, (unsigned)n);
        const size_t nvp = (size_t)((std::max(B.NvMax, 1) + 1) & ~1);
#define LGS_SMALL_CASE(L)                                                                                         \
    case L:                                                                                                      \
        hipLaunchKernelGGL(HIP_KERNEL_NAME(k_match_small<L>), g, dim3(64 * (L + 1)),                              \
                           sizeof(int2) * nvp + sizeof(double) * small_buf_doubles<L>(), st, d_items, mode,       \
                           ctx->guard_cap, ctx->guard_eps, inject, zero, dp, np, ctx->dts(tok));                 \
        break;
        if (!ctx->skipped(K_MATCH_SMALL)) switch (lr) {
            LGS_SMALL_CASE(2) LGS_SMALL_CASE(3) LGS_SMALL_CASE(4) LGS_SMALL_CASE(5) LGS_SMALL_CASE(6)
            LGS_SMALL_CASE(7)
            default: LGS_REQUIRE(false, "k_match_small: LowRes outside [2, 7]");
            }
#undef LGS_SMALL_CASE
        ctx->timing_end(tok);
        LGS_HIP_CHECK(hipGetLastError());
        const double kk = (2.0 * B.kernel_size + 1) * (2.0 * B.kernel_size + 1);
        double nbeams = 0.0;
        for (auto& it : items) nbeams += it.cp.N;
        const int tok_ = ctx->timing_begin(K_COST, 8.0 * 7.0 * 2.0 * kk * nbeams);
        if (!ctx->skipped(K_COST))
            hipLaunchKernelGGL(KCOST(B.kernel_size), dim3(7, n), dim3(kCostThreads), cost_lds(items), st, d_items,
                               ctx->guard_cap,
                               ctx->guard_eps, inject, 0, ctx->dts(tok_));
        ctx->timing_end(tok_);
        LGS_HIP_CHECK(hipGetLastError());
        if (opt.cost_patches && !opt.cost_patches->empty())
            enqueue_cost_patches(ctx, B, d_items, items, *opt.cost_patches);
        return;
    }
    if (opt.host_idx) {
        // single item: the full host projection replaces k_project
        const MatchItem& it = items[0];
        LGS_HIP_CHECK(hipMemcpyAsync(it.idx, opt.host_idx->data(), sizeof(int2) * opt.host_idx->size(),
                                     hipMemcpyHostToDevice, st));
        const size_t m = std::max<size_t>((size_t)it.pl.T * it.pl.Nv, kPad);
        hipLaunchKernelGGL(k_cinfo, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, st, d_items);
        LGS_HIP_CHECK(hipGetLastError());
    } else {
        // a lone scan: fewer angles per workgroup (its ~400 angles then fill
        // the GPU; a batch fills it anyway and shares each sincos over more)
        const bool lone = n < ctx->lanes_min_batch;
        const int rows = lone ? kProjRowsLone : kProjRows;
        dim3 g(std::max(1, (B.NvMax + 255) / 256), (B.Tmax + rows - 1) / rows, n);
        // lean batches: the beam / angle tables only (k_super_oct projects)
        const int tok_ = ctx->timing_begin(K_PROJECT, items[0].lean ? 32.0 * B.NvMax * n : 24.0 * beams_T);
        if (ctx->skipped(K_PROJECT)) {
        } else if (items[0].lean)
            hipLaunchKernelGGL(k_beams, dim3(std::max(1, (B.NvMax + 255) / 256), 1, n), dim3(256), 0, st, d_items,
                               ctx->dts(tok_));
        else if (lone)
            hipLaunchKernelGGL(HIP_KERNEL_NAME(k_project<kProjRowsLone>), g, dim3(256), 0, st, d_items, ctx->guard_cap,
                               ctx->guard_eps, inject, ctx->dts(tok_));
        else
            hipLaunchKernelGGL(HIP_KERNEL_NAME(k_project<kProjRows>), g, dim3(256), 0, st, d_items, ctx->guard_cap,
                               ctx->guard_eps, inject, ctx->dts(tok_));
        ctx->timing_end(tok_);
        LGS_HIP_CHECK(hipGetLastError());
        if (opt.patches && !opt.patches->empty()) {
            int4* dp = (int4*)ctx->ensure(S_PATCH, sizeof(int4) * opt.patches->size());
            LGS_HIP_CHECK(hipMemcpyAsync(dp, opt.patches->data(), sizeof(int4) * opt.patches->size(),
                                         hipMemcpyHostToDevice, st));
            const int np = (int)opt.patches->size();
            hipLaunchKernelGGL(k_patch, dim3((np + 255) / 256), dim3(256), 0, st, d_items, dp, np);
            LGS_HIP_CHECK(hipGetLastError());
        }
    }
    const bool dense = opt.dense || ctx->force_dense;
    if (B.pruned) {
        {
            const int tok = ctx->timing_begin(K_SUPER, 8.0 * B.nsb2 * beams_T);
            const size_t lds = sizeof(int) * ((size_t)std::max(B.NvMax, 1) + kOctRowPad);
            dim3 g(B.chunks, B.Tmax, n);
            if (ctx->skipped(K_SUPER)) {
            } else if (B.oct && B.nsby <= 5)
                hipLaunchKernelGGL(HIP_KERNEL_NAME(k_super_oct<5, 2>), g, dim3(64 * kSupWaves), lds, st, d_items, zero, ctx->dts(tok));
            else if (B.oct)   // nsby 6..9: 12-row units (set_plane_layout)
                hipLaunchKernelGGL(HIP_KERNEL_NAME(k_super_oct<9, 3>), g, dim3(64 * kSupWaves), lds, st, d_items, zero, ctx->dts(tok));
            else if (B.pair)
                hipLaunchKernelGGL(HIP_KERNEL_NAME(k_super<1>), g, dim3(64 * kSupWaves), lds, st, d_items, zero);
            else
                hipLaunchKernelGGL(HIP_KERNEL_NAME(k_super<0>), g, dim3(64 * kSupWaves), lds, st, d_items, zero);
            ctx->timing_end(tok);
            LGS_HIP_CHECK(hipGetLastError());
        }
        {
            const int tok = ctx->timing_begin(K_SEED, 8.0 * kSeedCands * (B.low_res * B.low_res + 16.0) * B.NvMax * n);
            const size_t lds = ((sizeof(int) * (size_t)std::max(B.NvMax, 1) + 15) & ~(size_t)15) +
                               sizeof(int2) * (size_t)std::max(B.NvMax, 1);   // coarse + fine beam rows
            // the wide seed for batches; a lone match keeps the one-launch seed
            // (measured r05: lone p50 0.132 -> 0.140 ms with the extra launch,
            // p90 0.155 -> 0.145)
            const int nwide = std::min(ctx->seed_wide, kSeedWide);
            bool wide = nwide > kSeedCands && n >= ctx->lanes_min_batch;
            for (const auto& itm : items) wide = wide && itm.nparts <= kSeedWideMaxParts;
            if (!ctx->skipped(K_SEED) && wide) {
                hipLaunchKernelGGL(k_seed_members, dim3(nwide, n), dim3(kSeedMembersThreads),
                                   sizeof(int) * (size_t)std::max(B.NvMax, 1), st, d_items, ctx->dts(tok));
                hipLaunchKernelGGL(HIP_KERNEL_NAME(k_seed_super<2>), dim3(kSeedCands, n), dim3(LGS_SEED2_THREADS), lds, st,
                                   d_items, zero, ctx->dts(tok));
            } else if (!ctx->skipped(K_SEED))
                hipLaunchKernelGGL(HIP_KERNEL_NAME(k_seed_super<0>), dim3(kSeedCands, n), dim3(1024), lds, st,
                                   d_items, zero, ctx->dts(tok));
            else if (B.wl.cnt)   // (diagnostics) the work-list counters k_seed_super zeroes
                LGS_HIP_CHECK(hipMemsetAsync(B.wl.cnt, 0, sizeof(int) * 16 * (size_t)n, st));
            ctx->timing_end(tok);
            LGS_HIP_CHECK(hipGetLastError());
        }
        // the work list's passes are timed apart (K_COARSE_AUX): K_COARSE is the
        // kernel that makes every coarse lookup (its algorithmic bytes)
        const bool wl = n >= ctx->lanes_min_batch && B.wl.cnt && !ctx->skipped(K_COARSE);
        if (wl) {
            const int tk = ctx->timing_begin(K_COARSE_AUX, 8.0 * (double)B.Tmax * B.nsb2 * n);   // bound reads
            hipLaunchKernelGGL(k_keep, dim3(B.Tmax, n), dim3(64), 0, st, d_items, B.wl, ctx->dts(tk));
            ctx->timing_end(tk);
            LGS_HIP_CHECK(hipGetLastError());
        }
        const int tok = ctx->timing_begin(K_COARSE, 8.0 * beams_K);
        if (tok >= 0) ctx->pending[tok].coarse_evals = true;   // algorithmic bytes from the records
        if (ctx->skipped(K_COARSE)) {
        } else if (wl) {
            hipLaunchKernelGGL(k_coarse_list_c, dim3(kListWaves), dim3(64), 0, st, d_items, B.wl, n, zero, ctx->dts(tok));
        } else {
            const size_t lds = ((sizeof(int) * (size_t)B.NvMax + 15) & ~(size_t)15) +
                               sizeof(double) * 128 * kRing * kRowWaves;
            hipLaunchKernelGGL(k_coarse_rows, dim3(B.Tmax, kSB, kRowSplit * n), dim3(64 * kRowWaves), lds, st,
                               d_items, zero);
        }
        ctx->timing_end(tok);
        LGS_HIP_CHECK(hipGetLastError());
        if (wl) {
            const int tk = ctx->timing_begin(K_COARSE_AUX, 0.0);
            hipLaunchKernelGGL(k_unsafe_list, dim3(std::min(kUnsafeGroups, n * B.Tmax)), dim3(64 * kLaneWaves), 0, st,
                               d_items, B.wl, n, zero, ctx->dts(tk));
            ctx->timing_end(tk);
            LGS_HIP_CHECK(hipGetLastError());
        }
    } else {
        {
            dim3 g((B.P + B.cb - 1) / B.cb, B.Tmax, n);
            const int tok = ctx->timing_begin(K_COARSE, 8.0 * beams_K);
            hipLaunchKernelGGL(k_coarse, g, dim3(B.cb), 0, st, d_items, zero);
            ctx->timing_end(tok);
            LGS_HIP_CHECK(hipGetLastError());
        }
        const int tok = ctx->timing_begin(K_SEED, 8.0 * B.low_res * B.low_res * (double)B.NvMax * n);
        if (B.lr5)
            hipLaunchKernelGGL(k_seed<5>, dim3(1, n), dim3(64 * 5), eval_t_smem<5>(B.NvMax), st, d_items, zero,
                               dense ? 1 : 0);
        else
            hipLaunchKernelGGL(k_seed<0>, dim3(1, n), dim3(64), sidx_bytes(B.NvMax), st, d_items, zero,
                               dense ? 1 : 0);
        ctx->timing_end(tok);
        LGS_HIP_CHECK(hipGetLastError());
    }
    {
        const int tok_ = ctx->timing_begin(K_SELECT, 10.0 * (double)B.Tmax * B.P * n);
        if (!ctx->skipped(K_SELECT)) {
            if (n >= ctx->lanes_min_batch)
                hipLaunchKernelGGL(HIP_KERNEL_NAME(k_select<256>), dim3((unsigned)B.nsegMax, n), dim3(256), 0, st,
                                   d_items, B.pruned ? 1 : 0, ctx->dts(tok_));
            else
                hipLaunchKernelGGL(HIP_KERNEL_NAME(k_select<kSelSeg>), dim3((unsigned)B.nsegMax, n), dim3(kSelSeg), 0,
                                   st, d_items, B.pruned ? 1 : 0, ctx->dts(tok_));
        }
        ctx->timing_end(tok_);
        LGS_HIP_CHECK(hipGetLastError());
    }
    if (B.fine_lanes) {
        hipLaunchKernelGGL(k_compact, dim3(n), dim3(256), pref_bytes(B.nsegMax), st, d_items);
        LGS_HIP_CHECK(hipGetLastError());
        const int tok_ = ctx->timing_begin(K_FINE, 0.0);
        if (ctx->skipped(K_FINE)) {
        } else if (B.fine_staged && ctx->fine_staged) {
            hipLaunchKernelGGL(k_fine_regs, dim3(4096), dim3(64), sizeof(unsigned) * (size_t)(B.NvMax + kFrPad), st,
                               d_items, n, zero, ctx->dts(tok_));
        } else {
            hipLaunchKernelGGL(k_fine_lanes, dim3(4096), dim3(64 * kFineLanesWaves),
                               sizeof(int2) * (size_t)(B.NvMax + 4 * kPipe), st, d_items, n, zero);
        }
        ctx->timing_end(tok_);
        LGS_HIP_CHECK(hipGetLastError());
    } else {
        const int tok_ = ctx->timing_begin(K_FINE, 0.0);
        dim3 g(fine_grid(n), n);
        if (ctx->skipped(K_FINE)) {
        } else if (B.lr5) {
            // one wave's share of the evaluator's LDS (row split)
            const size_t e = (sizeof(int2) * (size_t)((B.NvMax + 1) & ~1) + sizeof(double) * 2 * 5 * 65 + 15) &
                             ~size_t(15);
            hipLaunchKernelGGL(k_fine<5>, g, dim3(64), e + pref_bytes(B.nsegMax), st, d_items, zero, (unsigned)e);
        } else {
            const size_t e = (sidx_bytes(B.NvMax) + 15) & ~size_t(15);
            hipLaunchKernelGGL(k_fine<0>, g, dim3(64), e + pref_bytes(B.nsegMax), st, d_items, zero, (unsigned)e);
        }
        ctx->timing_end(tok_);
        LGS_HIP_CHECK(hipGetLastError());
    }
    {
        const int tok_ = ctx->timing_begin(K_REPLAY, 0.0);
        if (!ctx->skipped(K_REPLAY))
            hipLaunchKernelGGL(k_replay, dim3(n), dim3(64), pref_bytes(B.nsegMax), st, d_items, ctx->dts(tok_));
        ctx->timing_end(tok_);
        LGS_HIP_CHECK(hipGetLastError());
    }
    // cost + covariance terms at the 7 poses
    const double kk = (2.0 * B.kernel_size + 1) * (2.0 * B.kernel_size + 1);
    double nbeams = 0.0;
    for (auto& it : items) nbeams += it.cp.N;
    {
        const int tok_ = ctx->timing_begin(K_COST, 8.0 * 7.0 * 2.0 * kk * nbeams);
        if (!ctx->skipped(K_COST))
            hipLaunchKernelGGL(KCOST(B.kernel_size), dim3(7, n), dim3(kCostThreads), cost_lds(items), st, d_items,
                               ctx->guard_cap,
                               ctx->guard_eps, inject, 0, ctx->dts(tok_));
        ctx->timing_end(tok_);
        LGS_HIP_CHECK(hipGetLastError());
    }
    if (opt.cost_patches && !opt.cost_patches->empty())
        enqueue_cost_patches(ctx, B, d_items, items, *opt.cost_patches);
}

// Host view of a device record: the generation-tagged guard words decoded.
inline int tagged_count(unsigned long long w, int gen)
{
    return ((unsigned)(w >> 32) == (unsigned)gen) ? (int)(unsigned)w : 0;
}
struct HostRecord : RtcsmRecord {
    int guard_count = 0, cost_guard_count = 0;
    HostRecord(const RtcsmRecord& r, int gen) : RtcsmRecord(r)
    {
        guard_count = tagged_count(r.guard_word, gen);
        cost_guard_count = tagged_count(r.cost_guard_word, gen);
    }
};

// glibc recomputation of one projected index (host side of the guard).
void host_project(const RtcsmPlan& pl, const lgs_scan* scan, int vbeam, int tt, int& ix, int& iy)
{
    const double r = scan->h_ranges[vbeam];
    const double a = scan->h_angles[vbeam];
    const double th = pl.st + pl.step_t * (double)(tt - pl.win_t);
    double s, c;
    ref_sincos(th + a, s, c);
    const double hx = pl.sx + r * c;
    const double hy = pl.sy + r * s;
    ix = (int)std::floor((hx - pl.min_x) / pl.res);
    iy = (int)std::floor((hy - pl.min_y) / pl.res);
}

void host_cost_cells(const CostPlan& cp, const lgs_scan* scan, const double pose[3], int beam,
                     int cells[4])
{
    const double r = scan->h_ranges[beam];
    double s, c;
    ref_sincos(pose[2] + scan->h_angles[beam], s, c);
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
                             const HostRecord& rec, std::vector<int4>& patches,
                             std::vector<int2>& host_idx, bool& use_host_idx)
{
    use_host_idx = false;
    patches.clear();
    if (rec.guard_count == 0) return false;
    int nvl = 0;   // this match's compaction (the list of its ScanRangeMax)
    const int* vidx = scan_valid_indices(ctx, const_cast<lgs_scan*>(scan), pl.rmax, &nvl);
    LGS_REQUIRE(nvl == pl.Nv, "scan compaction changed under a match");
    if (rec.guard_count > ctx->guard_cap) {
        // too many to inspect: full host projection (exact, slow path)
        host_idx.resize((size_t)pl.T * pl.Nv);
        for (int tt = 0; tt < pl.T; ++tt)
            for (int v = 0; v < pl.Nv; ++v) {
                int ix, iy;
                host_project(pl, scan, vidx[v], tt, ix, iy);
                host_idx[(size_t)tt * pl.Nv + v] = make_int2(ix, iy);
            }
        use_host_idx = true;
        return true;
    }
    for (int k = 0; k < rec.guard_count; ++k) {
        const GuardRec& g = rec.guard[k];
        int ix, iy;
        host_project(pl, scan, vidx[g.v], g.t, ix, iy);
        if (ix != g.ix || iy != g.iy) patches.push_back(make_int4(g.t, g.v, ix, iy));
    }
    return !patches.empty();
}

bool check_cost_guards_p7(lgs_ctx* ctx, const double P7[7][3], const CostPlan& cp, const lgs_scan* scan,
                          const HostRecord& rec, std::vector<int4>& cpatch, bool& full);

bool check_cost_guards(lgs_ctx* ctx, const RtcsmPlan& pl, const CostPlan& cp,
                       const lgs_scan* scan, const HostRecord& rec, std::vector<int4>& cpatch,
                       bool& full)
{
    double P7[7][3];
    host_poses7(pl, rec.best, P7);
    return check_cost_guards_p7(ctx, P7, cp, scan, rec, cpatch, full);
}

// Verify the guarded cost cells of the 7 poses P7 against glibc; true if the
// costs must be re-evaluated (cpatch: (key, cells) pairs, or full = every row).
bool check_cost_guards_p7(lgs_ctx* ctx, const double P7[7][3], const CostPlan& cp, const lgs_scan* scan,
                          const HostRecord& rec, std::vector<int4>& cpatch, bool& full)
{
    cpatch.clear();
    full = false;
    if (rec.cost_guard_count == 0) return false;
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

void finish_summary(const RtcsmPlan& pl, const lgs_scan* scan, lgs_pose2d initial, bool pruned,
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
    out->coarse_blocks = pruned ? (int64_t)rec.coarse_evals : pl.K;
    out->fine_blocks = rec.n_eval;
}

void check_args(const lgs_grid* grid, const lgs_rtcsm_params* p, const lgs_cost_ge_params* c, const lgs_scan* s)
{
    LGS_REQUIRE(grid && p && c && s, "null argument");
    LGS_REQUIRE(p->low_resolution >= 1 && p->low_resolution <= 32, "low_resolution must be in [1, 32]");
    LGS_REQUIRE(p->range_x >= 0 && p->range_y >= 0 && p->range_theta >= 0, "negative search range");
    LGS_REQUIRE(s->n >= 1, "empty scan");
    LGS_REQUIRE(s->n <= 16384, "at most 16384 beams per scan (LDS-staged index rows)");
    LGS_REQUIRE(c->kernel_size >= 0, "negative kernel size");
}

void check_coarse(const lgs_grid* grid, const lgs_grid* coarse)
{
    LGS_REQUIRE(coarse, "null coarse map");
    LGS_REQUIRE(grid->w == coarse->w && grid->h == coarse->h && grid->min_x == coarse->min_x &&
                    grid->min_y == coarse->min_y && grid->res == coarse->res,
                "coarse map must have the fine map's geometry (CreateSameSizeMap)");
}

// Run n matches as one batch: the items share the search parameters and the
// map geometry; sets are the distinct coarse maps (set_of[j] = item j's).
// One host synchronisation in the common case; guarded projections and
// dangerous blocks trigger exact single-item reruns.
// A launched batch whose results the host has not taken yet.
struct InFlight {
    std::vector<MatchItem> items;
    BatchShape B;
    std::vector<int> gens;
    std::vector<PlaneSet> sets;
    const lgs_grid* const* grids = nullptr;
    lgs_scan* const* scans = nullptr;
    const lgs_pose2d* init = nullptr;
    lgs_rtcsm_summary* out = nullptr;
    RtcsmRecord* h_rec = nullptr;
    RtcsmRecord* d_rec = nullptr;
    int n = 0, bank = 0;
    long long id = 0;   // timing batch
    bool post = false;            // records written by k_post (LGS_OPT_POST_RECORDS)
    unsigned* flag = nullptr;     // its completion flag in the pinned record buffer
    unsigned post_gen = 0;
};

// Lean projection (LGS_OPT_LEAN_PROJECT): only when every kernel enqueue_items
// will launch on this batch forms its coarse-base and cell rows itself -- the
// pruned work-list chain with the wide seed and the staged fine evaluator
// (k_super_oct, k_seed_members + k_seed_super<2>, k_keep, k_coarse_list_c,
// k_unsafe_list, k_fine_regs) -- the same decisions enqueue_items makes.
bool lean_rows(const lgs_ctx* ctx, const BatchShape& B, const std::vector<MatchItem>& items)
{
    const int n = B.n;
    if (!ctx->lean_project || B.small || !B.pruned || !B.oct || n < ctx->lanes_min_batch || !B.wl.cnt) return false;
    if (ctx->skip_mask) return false;   // (diagnostics: skipped stages leave stale rows either way)
    if (!(B.fine_lanes && B.fine_staged && ctx->fine_staged)) return false;
    if (!(std::min(ctx->seed_wide, kSeedWide) > kSeedCands)) return false;
    for (const auto& it : items)
        if (it.nparts > kSeedWideMaxParts) return false;
    return true;
}

// The device part of a batch, on ctx->bank's buffers: every stage launched,
// the records' copy to the host queued and the bank's event recorded.
void launch_matches(lgs_ctx* ctx, const lgs_rtcsm_params* params, const lgs_cost_ge_params* cost,
                    const lgs_grid* const* grids, lgs_scan* const* scans, const lgs_pose2d* init, int n,
                    double nthr, std::vector<PlaneSet>& sets, const int* set_of, lgs_rtcsm_summary* out,
                    InFlight& F)
{
    LGS_HIP_CHECK(hipSetDevice(ctx->device));
    LGS_REQUIRE(n >= 1 && n <= kMaxBatchItems, "batch of 1..64 matches (run_chunked splits larger ones)");
    std::vector<MatchItem> items((size_t)n);
    BatchShape B;
    B.n = n;
    int Nmax = 1;
    for (int j = 0; j < n; ++j) {
        check_args(grids[j], params, cost, scans[j]);
        grid_acquire(ctx, grids[j]);
        LGS_REQUIRE(grids[j]->w == grids[0]->w && grids[j]->h == grids[0]->h && grids[j]->res == grids[0]->res,
                    "the maps of one batch must share their size and resolution");
        int nv = 0;
        scan_valid_indices(ctx, scans[j], params->scan_range_max, &nv);
        MatchItem& it = items[j];
        std::memset(&it, 0, sizeof(it));
        it.pl = make_plan(grids[j], params, scans[j], init[j], nthr, nv);
        // the segment prefix of the selection lives in LDS next to the evaluator
        LGS_REQUIRE(it.pl.K <= 7LL * 1024 * 1024, "search window too large (> 7M coarse blocks)");
        it.cp = make_cost_plan(grids[j], cost, scans[j]);
        B.Tmax = std::max(B.Tmax, it.pl.T);
        B.NvMax = std::max(B.NvMax, nv);
        Nmax = std::max(Nmax, scans[j]->n);
    }
    for (auto& s : sets)
        if (s.coarse) check_coarse(grids[0], s.coarse);
    const RtcsmPlan& p0 = items[0].pl;
    B.P = p0.P;
    B.nsb2 = p0.nsbx * p0.nsby;
    B.low_res = p0.low_res;
    B.cb = coarse_block(p0);
    B.pair = B.nsb2 <= 32;
    B.chunks = B.pair ? 1 : (B.nsb2 + 63) / 64;
    B.oct = p0.oct != 0;
    B.unit8 = p0.unit8;
    B.nsby = p0.nsby;
    B.pruned = uses_super(ctx, B.NvMax, B.nsb2, false);
    B.lr5 = lr5_path(B.NvMax, B.low_res);
    // lone matches keep the transposed row evaluator (LR waves per block: lower
    // latency for a handful of blocks); batches spread their blocks lane-per-pose
    B.fine_lanes = n >= ctx->lanes_min_batch && B.low_res * B.low_res <= 64 &&
                   B.NvMax <= kFineLanesMaxNv;
    B.frows = (B.lr5 && !B.fine_lanes) ? 5 : 1;
    B.fine_staged = B.fine_lanes && B.low_res == 5;
    for (int j = 0; j < n && B.fine_staged; ++j)
        B.fine_staged = grids[j]->w % 2 == 0 && ((uintptr_t)grids[j]->d & 15) == 0 && grids[j]->w <= 8192 &&
                        grids[j]->h <= 8192;
    B.kernel_size = cost->kernel_size;
    B.nsegMax = (int)(((long long)B.Tmax * B.P + kSelSeg - 1) / kSelSeg);
    // one coarse block per angle: the whole search in one launch, straight
    // from the fine map (no caller-supplied coarse map to honour)
    B.small = ctx->small_window && !ctx->force_dense && p0.P == 1 && B.low_res >= 2 && B.low_res <= 7 &&
              B.NvMax <= kSmallMaxNv && n <= kTedgeCtrs;
    for (int j = 0; j < n; ++j) B.small = B.small && grids[j]->w >= B.low_res && grids[j]->h >= 1;   // clamped runs
    for (auto& s : sets) B.small = B.small && !s.coarse;
    if (B.small) B.pruned = false;
    if (B.pruned && n >= ctx->lanes_min_batch && B.NvMax <= kListMaxNv && B.Tmax < (1 << 24) && B.nsb2 <= 64) {
        // the kept-superblock work list: counters | superblock entries | edge angles
        int region = 1;
        for (auto& it : items) region = std::max(region, it.pl.T * it.pl.nsbx * it.pl.nsby);
        int* wl = (int*)ctx->ensure(S_KEEP, sizeof(int) * (size_t)n * (16 + (size_t)region + (size_t)B.Tmax));
        B.wl = WorkList{ wl, wl + 16 * (size_t)n, wl + 16 * (size_t)n + (size_t)region * n, region, B.Tmax };
    }
    const ItemLayout L = item_layout(B.Tmax, B.NvMax, B.P, B.nsb2, B.chunks, B.cb, B.frows, Nmax);
    char* ws = (char*)ctx->ensure(ctx->banked(S_BATCH_WS), L.total * (size_t)n);
    RtcsmRecord* d_rec = (RtcsmRecord*)ctx->ensure(ctx->banked(S_RECORDS), sizeof(RtcsmRecord) * (size_t)n);
    // the records' host copy, then (k_post) a completion flag
    const size_t rec_bytes = sizeof(RtcsmRecord) * (size_t)n;
    // (pinned layout: records | flag (256 B) | the chunk's device-timing words)
    constexpr size_t kDtsBytes = sizeof(unsigned long long) * 2 * kDtsSub * kDtsSlots;
    RtcsmRecord* h_rec = (RtcsmRecord*)ctx->ensure_pinned_rec(align256(rec_bytes) + 256 + kDtsBytes);
    unsigned* h_flag = (unsigned*)((char*)h_rec + align256(rec_bytes));
    F.id = ++ctx->timing_batch;
    // LGS_OPT_DEVICE_TIMING: the chain's launches stamp this bank's words,
    // copied back with the records (k_post); reruns keep event timing
    struct DtsScope {
        lgs_ctx* c;
        ~DtsScope() { c->dts_dev = nullptr; }
    } dts_scope{ ctx };
    if (ctx->profile && ctx->dev_timing) {
        unsigned long long*& db = ctx->dts_buf[ctx->bank];
        if (++ctx->dts_gen >= (1u << 24) || !db) {   // a new buffer, or the generations wrapped: zero the words
            if (ctx->dts_gen >= (1u << 24)) ctx->dts_gen = 1;
            for (int b = 0; b < 2; ++b) {
                if (!ctx->dts_buf[b]) LGS_HIP_CHECK(hipMalloc((void**)&ctx->dts_buf[b], kDtsBytes));
                LGS_HIP_CHECK(hipMemsetAsync(ctx->dts_buf[b], 0, kDtsBytes, ctx->stream));
            }
        }
        ctx->dts_dev = db;
        ctx->dts_host = (const unsigned long long*)((char*)h_flag + 256);
        ctx->dts_used = 0;
    }
    // The angle flags are only ever SET (k_project stamps an angle whose lattice
    // leaves the map low with the match's generation).  They live in a buffer
    // of their own that holds nothing but stamps, so a stale flag can never
    // equal this match's generation and no clearing is needed.
    if (ctx->poison_ws) {   // diagnostics: any read-before-write of this batch sees 0xFF bytes
        LGS_HIP_CHECK(hipMemsetAsync(ws, 0xFF, L.total * (size_t)n, ctx->stream));
        LGS_HIP_CHECK(hipMemsetAsync(d_rec, 0xFF, sizeof(RtcsmRecord) * (size_t)n, ctx->stream));
    }
    int* tedge = ctx->tedge_buffer((size_t)n * B.Tmax);   // stamps only: no clearing per batch
    int* sctr = B.small ? ctx->small_counters((size_t)n * B.Tmax) : nullptr;
    Upload up(ctx);
    scans_to_device(ctx, scans, n, &up);
    const SetJobs sj = B.small ? SetJobs{} : build_sets(ctx, p0, sets, B.pruned, up);
    std::vector<int> gens((size_t)n);
    for (int j = 0; j < n; ++j) {
        MatchItem& it = items[j];
        bind_workspace(it, ws + L.total * (size_t)j, L, B.frows);
        it.tedge = tedge + (size_t)j * B.Tmax;
        it.grid = grids[j]->d;
        it.ranges = scans[j]->d_ranges;
        it.angles = scans[j]->d_angles;
        const PlaneSet& s = sets[set_of[j]];
        it.cmap = s.cmap;
        it.super = s.super;
        it.negflag = s.negflag;
        it.pgen = s.pgen;
        it.gen = gens[j] = ctx->generation = ctx->next_stamp();
        it.rec = d_rec + j;
        it.keepc = B.wl.cnt ? B.wl.cnt + 16 * j : sctr ? sctr + j : nullptr;
        it.nparts = item_nparts(B, it.pl, B.pruned);
        it.nseedm = std::min(ctx->seed_wide, kSeedWide);
        it.inject = ctx->inject_index ? 1 : 0;
        it.geps = ctx->guard_eps;
        it.gcap = ctx->guard_cap;
    }
    const bool lean = lean_rows(ctx, B, items);
    for (auto& it : items) it.lean = lean ? 1 : 0;
    ctx->dbg.assign((size_t)n, lgs_ctx::DbgItem{});
    for (int j = 0; j < n; ++j) {
        // every item's intermediates for lgs_debug_item_buffer (diagnostics)
        const MatchItem& ij = items[j];
        const RtcsmPlan& q = ij.pl;
        const size_t nidx = (size_t)q.T * std::max(q.Nv, 1) + kPad;
        const void* b[8] = { ij.sbound, ij.part_c, ij.part_k, ij.Lp, ij.tedge, ij.cbase, ij.idx, ij.cscore };
        const size_t sz[8] = { sizeof(double) * (size_t)q.T * B.nsb2, sizeof(double) * (size_t)ij.nparts,
                               sizeof(long long) * (size_t)ij.nparts, 64 + sizeof(double) * kSeedCands,
                               sizeof(int) * (size_t)q.T, sizeof(int) * 2 * nidx,
                               sizeof(int2) * (size_t)q.T * q.Nv, sizeof(double) * (size_t)q.K };
        lgs_ctx::DbgItem& d = ctx->dbg[j];
        for (int k = 0; k < 8; ++k) {
            d.buf[k] = b[k];
            d.bytes[k] = sz[k];
        }
        d.buf[8] = ij.cmap;   // the item's coarse phase planes and superblock planes (none: k_match_small)
        d.bytes[8] = ij.cmap ? plane_bytes(q) : 0;
        d.buf[9] = ij.super;
        d.bytes[9] = ij.super ? super_bytes(q) : 0;
        d.gen = ij.gen;
    }
    const size_t items_off = up.append(items.data(), items.size());
    up.flush();
    if (!B.small) launch_sets(ctx, p0, sets, sj, up);
    // the stages after the coarse-map builds on the high-priority stream (the
    // context's stream is restored when this function returns)
    struct StreamRestore {
        lgs_ctx* c;
        hipStream_t s;
        ~StreamRestore() { c->stream = s; }
    } restore{ ctx, ctx->stream };
    if (!B.small && ctx->prio_tail && ctx->hi) {
        LGS_HIP_CHECK(hipEventRecord(ctx->split_ev[ctx->bank], ctx->stream));
        LGS_HIP_CHECK(hipStreamWaitEvent(ctx->hi, ctx->split_ev[ctx->bank], 0));
        ctx->stream = ctx->hi;
    }
    enqueue_items(ctx, B, up.at<MatchItem>(items_off), items, ScanOptions{});
    F.post = ctx->post_records;
    if (F.post) {
        static_assert(sizeof(RtcsmRecord) % 16 == 0, "k_post copies 16-byte words");
        F.flag = h_flag;
        F.post_gen = (unsigned)ctx->next_stamp();
        *(volatile unsigned*)h_flag = 0u;   // before the launch: k_post's store comes after it
        const int n16 = (int)(rec_bytes / 16);   // one word per thread where it fits (a lone match: one wave)
        const int n2 = ctx->dts_dev ? (int)(kDtsBytes / 16) : 0;
        hipLaunchKernelGGL(k_post, dim3(1), dim3(std::min(kPostThreads, (std::max(n16, n2) + 63) / 64 * 64)), 0,
                           ctx->stream, (const uint4*)d_rec, (uint4*)h_rec, (int)(rec_bytes / 16), h_flag, F.post_gen,
                           (const uint4*)ctx->dts_dev, (uint4*)ctx->dts_host, n2);
        LGS_HIP_CHECK(hipGetLastError());
    } else {
        LGS_HIP_CHECK(hipMemcpyAsync(h_rec, d_rec, rec_bytes, hipMemcpyDeviceToHost, ctx->stream));
        if (ctx->dts_dev)
            LGS_HIP_CHECK(hipMemcpyAsync(const_cast<unsigned long long*>(ctx->dts_host), ctx->dts_dev, kDtsBytes,
                                         hipMemcpyDeviceToHost, ctx->stream));
    }
    hipEvent_t& ev = ctx->bank_ev[ctx->bank];
    if (!ev) LGS_HIP_CHECK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    LGS_HIP_CHECK(hipEventRecord(ev, ctx->stream));
    // the tail ran on the priority stream: the context's own stream waits for
    // it, so every later synchronisation of that stream (sync(), a scratch
    // regrow in ensure*) also covers the tail's reads of the scratch
    if (ctx->stream != restore.s) LGS_HIP_CHECK(hipStreamWaitEvent(restore.s, ev, 0));
    F.items = std::move(items);
    F.B = B;
    F.gens = std::move(gens);
    F.sets = sets;
    F.grids = grids;
    F.scans = scans;
    F.init = init;
    F.out = out;
    F.h_rec = h_rec;
    F.d_rec = d_rec;
    F.n = n;
    F.bank = ctx->bank;
}

// The host part: wait for the batch's records (not for later batches), then
// the guard checks, exactness reruns (on the batch's own bank) and summaries.
void finish_matches(lgs_ctx* ctx, InFlight& F)
{
    ctx->bank = F.bank;
    if (F.post) {
        // spin on the flag k_post writes last; the stream's event (recorded
        // after it) tells a fault or a lost flag apart from work in flight
        volatile unsigned* f = F.flag;
        for (unsigned spins = 1; *f != F.post_gen; ++spins) {
            if (spins % 4096) continue;
            const hipError_t e = hipEventQuery(ctx->bank_ev[F.bank]);
            if (e == hipSuccess && *f != F.post_gen) throw Error(LGS_ERR_INTERNAL, "k_post: completion flag lost");
            if (e != hipSuccess && e != hipErrorNotReady) LGS_HIP_CHECK(e);
        }
        std::atomic_thread_fence(std::memory_order_acquire);
    } else {
        ctx->wait_event(ctx->bank_ev[F.bank]);
    }
    ctx->up_busy[F.bank] = false;   // the chunk, its descriptor copy included, is complete
    std::vector<MatchItem>& items = F.items;
    const BatchShape& B = F.B;
    const std::vector<int>& gens = F.gens;
    lgs_scan* const* scans = F.scans;
    const lgs_pose2d* init = F.init;
    lgs_rtcsm_summary* out = F.out;
    RtcsmRecord* h_rec = F.h_rec;
    RtcsmRecord* d_rec = F.d_rec;
    const int n = F.n;
    if (ctx->profile) {
        double coarse_bytes = 0.0;   // pruned k_coarse: 8 B x Nv per block it scored
        for (int j = 0; j < n; ++j) coarse_bytes += 8.0 * items[j].pl.Nv * (double)h_rec[j].coarse_evals;
        for (auto& pt : ctx->pending)
            if (pt.coarse_evals && pt.batch == F.id) {
                pt.algo_bytes = coarse_bytes;
                pt.coarse_evals = false;
            }
        ctx->harvest_upto(F.id);
    }
    const long long saved_batch = ctx->timing_batch;
    ctx->timing_batch = F.id;   // reruns' timings belong to this batch

    for (int j = 0; j < n; ++j) {
        HostRecord rec(h_rec[j], gens[j]);
        const int guard_hits = rec.guard_count + rec.cost_guard_count;
        int fixups = 0, slow = 0;
        bool pruned = B.pruned;
        // exactness loop: at most a few reruns
        ScanOptions opt;
        std::vector<int4> patches, cpatch;
        std::vector<int2> hidx;
        for (int iter = 0; iter < 4; ++iter) {
            bool use_hidx = false, full_cost = false;
            bool rerun = false;
            if (!opt.host_idx && !opt.patches &&
                check_projection_guards(ctx, items[j].pl, scans[j], rec, patches, hidx, use_hidx)) {
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
                const CostPlan& cp = items[j].cp;
                if (check_cost_guards(ctx, items[j].pl, cp, scans[j], rec, cpatch, full_cost)) {
                    if (full_cost) {
                        // rebuild every cost cell on the host
                        double P7[7][3];
                        host_poses7(items[j].pl, rec.best, P7);
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
                    opt.cost_only = true;   // the search result stands: redo the cost terms only
                    rerun = true;
                    fixups = 1;
                }
            }
            if (!rerun) break;
            // single-item rerun in the item's own workspace and planes
            BatchShape B1 = B;
            B1.n = 1;
            B1.Tmax = items[j].pl.T;
            B1.nsegMax = items[j].nseg;
            B1.pruned = pruned = !B.small && uses_super(ctx, B.NvMax, B.nsb2, opt.dense);
            std::vector<MatchItem> one(1, items[j]);
            one[0].nparts = item_nparts(B1, one[0].pl, B1.pruned);
            one[0].lean = 0;   // a rerun materialises its rows (k_patch / the host's rows patch them)
            const int g = one[0].gen = ctx->generation = ctx->next_stamp();
            if ((size_t)j < ctx->dbg.size()) ctx->dbg[j].gen = g;
            Upload u1(ctx);
            const size_t off = u1.append(one.data(), 1);
            u1.flush();
            enqueue_items(ctx, B1, u1.at<MatchItem>(off), one, opt);
            LGS_HIP_CHECK(hipMemcpyAsync(&h_rec[j], d_rec + j, sizeof(RtcsmRecord), hipMemcpyDeviceToHost,
                                         ctx->stream));
            ctx->sync();
            if (ctx->profile) ctx->harvest_upto(F.id);
            rec = HostRecord(h_rec[j], g);
            if (opt.patches || opt.host_idx) rec.guard_count = 0;  // already exact
        }
        finish_summary(items[j].pl, scans[j], init[j], pruned, rec, &out[j]);
        out[j].guard_hits = guard_hits;
        out[j].fixups = fixups;
        out[j].slow_path = slow;
        ctx->count_matches += 1;
        ctx->count_coarse_blocks += out[j].coarse_blocks;
        ctx->count_coarse_blocks_dense += items[j].pl.K;
        ctx->count_pruned += pruned ? 1 : 0;
    }
    ctx->timing_batch = saved_batch;
    ctx->bank = 0;
}

void run_matches(lgs_ctx* ctx, const lgs_rtcsm_params* params, const lgs_cost_ge_params* cost,
                 const lgs_grid* const* grids, lgs_scan* const* scans, const lgs_pose2d* init, int n,
                 double nthr, std::vector<PlaneSet>& sets, const int* set_of, lgs_rtcsm_summary* out)
{
    InFlight F;
    ctx->bank = 0;
    launch_matches(ctx, params, cost, grids, scans, init, n, nthr, sets, set_of, out, F);
    finish_matches(ctx, F);
}


// Batches of at most kMaxBatch items (bounded scratch: ~20 MB per config-2
// item), each with only the coarse maps its items reference.
constexpr int kMaxBatch = kMaxBatchItems;
constexpr int kSplitMin = 16;   // smallest chunk of a split call
void run_chunked(lgs_ctx* ctx, const lgs_rtcsm_params* params, const lgs_cost_ge_params* cost,
                 const lgs_grid* const* grids, lgs_scan* const* scans, const lgs_pose2d* init, int n,
                 double nthr, const std::vector<PlaneSet>& sets_all, const int* set_of, lgs_rtcsm_summary* out)
{
    // two chunks in flight: chunk c + 1 is launched (on the other bank)
    // before the host takes chunk c's results, so the device never waits for
    // the host between chunks of one call
    InFlight fl[2];
    bool busy[2] = { false, false };
    int c = 0;
    // a call of 2 x kSplitMin .. kMaxBatch matches runs as two chunks, so that
    // the two banks overlap even then (an 8-rank shard of the 512-candidate
    // loop batch is 64 candidates)
    const int step = (ctx->split_chunks && n <= kMaxBatch && n >= 2 * kSplitMin) ? (n + 1) / 2 : kMaxBatch;
    try {
        for (int j0 = 0; j0 < n; j0 += step, ++c) {
            const int m = std::min(step, n - j0);
            std::vector<PlaneSet> sets;
            std::vector<int> so((size_t)m), remap(sets_all.size(), -1);
            for (int k = 0; k < m; ++k) {
                const int s = set_of[j0 + k];
                if (remap[s] < 0) {
                    remap[s] = (int)sets.size();
                    sets.push_back(sets_all[s]);
                }
                so[k] = remap[s];
            }
            const int b = c & 1;
            ctx->bank = b;
            fl[b] = InFlight{};
            launch_matches(ctx, params, cost, grids + j0, scans + j0, init + j0, m, nthr, sets, so.data(), out + j0,
                           fl[b]);
            busy[b] = true;
            if (busy[b ^ 1]) {
                finish_matches(ctx, fl[b ^ 1]);
                busy[b ^ 1] = false;
            }
        }
        const int last = (c - 1) & 1;
        if (busy[last]) {
            finish_matches(ctx, fl[last]);
            busy[last] = false;
        }
    } catch (...) {
        ctx->bank = 0;
        throw;
    }
    ctx->bank = 0;
}

}  // namespace

namespace lgs {
// CostGreedyEndpoint::Cost at the seven poses of ComputeGradient /
// ComputeCovariance around each item's best sensor pose
// (C/mapping/cost_function_greedy_endpoint.cpp:32-171), one k_cost launch for
// all n items; then the summary fields every matcher derives from them
// (:128-138 of the RTCSM matcher, :142-153 of the branch-and-bound one):
// normalized cost, estimated pose, covariance.  Guarded cells are re-checked
// with glibc and mismatching items re-evaluated with host cells.
void cost_summaries(lgs_ctx* ctx, const lgs_grid* grid, const lgs_cost_ge_params* cost, lgs_scan* const* scans,
                    const lgs_pose2d* best, int n, lgs_rtcsm_summary* out)
{
    if (n <= 0) return;
    grid_acquire(ctx, grid);
    int Nmax = 1;
    for (int j = 0; j < n; ++j) Nmax = std::max(Nmax, scans[j]->n);
    const ItemLayout L = item_layout(1, 1, 1, 1, 1, 64, 1, Nmax);
    char* ws = (char*)ctx->ensure(S_BATCH_WS, L.total * (size_t)n);
    RtcsmRecord* d_rec = (RtcsmRecord*)ctx->ensure(S_RECORDS, sizeof(RtcsmRecord) * (size_t)n);
    RtcsmRecord* h_rec = (RtcsmRecord*)ctx->ensure_pinned(sizeof(RtcsmRecord) * (size_t)n);
    std::vector<MatchItem> items((size_t)n);
    std::vector<double> P7((size_t)n * 21);
    std::vector<int> gens((size_t)n);
    scans_to_device(ctx, scans, n);
    for (int j = 0; j < n; ++j) {
        MatchItem& it = items[j];
        std::memset(&it, 0, sizeof(it));
        bind_workspace(it, ws + L.total * (size_t)j, L, 1);
        it.cp = make_cost_plan(grid, cost, scans[j]);
        it.grid = grid->d;
        it.ranges = scans[j]->d_ranges;
        it.angles = scans[j]->d_angles;
        it.rec = d_rec + j;
        it.gen = gens[j] = ctx->generation = ctx->next_stamp();
        // the poses of ComputeGradient (:119-136), as k_replay forms them
        const double x = best[j].x, y = best[j].y, th = best[j].theta, dl = grid->res, da = 1e-2;
        const double v[21] = { x, y, th, x + dl, y + 0.0, th + 0.0, x - dl, y - 0.0, th - 0.0,
                               x + 0.0, y + dl, th + 0.0, x - 0.0, y - dl, th - 0.0,
                               x + 0.0, y + 0.0, th + da, x - 0.0, y - 0.0, th - da };
        std::memcpy(&P7[(size_t)j * 21], v, sizeof(v));
    }
    Upload up(ctx);
    const size_t poff = up.append(P7.data(), P7.size());
    const size_t ioff = up.append(items.data(), items.size());
    char* dev = up.prepare();
    for (int j = 0; j < n; ++j) up.host_at<MatchItem>(ioff)[j].poses7 = (double*)(dev + poff) + 21 * (size_t)j;
    up.copy();
    Items d_items = up.at<MatchItem>(ioff);
    const int ks = cost->kernel_size;
    hipLaunchKernelGGL(KCOST(ks), dim3(7, n), dim3(kCostThreads), cost_lds(items), ctx->stream, d_items,
                       ctx->guard_cap,
                       ctx->guard_eps, ctx->inject_index ? 1 : 0, 0, DevTs{});
    LGS_HIP_CHECK(hipGetLastError());
    LGS_HIP_CHECK(hipMemcpyAsync(h_rec, d_rec, sizeof(RtcsmRecord) * (size_t)n, hipMemcpyDeviceToHost, ctx->stream));
    ctx->sync();
    for (int j = 0; j < n; ++j) {
        HostRecord rec(h_rec[j], gens[j]);
        double p7[7][3];
        std::memcpy(p7, &P7[(size_t)j * 21], sizeof(p7));
        std::vector<int4> cpatch;
        bool full = false;
        out[j].guard_hits += rec.cost_guard_count;
        if (check_cost_guards_p7(ctx, p7, items[j].cp, scans[j], rec, cpatch, full)) {
            const CostPlan& cp = items[j].cp;
            if (full) {
                cpatch.clear();
                for (int pi = 0; pi < 7; ++pi)
                    for (int b = 0; b < cp.N; ++b) {
                        const double r = scans[j]->h_ranges[b];
                        if (r >= cp.max_range || r <= cp.min_range) continue;
                        int cells[4];
                        host_cost_cells(cp, scans[j], p7[pi], b, cells);
                        cpatch.push_back(make_int4(pi * cp.N + b, 0, 0, 0));
                        cpatch.push_back(make_int4(cells[0], cells[1], cells[2], cells[3]));
                    }
            }
            // single-item rerun reading the patched cells (mode 1)
            const int np = (int)(cpatch.size() / 2);
            int4* dp = (int4*)ctx->ensure(S_PATCH, sizeof(int4) * std::max<size_t>(cpatch.size(), 1));
            LGS_HIP_CHECK(hipMemcpyAsync(dp, cpatch.data(), sizeof(int4) * cpatch.size(), hipMemcpyHostToDevice,
                                         ctx->stream));
            if (np) hipLaunchKernelGGL(k_cost_patch, dim3((np + 255) / 256), dim3(256), 0, ctx->stream,
                                       items[j].cidx, dp, np);
            hipLaunchKernelGGL(KCOST(ks), dim3(7, 1), dim3(kCostThreads), cost_lds(items), ctx->stream, d_items + j,
                               ctx->guard_cap, ctx->guard_eps, 0, 1, DevTs{});
            LGS_HIP_CHECK(hipGetLastError());
            LGS_HIP_CHECK(hipMemcpyAsync(&h_rec[j], d_rec + j, sizeof(RtcsmRecord), hipMemcpyDeviceToHost,
                                         ctx->stream));
            ctx->sync();
            out[j].fixups = 1;
        }
        const double* c = h_rec[j].costs;
        out[j].normalized_cost = c[0] / (double)scans[j]->n;
        out[j].estimated_pose = move_backward(best[j], scans[j]->rel);
        const double dl = grid->res, da = 1e-2;
        const double g[3] = { 0.5 * (c[1] - c[2]) / dl, 0.5 * (c[3] - c[4]) / dl, 0.5 * (c[5] - c[6]) / da };
        for (int a = 0; a < 3; ++a)
            for (int b = 0; b < 3; ++b) out[j].covariance[3 * a + b] = g[a] * g[b];
        out[j].covariance[0] += 0.01;
        out[j].covariance[4] += 0.01;
        out[j].covariance[8] += 0.01;
    }
}
}  // namespace lgs

extern "C" int lgs_debug_item_buffer(lgs_ctx* ctx, int item, int which, void* out, size_t cap, size_t* bytes)
{
    if (!ctx || which < 0 || which >= 10 || item < 0) return LGS_ERR_INVALID_ARG;
    return guarded(ctx, [&] {
        LGS_REQUIRE((size_t)item < ctx->dbg.size(), "no such item in the last correlative batch");
        const lgs_ctx::DbgItem& d = ctx->dbg[(size_t)item];
        const size_t n = d.bytes[which];
        if (bytes) *bytes = n;
        if (!out || cap == 0) return;
        const size_t k = std::min(cap, n);
        LGS_HIP_CHECK(hipSetDevice(ctx->device));
        ctx->sync();
        LGS_HIP_CHECK(hipMemcpy(out, d.buf[which], k, hipMemcpyDeviceToHost));
        if (which == 4) {   // generation stamps -> flags of the item's last enqueue
            int* f = (int*)out;
            for (size_t i = 0; i < k / sizeof(int); ++i) f[i] = f[i] == d.gen ? 1 : 0;
        }
    });
}

extern "C" int lgs_rtcsm_optimize_pose(lgs_ctx* ctx, const lgs_grid* grid, const lgs_grid* coarse,
                                       const lgs_rtcsm_params* params,
                                       const lgs_cost_ge_params* cost, const lgs_scan* scan,
                                       lgs_pose2d initial, double nthr, lgs_rtcsm_summary* out)
{
    if (!ctx || !out || !grid || !coarse || !scan) return LGS_ERR_INVALID_ARG;
    return guarded(ctx, [&] {
        std::vector<PlaneSet> sets(1);
        sets[0].coarse = coarse;
        const int set0 = 0;
        lgs_scan* s = const_cast<lgs_scan*>(scan);
        run_matches(ctx, params, cost, &grid, &s, &initial, 1, nthr, sets, &set0, out);
    });
}

extern "C" int lgs_rtcsm_optimize_pose_batch(lgs_ctx* ctx, const lgs_grid* grid,
                                             const lgs_grid* coarse, const lgs_rtcsm_params* params,
                                             const lgs_cost_ge_params* cost,
                                             const lgs_scan* const* scans,
                                             const lgs_pose2d* initial, int n, double nthr,
                                             lgs_rtcsm_summary* out)
{
    if (!ctx || !out || !scans || !initial || n < 0 || !grid || !coarse) return LGS_ERR_INVALID_ARG;
    if (n == 0) return LGS_OK;
    return guarded(ctx, [&] {
        std::vector<PlaneSet> sets(1);
        sets[0].coarse = coarse;
        const std::vector<int> set_of((size_t)n, 0);
        const std::vector<const lgs_grid*> grids((size_t)n, grid);
        run_chunked(ctx, params, cost, grids.data(), const_cast<lgs_scan* const*>(scans), initial, n, nthr, sets,
                    set_of.data(), out);
    });
}

extern "C" int lgs_rtcsm_optimize_pose_query(lgs_ctx* ctx, const lgs_grid* grid,
                                             const lgs_rtcsm_params* params,
                                             const lgs_cost_ge_params* cost,
                                             const lgs_scan* scan, lgs_pose2d initial,
                                             lgs_rtcsm_summary* out)
{
    if (!ctx || !grid || !params || !out || !scan) return LGS_ERR_INVALID_ARG;
    return guarded(ctx, [&] {
        std::vector<PlaneSet> sets(1);
        sets[0].fine = grid;   // ComputeCoarserMap (:148-153) of the query's own map
        const int set0 = 0;
        lgs_scan* s = const_cast<lgs_scan*>(scan);
        run_matches(ctx, params, cost, &grid, &s, &initial, 1, DBL_MIN, sets, &set0, out);
    });
}

extern "C" int lgs_rtcsm_optimize_pose_query_batch(lgs_ctx* ctx, const lgs_grid* const* grids,
                                                   const lgs_rtcsm_params* params,
                                                   const lgs_cost_ge_params* cost,
                                                   const lgs_scan* const* scans,
                                                   const lgs_pose2d* initial, int n,
                                                   lgs_rtcsm_summary* out)
{
    if (!ctx || !grids || !params || !cost || !scans || !initial || !out || n < 0) return LGS_ERR_INVALID_ARG;
    if (n == 0) return LGS_OK;
    return guarded(ctx, [&] {
        // every query precomputes its own coarse map, as OptimizePose(query)
        // does (:31-47) -- also when two queries pass the same map
        std::vector<PlaneSet> sets((size_t)n);
        std::vector<int> set_of((size_t)n);
        for (int j = 0; j < n; ++j) {
            LGS_REQUIRE(grids[j] && scans[j], "null query");
            sets[j].fine = grids[j];
            set_of[j] = j;
        }
        run_chunked(ctx, params, cost, grids, const_cast<lgs_scan* const*>(scans), initial, n, DBL_MIN, sets,
                    set_of.data(), out);
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
        grid_acquire(ctx, grid);
        grid_acquire(ctx, coarse);
        lgs_scan* s = const_cast<lgs_scan*>(scan);
        int nv = 0;
        scan_valid_indices(ctx, s, params->scan_range_max, &nv);
        RtcsmPlan pl = make_plan(grid, params, s, initial, DBL_MIN, nv);
        const int nfx = pl.ncx * pl.low_res, nfy = pl.ncy * pl.low_res;
        if (dims) {
            dims[0] = pl.win_x; dims[1] = pl.win_y; dims[2] = pl.win_t;
            dims[3] = pl.ncx; dims[4] = pl.ncy; dims[5] = nfx; dims[6] = nfy;
        }
        if (!coarse_scores && !fine_scores) return;
        check_coarse(grid, coarse);
        const int cb = coarse_block(pl);
        const ItemLayout L = item_layout(pl.T, nv, pl.P, pl.nsbx * pl.nsby, 1, cb, 1, s->n);
        char* ws = (char*)ctx->ensure(S_BATCH_WS, L.total);
        RtcsmRecord* d_rec = (RtcsmRecord*)ctx->ensure(S_RECORDS, sizeof(RtcsmRecord));
        LGS_HIP_CHECK(hipMemsetAsync(d_rec, 0, sizeof(RtcsmRecord), ctx->stream));
        std::vector<PlaneSet> sets(1);
        sets[0].coarse = coarse;
        scan_to_device(ctx, s);
        Upload up(ctx);
        const SetJobs sj = build_sets(ctx, pl, sets, false, up);
        MatchItem it;
        std::memset(&it, 0, sizeof(it));
        it.pl = pl;
        bind_workspace(it, ws, L, 1);
        it.tedge = ctx->tedge_buffer((size_t)pl.T);
        it.grid = grid->d;
        it.ranges = s->d_ranges;
        it.angles = s->d_angles;
        it.cmap = sets[0].cmap;
        it.gen = ctx->generation = ctx->next_stamp();
        it.rec = d_rec;
        const size_t off = up.append(&it, 1);
        up.flush();
        launch_sets(ctx, pl, sets, sj, up);
        Items d_items = up.at<MatchItem>(off);
        dim3 g(std::max(1, (nv + 255) / 256), (pl.T + kProjRows - 1) / kProjRows, 1);
        hipLaunchKernelGGL(HIP_KERNEL_NAME(k_project<kProjRows>), g, dim3(256), 0, ctx->stream, d_items, 0, -1.0, 0,
                           DevTs{});
        LGS_HIP_CHECK(hipGetLastError());
        if (coarse_scores) {
            dim3 gc((pl.P + cb - 1) / cb, pl.T, 1);
            hipLaunchKernelGGL(k_coarse, gc, dim3(cb), 0, ctx->stream, d_items, ctx->zero);
            LGS_HIP_CHECK(hipGetLastError());
            LGS_HIP_CHECK(hipMemcpyAsync(coarse_scores, it.cscore, sizeof(double) * (size_t)pl.K,
                                         hipMemcpyDeviceToHost, ctx->stream));
        }
        if (fine_scores) {
            const size_t nf = (size_t)pl.T * nfx * nfy;
            double* d = (double*)ctx->ensure(S_DENSE_FINE, sizeof(double) * nf);
            dim3 gf((nfx * nfy + 255) / 256, pl.T);
            hipLaunchKernelGGL(k_fine_dense, gf, dim3(256), 0, ctx->stream, pl, grid->d, it.idx, nfx,
                               nfy, d);
            LGS_HIP_CHECK(hipGetLastError());
            LGS_HIP_CHECK(hipMemcpyAsync(fine_scores, d, sizeof(double) * nf, hipMemcpyDeviceToHost,
                                         ctx->stream));
        }
        ctx->sync();
    });
}

extern "C" int lgs_cost_greedy_endpoint(lgs_ctx* ctx, const lgs_grid* grid,
                                        const lgs_cost_ge_params* cost, const lgs_scan* scan,
                                        lgs_pose2d pose, double* out_cost)
{
    if (!ctx || !grid || !cost || !scan || !out_cost) return LGS_ERR_INVALID_ARG;
    return guarded(ctx, [&] {
        LGS_HIP_CHECK(hipSetDevice(ctx->device));
        grid_acquire(ctx, grid);
        const CostPlan cp = make_cost_plan(grid, cost, scan);
        scan_to_device(ctx, scan);
        const ItemLayout L = item_layout(1, 1, 1, 1, 1, 64, 1, scan->n);
        char* ws = (char*)ctx->ensure(S_BATCH_WS, L.total);
        RtcsmRecord* d_rec = (RtcsmRecord*)ctx->ensure(S_RECORDS, sizeof(RtcsmRecord));
        RtcsmRecord* h_rec = (RtcsmRecord*)ctx->ensure_pinned(sizeof(RtcsmRecord));
        MatchItem it;
        std::memset(&it, 0, sizeof(it));
        bind_workspace(it, ws, L, 1);
        it.cp = cp;
        it.grid = grid->d;
        it.ranges = scan->d_ranges;
        it.angles = scan->d_angles;
        it.rec = d_rec;
        const int gen = it.gen = ctx->generation = ctx->next_stamp();
        double hp[3] = { pose.x, pose.y, pose.theta };
        LGS_HIP_CHECK(hipMemcpyAsync(it.poses7, hp, sizeof(hp), hipMemcpyHostToDevice, ctx->stream));
        Upload up(ctx);
        const size_t off = up.append(&it, 1);
        up.flush();
        Items d_items = up.at<MatchItem>(off);
        hipLaunchKernelGGL(KCOST(cp.kernel_size), dim3(1, 1), dim3(kCostThreads), cost_lds(std::vector<MatchItem>{ it }),
                           ctx->stream, d_items,
                           ctx->guard_cap, ctx->guard_eps, 0, 0, DevTs{});
        LGS_HIP_CHECK(hipGetLastError());
        LGS_HIP_CHECK(hipMemcpyAsync(h_rec, d_rec, sizeof(RtcsmRecord), hipMemcpyDeviceToHost,
                                     ctx->stream));
        ctx->sync();
        if (tagged_count(h_rec->cost_guard_word, gen) > 0) {
            // exact host recomputation of every cell row, then re-evaluate
            std::vector<int4> row((size_t)cp.N, make_int4(INT_MIN, 0, 0, 0));
            for (int b = 0; b < cp.N; ++b) {
                const double r = scan->h_ranges[b];
                if (r >= cp.max_range || r <= cp.min_range) continue;
                int cells[4];
                host_cost_cells(cp, scan, hp, b, cells);
                row[b] = make_int4(cells[0], cells[1], cells[2], cells[3]);
            }
            LGS_HIP_CHECK(hipMemcpyAsync(it.cidx, row.data(), sizeof(int4) * row.size(),
                                         hipMemcpyHostToDevice, ctx->stream));
            hipLaunchKernelGGL(KCOST(cp.kernel_size), dim3(1, 1), dim3(kCostThreads), cost_lds(std::vector<MatchItem>{ it }),
                           ctx->stream, d_items,
                               ctx->guard_cap, ctx->guard_eps, 0, 1, DevTs{});
            LGS_HIP_CHECK(hipGetLastError());
            LGS_HIP_CHECK(hipMemcpyAsync(h_rec, d_rec, sizeof(RtcsmRecord), hipMemcpyDeviceToHost,
                                         ctx->stream));
            ctx->sync();
        }
        *out_cost = h_rec->costs[0];
    });
}

// LoopDetectorRealTimeCorrelative::Detect (C/mapping/loop_detector_real_time_correlative.cpp:26-92)
// with FindCorrespondingPose (:96-125): per query, the coarse map (computed here
// when the caller has none cached, :52-60), then every candidate node matched
// with OptimizePose(.., ScoreThreshold) and, when found, the loop edge
// InverseCompound(localMapNode.Pose(), estimatedPose).  One result per
// candidate, in candidate order (found == 0 where the reference appends none).
// Candidates are independent, so the queries whose local maps share a size
// are matched together in batches (each query's coarse map built once per batch).
extern "C" int lgs_loop_detect_rtcsm(lgs_ctx* ctx, const lgs_rtcsm_params* params,
                                     const lgs_cost_ge_params* cost, double score_threshold,
                                     const lgs_loop_query* queries, int num_queries,
                                     const lgs_loop_candidate* candidates, int num_candidates,
                                     lgs_loop_result* results)
{
    if (!ctx || !params || !cost || (num_queries > 0 && !queries) || num_queries < 0 ||
        num_candidates < 0 || (num_candidates > 0 && (!candidates || !results)))
        return LGS_ERR_INVALID_ARG;
    return guarded(ctx, [&] {
        LGS_REQUIRE(score_threshold > 0.0 && score_threshold <= 1.0,
                    "score threshold must be in (0, 1] (:21-22)");
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
        // group the queries by map geometry (one batch shape per group)
        std::vector<bool> done((size_t)num_queries, false);
        for (int q0 = 0; q0 < num_queries; ++q0) {
            if (done[q0]) continue;
            const lgs_grid* m0 = queries[q0].map;
            std::vector<PlaneSet> sets;
            std::vector<int> set_of, cand;
            std::vector<const lgs_grid*> grids;
            std::vector<lgs_scan*> scans;
            std::vector<lgs_pose2d> poses;
            for (int q = q0; q < num_queries; ++q) {
                const lgs_loop_query& Q = queries[q];
                if (done[q] || Q.map->w != m0->w || Q.map->h != m0->h || Q.map->res != m0->res) continue;
                done[q] = true;
                if (Q.num_candidates == 0) continue;
                PlaneSet ps;
                if (Q.coarse) ps.coarse = Q.coarse;
                else ps.fine = Q.map;
                sets.push_back(ps);
                for (int j = 0; j < Q.num_candidates; ++j) {
                    const lgs_loop_candidate& c = candidates[Q.first_candidate + j];
                    set_of.push_back((int)sets.size() - 1);
                    cand.push_back(Q.first_candidate + j);
                    grids.push_back(Q.map);
                    scans.push_back(const_cast<lgs_scan*>(c.scan));
                    poses.push_back(c.node_pose);
                }
            }
            if (cand.empty()) continue;
            std::vector<lgs_rtcsm_summary> sums(cand.size());
            run_chunked(ctx, params, cost, grids.data(), scans.data(), poses.data(), (int)cand.size(),
                        score_threshold, sets, set_of.data(), sums.data());
            for (size_t k = 0; k < cand.size(); ++k) {
                const int ci = cand[k];
                int qi = 0;
                while (!(ci >= queries[qi].first_candidate &&
                         ci < queries[qi].first_candidate + queries[qi].num_candidates))
                    ++qi;
                const lgs_loop_query& Q = queries[qi];
                lgs_loop_result& r = results[ci];
                std::memset(&r, 0, sizeof(r));
                const lgs_rtcsm_summary& s = sums[k];
                r.found = s.pose_found;
                r.start_node_index = Q.local_map_node_index;
                r.end_node_index = candidates[ci].node_index;
                r.start_node_pose = Q.local_map_node_pose;
                r.estimated_pose = s.estimated_pose;
                r.score = s.score_max;
                r.normalized_cost = s.normalized_cost;
                if (s.pose_found) r.relative_pose = inverse_compound(Q.local_map_node_pose, s.estimated_pose);
                std::memcpy(r.covariance, s.covariance, sizeof(r.covariance));
            }
        }
    });
}

namespace {

// A copy of `src` (any device) owned by ctx: peer copy over xGMI, or a plain
// device copy when both live on the same GPU.
// Peer access from ctx's device to `peer` (hipDeviceEnablePeerAccess once per
// pair and process): true when direct device-to-device copies may be used.
bool peer_access(int dev, int peer)
{
    if (dev == peer) return true;
    static std::mutex mu;
    static std::map<std::pair<int, int>, bool> known;
    std::lock_guard<std::mutex> lock(mu);
    const auto key = std::make_pair(dev, peer);
    auto it = known.find(key);
    if (it != known.end()) return it->second;
    int can = 0;
    bool ok = hipDeviceCanAccessPeer(&can, dev, peer) == hipSuccess && can;
    if (ok) {
        int cur = 0;
        hipGetDevice(&cur);
        hipSetDevice(dev);
        const hipError_t e = hipDeviceEnablePeerAccess(peer, 0);
        ok = e == hipSuccess || e == hipErrorPeerAccessAlreadyEnabled;
        (void)hipGetLastError();
        hipSetDevice(cur);
    }
    known[key] = ok;
    return ok;
}

// A copy of another context's map on ctx: device to device (one device, or
// peer access over xGMI), else -- or with LGS_OPT_PEER_COPY -- staged
// through pinned host memory.  The source's pending writer is waited for.
lgs_grid* clone_grid(lgs_ctx* ctx, const lgs_grid* src)
{
    lgs_grid* g = nullptr;
    const int rc = lgs_grid_create(ctx, src->w, src->h, src->min_x, src->min_y, src->res, &g);
    if (rc != LGS_OK) throw Error(rc, ctx->last_error);
    const size_t bytes = sizeof(double) * (size_t)src->w * (size_t)src->h;
    try {
        if (bytes) {
            if (src->writer) src->writer->wait();
            if (!ctx->peer_staged && peer_access(ctx->device, src->device)) {
                LGS_HIP_CHECK(hipMemcpyPeerAsync(g->d, ctx->device, src->d, src->device, bytes, ctx->stream));
                ctx->sync();
                ++ctx->copies_direct;
            } else {
                // one bounce buffer: device -> host on the source's device,
                // host -> device on ctx's
                void* pin = nullptr;
                LGS_HIP_CHECK(hipHostMalloc(&pin, bytes));
                hipError_t e = hipMemcpy(pin, src->d, bytes, hipMemcpyDeviceToHost);
                if (e == hipSuccess) e = hipMemcpyAsync(g->d, pin, bytes, hipMemcpyHostToDevice, ctx->stream);
                if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
                hipHostFree(pin);
                LGS_HIP_CHECK(e);
                ++ctx->copies_staged;
            }
        }
    } catch (...) {
        lgs_grid_destroy(g);
        throw;
    }
    return g;
}

lgs_scan* clone_scan(lgs_ctx* ctx, const lgs_scan* src)
{
    lgs_scan_host h{};
    h.n = src->n;
    h.ranges = src->h_ranges.data();
    h.angles = src->h_angles.data();
    h.rel_sensor_pose = src->rel;
    h.min_range = src->min_range;
    h.max_range = src->max_range;
    lgs_scan* s = nullptr;
    const int rc = lgs_scan_create(ctx, &h, &s);
    if (rc != LGS_OK) throw Error(rc, ctx->last_error);
    return s;
}

// One shard of a multi-device loop batch: candidates [lo, hi) on ctx, the
// queries clipped to that range; maps and scans are cloned onto ctx unless
// they are its own.
struct LoopShard {
    lgs_ctx* ctx = nullptr;
    int lo = 0, hi = 0;
    std::vector<lgs_loop_query> qs;
    std::vector<lgs_loop_candidate> cs;
    std::vector<lgs_grid*> grids;   // owned clones
    std::vector<lgs_scan*> scans;   // owned clones
    int status = LGS_OK;
    std::string error;

    ~LoopShard()
    {
        for (lgs_grid* g : grids) lgs_grid_destroy(g);
        for (lgs_scan* s : scans) lgs_scan_destroy(s);
    }
    const lgs_grid* own(const lgs_grid* g, std::vector<std::pair<const lgs_grid*, lgs_grid*>>& memo)
    {
        if (!g || g->ctx == ctx) return g;
        for (auto& m : memo)
            if (m.first == g) return m.second;
        grids.push_back(clone_grid(ctx, g));
        memo.push_back({ g, grids.back() });
        return grids.back();
    }
    void prepare(const lgs_loop_query* queries, int num_queries, const lgs_loop_candidate* candidates)
    {
        std::vector<std::pair<const lgs_grid*, lgs_grid*>> memo;
        for (int q = 0; q < num_queries; ++q) {
            const lgs_loop_query& Q = queries[q];
            const int a = std::max(Q.first_candidate, lo), b = std::min(Q.first_candidate + Q.num_candidates, hi);
            if (a >= b) continue;
            lgs_loop_query c = Q;
            c.map = own(Q.map, memo);
            c.coarse = own(Q.coarse, memo);
            c.first_candidate = (int)cs.size();
            c.num_candidates = b - a;
            qs.push_back(c);
            for (int i = a; i < b; ++i) {
                lgs_loop_candidate k = candidates[i];
                if (k.scan->ctx != ctx) {
                    scans.push_back(clone_scan(ctx, k.scan));
                    k.scan = scans.back();
                }
                cs.push_back(k);
            }
        }
    }
};

}  // namespace

extern "C" int lgs_loop_detect_rtcsm_multi(lgs_ctx* const* ctxs, int num_ctx, const lgs_rtcsm_params* params,
                                           const lgs_cost_ge_params* cost, double score_threshold,
                                           const lgs_loop_query* queries, int num_queries,
                                           const lgs_loop_candidate* candidates, int num_candidates,
                                           lgs_loop_result* results)
{
    if (!ctxs || num_ctx < 1 || !ctxs[0]) return LGS_ERR_INVALID_ARG;
    for (int k = 1; k < num_ctx; ++k)
        if (!ctxs[k]) return LGS_ERR_INVALID_ARG;
    lgs_ctx* const c0 = ctxs[0];
    if (num_ctx == 1 || num_candidates <= 1)
        return lgs_loop_detect_rtcsm(c0, params, cost, score_threshold, queries, num_queries, candidates,
                                     num_candidates, results);
    if (!params || !cost || (num_queries > 0 && !queries) || num_queries < 0 || num_candidates < 0 ||
        (num_candidates > 0 && (!candidates || !results)))
        return LGS_ERR_INVALID_ARG;
    return guarded(c0, [&] {
        // the single-context contract first, so a bad batch fails the same way
        // whatever the shard boundaries (:21-22, queries covering the candidates)
        LGS_REQUIRE(score_threshold > 0.0 && score_threshold <= 1.0, "score threshold must be in (0, 1] (:21-22)");
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
        const int N = std::min(num_ctx, num_candidates);
        std::vector<LoopShard> shards((size_t)N);
        for (int k = 0; k < N; ++k) {   // contiguous shards, as the gloo/RCCL path
            shards[k].ctx = ctxs[k];
            shards[k].lo = (int)((long long)num_candidates * k / N);
            shards[k].hi = (int)((long long)num_candidates * (k + 1) / N);
        }
        auto work = [&](LoopShard& sh) {
            try {
                if (hipSetDevice(sh.ctx->device) != hipSuccess) throw Error(LGS_ERR_HIP, "hipSetDevice failed");
                sh.prepare(queries, num_queries, candidates);
                sh.status = lgs_loop_detect_rtcsm(sh.ctx, params, cost, score_threshold, sh.qs.data(),
                                                  (int)sh.qs.size(), sh.cs.data(), (int)sh.cs.size(),
                                                  results + sh.lo);
                if (sh.status != LGS_OK) sh.error = sh.ctx->last_error;
            } catch (const Error& e) {
                sh.status = e.code;
                sh.error = e.what();
            } catch (const std::exception& e) {
                sh.status = LGS_ERR_INTERNAL;
                sh.error = e.what();
            }
        };
        std::vector<std::thread> threads;
        for (int k = 1; k < N; ++k) threads.emplace_back(work, std::ref(shards[k]));
        work(shards[0]);
        for (auto& t : threads) t.join();
        LGS_HIP_CHECK(hipSetDevice(c0->device));
        for (int k = 0; k < N; ++k)
            if (shards[k].status != LGS_OK)
                throw Error(shards[k].status, "shard " + std::to_string(k) + " (device " +
                                                  std::to_string(shards[k].ctx->device) + "): " + shards[k].error);
        // a result's start_node_index etc. come from its query, which each
        // shard saw clipped but unchanged: nothing to remap
    });
}

extern "C" int lgs_debug_offset_checks(lgs_ctx* ctx, int reset, unsigned long long* out)
{
    if (!ctx || !out) return LGS_ERR_INVALID_ARG;
#ifdef LGS_CHECK_OFFSETS
    return guarded(ctx, [&] {
        LGS_HIP_CHECK(hipSetDevice(ctx->device));
        LGS_HIP_CHECK(hipStreamSynchronize(ctx->stream));
        LGS_HIP_CHECK(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_offchk), sizeof(unsigned long long) * 4));
        if (reset) {
            const unsigned long long z[4] = { 0, 0, 0, 0 };
            LGS_HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_offchk), z, sizeof(z)));
        }
    });
#else
    (void)reset;
    return LGS_ERR_INVALID_ARG;   // product build: no checks compiled in
#endif
}

extern "C" int lgs_debug_copy_counters(const lgs_ctx* ctx, long long* direct, long long* staged)
{
    if (!ctx || !direct || !staged) return LGS_ERR_INVALID_ARG;
    *direct = ctx->copies_direct;
    *staged = ctx->copies_staged;
    return LGS_OK;
}
