// k_raycast.hip -- K3: Bresenham ray-cast + binary Bayes occupancy update on MI355X,
// and the reference's GridMap geometry (patches, Resize/Expand) around it.
//
// Restates GridMapBuilder's integration loop (C/mapping/grid_map_builder.cpp:167-186
// and :292-329): per beam, the cells of Bresenham(sensorCell, hitCell) minus the
// last are updated with pMiss, then the hit cell with pHit
// (BinaryBayesGridCell::Update, H/grid_map/binary_bayes_grid_cell.hpp:75-119).
// The update is order-dependent (clamped odds products), so the device keeps the
// reference's order exactly:
//
//   host       hit points with glibc sin/cos (bit-exact), bounding box, map
//              geometry (Expand/Resize), sensor/hit cells, ray lengths + offsets
//   k_emit     one wave per ray computes its Bresenham cells (H/util.hpp:256-303) and emits
//              a 32-bit key (cell << 1 | is_hit) per visited cell at the ray's
//              offset, so the key array is in ray order
//   sort       stable radix sort on the cell bits only (k_sort.hip): each
//              cell's updates become a contiguous run that keeps ray order =
//              the reference's update order (a ray visits a cell at most once)
//   k_runmask  hit and run-end bitmaps of the sorted keys (one ballot per 64)
//   k_apply    one thread per run applies the Bayes updates sequentially and
//              counts hits/misses
#include "lgs_internal.hpp"

#include <atomic>
#include "glibc_math.hpp"

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <unordered_map>

#include <algorithm>
#include <array>
#include <cfloat>
#include <climits>
#include <cstring>

using namespace lgs;

namespace {
struct LatestCache;
}

struct lgs_map {
    lgs_ctx* ctx = nullptr;
    int device = 0;
    double res = 0;
    int ps = 0;
    int npx = 0, npy = 0;
    int w = 0, h = 0;
    double min_x = 0, min_y = 0;
    double* d_cells = nullptr;
    uint32_t* d_hit = nullptr;
    uint32_t* d_miss = nullptr;
    size_t cap = 0;  // cells allocated (>= w*h; construct reuses a large enough allocation)
    // Patch::IsAllocated per patch (npx*npy bytes, H/grid_map/grid_map_patch.hpp:40):
    // set by k_apply for every patch a ray updates (GridCellAt allocates,
    // H/grid_map/grid_map.hpp:807-823), moved by Resize (:676-697), kept by
    // Reset (grid_map_patch.hpp:194-203).  d_palloc2 is the spare of a remap.
    uint8_t* d_palloc = nullptr;
    uint8_t* d_palloc2 = nullptr;
    size_t pcap = 0, pcap2 = 0;
    lgs_grid view;
    LatestCache* cache = nullptr;   // the latest map's window lists (§4.4b), created on first use
};

namespace {

constexpr double kPMin = 1e-3;
constexpr double kPMax = 1.0 - kPMin;

__host__ __device__ __forceinline__ double clampv(double v, double lo, double hi)
{
    return (v < lo) ? lo : (hi < v) ? hi : v;  // std::clamp
}

// BinaryBayesGridCell::Update (H/grid_map/binary_bayes_grid_cell.hpp:75-119)
__host__ __device__ __forceinline__ double bayes_update(double v, double p)
{
    if (v == 0.0) return clampv(p, kPMin, kPMax);
    const double co = clampv(v, kPMin, kPMax);
    const double cp = clampv(p, kPMin, kPMax);
    const double o = (co / (1.0 - co)) * (cp / (1.0 - cp));
    return clampv(clampv(o / (1.0 + o), kPMin, kPMax), kPMin, kPMax);
}

// The same operations with clamp(p) and odds(clamp(p)) evaluated once by the
// caller (identical values: the reference recomputes the same constant).
__device__ __forceinline__ double bayes_update_k(double v, double cp, double op)
{
    if (v == 0.0) return cp;
    const double co = clampv(v, kPMin, kPMax);
    const double o = (co / (1.0 - co)) * op;
    return clampv(clampv(o / (1.0 + o), kPMin, kPMax), kPMin, kPMax);
}

// One map of a ray-cast pass.  Several maps (AfterLoopClosure's local maps)
// share one emit/sort/apply pass: map j owns the global cell range
// [base, base + w*h) of the 31-bit cell space of the keys.
struct RayMap {
    unsigned long long base;
    int w, h;
    double* cells;
    uint32_t* hit;
    uint32_t* miss;
    uint8_t* palloc;   // patch allocation flags (lgs_map::d_palloc)
    int ps, npx;
};

// One wave per ray: the ray's Bresenham cells (H/util.hpp:256-303, start cell
// inclusive, the hit cell last) in closed form, so the 64 lanes write 64
// consecutive keys of the ray (coalesced) instead of one lane walking it.
// With major axis M (|dM| >= |dm|, ties go to y as in the reference's else
// branch), doubled deltas DM = 2|dM|, Dm = 2|dm| and err0 = Dm - DM/2, the
// reference's loop emits at iteration k (k = 0 .. |dM| - 1) the cell
// (M0 + k sM, m0 + j_k sm) where j_k counts the minor steps taken before it:
// j_0 = 0 and j_k = floor((err0 + (k - 1) Dm) / DM) + 1 (its err stays in
// [-DM, Dm), and err_k - Dm lies in [-DM, 0) after every iteration); the
// hit cell (key k = |dM|) follows.  rmap[r] = map index | slot tag << 16.
__global__ __launch_bounds__(256) void k_emit(const int4* __restrict__ rays,
                                              const long long* __restrict__ offs,
                                              const int* __restrict__ rmap, int nrays,
                                              const RayMap* __restrict__ maps,
                                              unsigned* __restrict__ keys,
                                              int* __restrict__ outside, int ksh)
{
    const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (r >= nrays) return;
    const int4 ry = rays[r];
    const int rm = rmap ? rmap[r] : 0;
    const RayMap mp = maps[rm & 0xffff];
    const unsigned tag = ((unsigned)rm >> 16) << 1;
    const unsigned W = (unsigned)mp.w, H = (unsigned)mp.h;
    const unsigned cbase = (unsigned)mp.base;
    const int dx = ry.z - ry.x, dy = ry.w - ry.y;
    const bool xmaj = 2 * abs(dx) > 2 * abs(dy);
    const int sM = xmaj ? ((dx < 0) ? -1 : 1) : ((dy < 0) ? -1 : 1);
    const int sm = xmaj ? ((dy < 0) ? -1 : 1) : ((dx < 0) ? -1 : 1);
    const long long DM = 2LL * (xmaj ? abs(dx) : abs(dy)), Dm = 2LL * (xmaj ? abs(dy) : abs(dx));
    const long long err0 = Dm - DM / 2;
    const int L = (int)(DM / 2);               // cells before the hit cell
    unsigned* out = keys + offs[r];
    const bool small = err0 + (long long)L * Dm < (1LL << 31);   // 32-bit division suffices (uniform)
    int bad = 0;
#pragma nounroll
    for (int k = lane; k <= L; k += 64) {
        int x, y;
        unsigned hit = 0u;
        if (k == L) {
            x = ry.z, y = ry.w, hit = 1u;
        } else {
            const long long num = err0 + (long long)(k - 1) * Dm;
            long long j = 0;
            if (k > 0 && num >= 0)
                j = (small ? (long long)((unsigned)num / (unsigned)DM) : num / DM) + 1;
            const int M = k * sM, m = (int)j * sm;
            x = ry.x + (xmaj ? M : m);
            y = ry.y + (xmaj ? m : M);
        }
        const bool in = (unsigned)x < W && (unsigned)y < H;
        bad |= !in;
        const unsigned cell = cbase + (in ? (unsigned)y * W + (unsigned)x : 0u);
        out[k] = (cell << ksh) | tag | hit;
    }
    if (bad) *outside = 1;
}

// ---------------------------------------------------------------------------
// Device hit points and ray cells (r05; the map rebuilds of many scans --
// AfterLoopClosure, ConstructGlobalMap): ComputeBoundingBoxAndScanPoints'
// hit points (C/mapping/grid_map_builder.cpp:335-380) with glibc's sincos
// restated bit for bit (glibc_math.hpp gl_sincos), the boxes back to the host
// for the maps' geometry (Resize), then the sensor / hit cells
// (WorldCoordinateToGridCellIndex, H/grid_map/grid_map.hpp:779-790: a floor of
// the IEEE quotient, as on the host), the ray lengths and key offsets -- the
// host computed all of that (and staged 12 MB) in r04.
struct HitUnit {              // one (map, scan) of the pass
    const double* ranges;
    const double* angles;
    int n;                    // beams
    int job;                  // map of the pass
    double sx, sy, st;        // sensor pose (Compound on the host, glibc sincos)
    double min_r, max_r;      // usable range (open interval)
    long long beam0;          // the unit's region of the hit buffer (n slots)
};
struct MapGeo {
    double min_x, min_y, res;
};
__device__ __forceinline__ double dmin_ref(double a, double b) { return (b < a) ? b : a; }  // std::min
__device__ __forceinline__ double dmax_ref(double a, double b) { return (a < b) ? b : a; }  // std::max

// Block-wide exclusive prefix of v over the 256 threads; returns it, *total = sum.
template <class T>
__device__ __forceinline__ T block_excl_scan(T v, T* sw, T* total)
{
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    T x = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const T u = __shfl_up(x, off, 64);
        if (lane >= off) x += u;
    }
    if (lane == 63) sw[w] = x;
    __syncthreads();
    T base = 0, tot = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        if (i < w) base += sw[i];
        tot += sw[i];
    }
    __syncthreads();
    *total = tot;
    return base + x - v;
}

// k_hits: one workgroup per unit: the usable beams' hit points, compacted in
// beam order into the unit's region; the unit's count and box (sensor and
// hits: min x, min y, max x, max y, with std::min / std::max).  bad |= 4 if
// an angle lies outside gl_sincos's domain (the host path then runs).
__global__ __launch_bounds__(256) void k_hits(const HitUnit* __restrict__ units, double2* __restrict__ hits,
                                              int* __restrict__ counts, double4* __restrict__ boxes,
                                              int* __restrict__ bad)
{
    const HitUnit U = units[blockIdx.x];
    __shared__ int sw[4];
    __shared__ double sb[4][256];
    double b0 = U.sx, b1 = U.sy, b2 = U.sx, b3 = U.sy;
    int base = 0, oob = 0;
    for (int i0 = 0; i0 < U.n; i0 += 256) {
        const int i = i0 + (int)threadIdx.x;
        double r = 0.0, a = 0.0;
        if (i < U.n) {
            r = U.ranges[i];
            a = U.angles[i];
        }
        const bool ok = i < U.n && !(r >= U.max_r || r <= U.min_r);
        int tot = 0;
        const int pos = base + block_excl_scan<int>(ok ? 1 : 0, sw, &tot);
        if (ok) {
            const double th = U.st + a;
            double sn = 0.0, c = 0.0;
            if (glm::gl_sincos_ok(th)) glm::gl_sincos(th, &sn, &c);
            else oob = 1;
            const double hx = U.sx + r * c, hy = U.sy + r * sn;
            hits[U.beam0 + pos] = make_double2(hx, hy);
            b0 = dmin_ref(b0, hx);
            b1 = dmin_ref(b1, hy);
            b2 = dmax_ref(b2, hx);
            b3 = dmax_ref(b3, hy);
        }
        base += tot;
    }
    if (oob) *bad |= 4;
    sb[0][threadIdx.x] = b0;
    sb[1][threadIdx.x] = b1;
    sb[2][threadIdx.x] = b2;
    sb[3][threadIdx.x] = b3;
    __syncthreads();
    for (int h = 128; h > 0; h >>= 1) {   // min / max are exact: any order
        if ((int)threadIdx.x < h) {
            const int t = threadIdx.x;
            sb[0][t] = dmin_ref(sb[0][t], sb[0][t + h]);
            sb[1][t] = dmin_ref(sb[1][t], sb[1][t + h]);
            sb[2][t] = dmax_ref(sb[2][t], sb[2][t + h]);
            sb[3][t] = dmax_ref(sb[3][t], sb[3][t + h]);
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        counts[blockIdx.x] = base;
        boxes[blockIdx.x] = make_double4(sb[0][0], sb[1][0], sb[2][0], sb[3][0]);
    }
}

// k_raycells: one workgroup per unit: sensor and hit cells of its rays at
// [ray0[u], ray0[u] + counts[u]) of the pass, the ray -> map index, and the
// keys' offsets inside the unit (ray lengths max(|dx|, |dy|) + 1, prefix in
// ray order); ukeys[u] = the unit's keys.
__global__ __launch_bounds__(256) void k_raycells(const HitUnit* __restrict__ units, const double2* __restrict__ hits,
                                                  const int* __restrict__ counts, const MapGeo* __restrict__ geo,
                                                  const int* __restrict__ ray0, int4* __restrict__ rays,
                                                  long long* __restrict__ offs, int* __restrict__ rmap,
                                                  long long* __restrict__ ukeys)
{
    const int u = blockIdx.x;
    const HitUnit U = units[u];
    const MapGeo G = geo[U.job];
    const int n = counts[u], r0 = ray0[u];
    __shared__ long long sw[4];
    const int sx = (int)floor((U.sx - G.min_x) / G.res), sy = (int)floor((U.sy - G.min_y) / G.res);
    long long base = 0;
    for (int j0 = 0; j0 < n; j0 += 256) {
        const int j = j0 + (int)threadIdx.x;
        long long len = 0;
        int4 ry = make_int4(0, 0, 0, 0);
        if (j < n) {
            const double2 h = hits[U.beam0 + j];
            const int hx = (int)floor((h.x - G.min_x) / G.res), hy = (int)floor((h.y - G.min_y) / G.res);
            ry = make_int4(sx, sy, hx, hy);
            len = (long long)max(abs(hx - sx), abs(hy - sy)) + 1;
        }
        long long tot = 0;
        const long long pos = base + block_excl_scan<long long>(len, sw, &tot);
        if (j < n) {
            rays[r0 + j] = ry;
            offs[r0 + j] = pos;
            if (rmap) rmap[r0 + j] = U.job;
        }
        base += tot;
    }
    if (threadIdx.x == 0) ukeys[u] = base;
}

// The units' key bases (exclusive prefix over units, one workgroup; n small)
// and the total (*total); then k_addbase moves every ray's offset by its
// unit's base.
__global__ __launch_bounds__(256) void k_unit_scan(const long long* __restrict__ ukeys, int nu,
                                                   long long* __restrict__ kbase, long long* __restrict__ total)
{
    __shared__ long long sw[4];
    long long base = 0;
    for (int i0 = 0; i0 < nu; i0 += 256) {
        const int i = i0 + (int)threadIdx.x;
        const long long v = i < nu ? ukeys[i] : 0;
        long long tot = 0;
        const long long pos = base + block_excl_scan<long long>(v, sw, &tot);
        if (i < nu) kbase[i] = pos;
        base += tot;
    }
    if (threadIdx.x == 0) *total = base;
}
__global__ __launch_bounds__(256) void k_addbase(const int* __restrict__ counts, const int* __restrict__ ray0,
                                                 const long long* __restrict__ kbase, long long* __restrict__ offs)
{
    const int u = blockIdx.x;
    const long long b = kbase[u];
    const int r0 = ray0[u], n = counts[u];
    for (int j = threadIdx.x; j < n; j += 256) offs[r0 + j] += b;
}

// k_runmask: one thread per sorted key; each wavefront covers 64 consecutive
// keys (64-aligned) and writes two 64-bit words with ballots -- bit j of
// hitw = key j is a hit, bit j of endw = key j is the last of its run (keys
// equal above bit rsh: rsh = ksh, runs of one cell; rsh = 1, runs of one
// (cell, slot) pair in the latest map's slot lists).  With an index table,
// the key at the start of each run below `nidx` also records the run:
// tbl[cell * kSlots + slot] = stamp(slot) << 32 | entry, where the entry of a
// run of at most kShortRun keys inside this wave's 64 keys is the run itself
// (length << 26 | hit bits, bit j = update j is a hit), and any other run's
// is kLongRun | its position (walked through the bitmaps).
constexpr int kSlots = 16;          // latest-map scan slots (slot tag: key bits 1..4)
constexpr int kTagShift = 5;        // tagged keys: cell << 5 | slot << 1 | hit
constexpr int kShortRun = 26;       // runs stored inline in the index
constexpr unsigned kLongRun = 0x80000000u;
struct SlotStamps {
    unsigned s[kSlots];
};
struct RunIndex {
    unsigned long long* tbl;        // null: no index
    long long nidx;
    SlotStamps st;
    unsigned* clear;                // non-null: a word zeroed by thread 0 (the long-cell queue count)
};
__global__ __launch_bounds__(256) void k_runmask(const unsigned* __restrict__ keys, long long n, int rsh,
                                                 unsigned long long* __restrict__ hitw,
                                                 unsigned long long* __restrict__ endw, RunIndex ix)
{
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (ix.clear && i == 0) *ix.clear = 0u;
    const bool in = i < n;
    const unsigned k = in ? keys[i] : 0u;
    const bool last = in && (i + 1 >= n || (keys[i + 1] >> rsh) != (k >> rsh));
    const unsigned long long hb = __ballot(in && (k & 1u));
    const unsigned long long eb = __ballot(last);
    if ((threadIdx.x & 63) == 0 && in) {
        hitw[i >> 6] = hb;
        endw[i >> 6] = eb;
    }
    if (ix.tbl && i < ix.nidx && (i == 0 || (keys[i - 1] >> rsh) != (k >> rsh))) {
        const unsigned slot = (k >> 1) & (kSlots - 1);
        const int lane = (int)(i & 63);
        const unsigned long long rest = eb >> lane;   // run ends at the first set bit
        int len = rest ? __ffsll((long long)rest) : 0;
        unsigned bits = len ? (unsigned)((hb >> lane) & ((len >= 64) ? ~0ull : ((1ull << len) - 1ull))) : 0u;
        if (!len && 64 - lane < kShortRun) {
            // the run continues past this wave's keys: read on up to kShortRun keys
            len = 64 - lane;
            bits = (unsigned)(hb >> lane);
            while (len <= kShortRun && i + len < n && (keys[i + len] >> rsh) == (k >> rsh)) {
                bits |= (keys[i + len] & 1u) << len;
                ++len;
            }
        }
        const unsigned entry = (len >= 1 && len <= kShortRun) ? ((unsigned)len << 26) | bits : kLongRun | (unsigned)i;
        ix.tbl[(size_t)(k >> kTagShift) * kSlots + slot] = ((unsigned long long)ix.st.s[slot] << 32) | entry;
    }
}

// Summaries of the words, one bit per word (64 words = 4096 keys per
// summary word): the word holds a hit (hit2), a miss (miss2), a run end
// (end2).  k_apply jumps over whole words of identity updates with them.
__global__ __launch_bounds__(256) void k_runsummary(const unsigned long long* __restrict__ hitw,
                                                    const unsigned long long* __restrict__ endw, long long nw,
                                                    unsigned long long* __restrict__ hit2,
                                                    unsigned long long* __restrict__ miss2,
                                                    unsigned long long* __restrict__ end2)
{
    const long long w = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    const bool in = w < nw;
    const unsigned long long hw = in ? hitw[w] : 0ull, ew = in ? endw[w] : 0ull;
    const unsigned long long h2 = __ballot(in && hw != 0ull);
    const unsigned long long m2 = __ballot(in && ~hw != 0ull);
    const unsigned long long e2 = __ballot(in && ew != 0ull);
    if ((threadIdx.x & 63) == 0 && in) {
        hit2[w >> 6] = h2;
        miss2[w >> 6] = m2;
        end2[w >> 6] = e2;
    }
}

// Number of runs (set bits of endw) -- for the algorithmic bytes of a timed
// pass only, launched outside the timed span.
__global__ __launch_bounds__(256) void k_count_runs(const unsigned long long* __restrict__ endw, long long nw,
                                                    unsigned long long* __restrict__ runs)
{
    __shared__ unsigned long long part[4];
    unsigned long long c = 0;
    for (long long w = (long long)blockIdx.x * blockDim.x + threadIdx.x; w < nw; w += (long long)gridDim.x * blockDim.x)
        c += __popcll(endw[w]);
    for (int o = 32; o > 0; o >>= 1) c += __shfl_down(c, o);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) atomicAdd(runs, part[0] + part[1] + part[2] + part[3]);
}

__device__ __forceinline__ int find_map(const RayMap* __restrict__ maps, int nmaps, unsigned cell)
{
    int lo = 0, hi = nmaps - 1;  // last j with base <= cell
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (maps[mid].base <= cell) lo = mid; else hi = mid - 1;
    }
    return lo;
}

// Update chains (memoised Bayes updates).  Chain c starts at anchor a[c] and
// applies one update type (type[c]: 0 miss, 1 hit) repeatedly: t[c][j] is the
// value after j such updates, up to a fixed point (fixed[c]) or kChain
// entries.  The anchors are the values where long same-type stretches start:
// clamp(pMiss) and clamp(pHit) (first update of a fresh cell), Update(1e-3,
// pHit) and Update(1 - 1e-3, pMiss) (leaving a saturated value).  Built on the
// host with the same IEEE operations as bayes_update (the parity tests compare
// every cell bit for bit with the CPU restatement).
constexpr int kChain = 64;
struct BayesChains {
    double a[4];
    double t[4][kChain];
    int len[4];
    int fixed[4];
};

BayesChains make_chains(double p_hit, double p_miss)
{
    BayesChains c{};
    const double anchor[4] = { clampv(p_miss, kPMin, kPMax), clampv(p_hit, kPMin, kPMax),
                               bayes_update(kPMin, p_hit), bayes_update(kPMax, p_miss) };
    const double p[4] = { p_miss, p_hit, p_miss, p_hit };  // chain types: miss, hit, miss, hit
    for (int k = 0; k < 4; ++k) {
        c.a[k] = anchor[k];
        double v = anchor[k];
        c.t[k][0] = v;
        int j = 1;
        c.fixed[k] = 0;
        for (; j < kChain; ++j) {
            const double nv = bayes_update(v, p[k]);
            if (nv == v) {
                c.fixed[k] = 1;
                break;
            }
            c.t[k][j] = v = nv;
        }
        c.len[k] = j;
    }
    return c;
}

// The run bitmaps of one sorted key array (k_runmask / k_runsummary).
struct RunBits {
    const unsigned long long *hitw, *endw, *hit2, *miss2, *end2;
    long long nw;   // words of hitw / endw
};

// Constants of the Bayes walk, evaluated once per thread.
struct BayesK {
    bool miss_fixed, hit_fixed;
    double cph, cpm, oph, opm;
    __device__ BayesK(double p_hit, double p_miss)
    {
        miss_fixed = bayes_update(kPMin, p_miss) == kPMin;
        hit_fixed = bayes_update(kPMax, p_hit) == kPMax;
        cph = clampv(p_hit, kPMin, kPMax), cpm = clampv(p_miss, kPMin, kPMax);
        oph = cph / (1.0 - cph), opm = cpm / (1.0 - cpm);
    }
};

// Where v sits on the memoised chains (-1: on none) and its index there.
struct ChainState {
    int cm, jm, ck, jk;
    __device__ ChainState(double v, const BayesChains* __restrict__ ch)
    {
        cm = (v == ch->a[0]) ? 0 : (v == ch->a[2]) ? 2 : -1;
        ck = (v == ch->a[1]) ? 1 : (v == ch->a[3]) ? 3 : -1;
        jm = jk = 0;
    }
};

// cnt updates in order (bit j of h: update j is a hit, of m: a miss) applied
// to v: same-type stretches jump along the chains, identity updates are
// skipped; every other update is BinaryBayesGridCell::Update itself.
__device__ __forceinline__ double apply_word(double v, ChainState& s, unsigned long long h, unsigned long long m,
                                             int cnt, const BayesChains* __restrict__ ch, const BayesK& K)
{
    const double a0 = ch->a[0], a1 = ch->a[1], a2 = ch->a[2], a3 = ch->a[3];
    int pos = 0;
    while (pos < cnt) {
        if (K.miss_fixed && v == kPMin) {        // misses are identities: next hit
            const unsigned long long rest = h >> pos;
            if (!rest) break;
            pos += __ffsll((long long)rest) - 1;
        } else if (K.hit_fixed && v == kPMax) {  // hits are identities: next miss
            const unsigned long long rest = m >> pos;
            if (!rest) break;
            pos += __ffsll((long long)rest) - 1;
        }
        const bool is_hit = (h >> pos) & 1ull;
        const int c = is_hit ? s.ck : s.cm;
        if (c >= 0) {
            // k same-type updates from pos: jump along the chain
            const unsigned long long other = (is_hit ? m : h) >> pos;
            const int k = other ? __ffsll((long long)other) - 1 : cnt - pos;
            const int last = ch->len[c] - 1;
            const int j0 = is_hit ? s.jk : s.jm;
            int j = j0 + k, used = k;
            if (j > last) {
                if (!ch->fixed[c]) used = last - j0;  // table ends: the rest normally
                j = last;
            }
            v = ch->t[c][j];
            pos += used;
            if (is_hit) {
                s.jk = j;
                if (used < k) s.ck = -1;
                s.cm = (v == a0) ? 0 : (v == a2) ? 2 : -1, s.jm = 0;
            } else {
                s.jm = j;
                if (used < k) s.cm = -1;
                s.ck = (v == a1) ? 1 : (v == a3) ? 3 : -1, s.jk = 0;
            }
            continue;
        }
        v = bayes_update_k(v, is_hit ? K.cph : K.cpm, is_hit ? K.oph : K.opm);
        ++pos;
        s.cm = (v == a0) ? 0 : (v == a2) ? 2 : -1, s.jm = 0;
        s.ck = (v == a1) ? 1 : (v == a3) ? 3 : -1, s.jk = 0;
    }
    return v;
}

// Apply BinaryBayesGridCell::Update for the run that starts at key position i
// (in key order = the reference's order) to the value v; counts hits/misses.
// The run is read 64 keys at a time from the hit/end words, not key by key,
// and the updates that are exact fixed points -- a miss at v == 1e-3 with
// odds(pMiss) <= 1, a hit at v == 1 - 1e-3 -- are jumped over with the masks
// after the kernel has checked on the device that they are identities (cells
// next to the sensor see thousands of such misses).
__device__ double walk_run(long long i, double v, uint32_t& nh, uint32_t& nm, const RunBits& rb,
                           const BayesChains* __restrict__ ch, const BayesK& K)
{
    ChainState cs(v, ch);
    for (long long p = i;;) {
        const int sh = (int)(p & 63);
        const bool id_miss = K.miss_fixed && v == kPMin, id_hit = K.hit_fixed && v == kPMax;
        if (sh == 0 && (id_miss || id_hit)) {
            // whole words inside the run whose updates are all identities:
            // no run end and no hit (resp. miss) in them
            const long long w = p >> 6;
            const int b = (int)(w & 63);
            const unsigned long long stop =
                (rb.end2[w >> 6] | (id_miss ? rb.hit2[w >> 6] : rb.miss2[w >> 6])) >> b;
            const int k = stop ? __ffsll((long long)stop) - 1 : 64 - b;
            if (k > 0) {
                if (id_miss) nm += 64u * (unsigned)k; else nh += 64u * (unsigned)k;
                p += 64LL * k;
                continue;
            }
        }
        const unsigned long long hm = rb.hitw[p >> 6] >> sh;
        const unsigned long long em = rb.endw[p >> 6] >> sh;
        const int cnt = em ? __ffsll((long long)em) : 64 - sh;  // keys of the run in this word
        const unsigned long long inm = (cnt == 64) ? ~0ull : ((1ull << cnt) - 1ull);
        const unsigned long long h = hm & inm;
        nh += __popcll(h);
        nm += cnt - __popcll(h);
        v = apply_word(v, cs, h, inm & ~hm, cnt, ch, K);
        if (em) return v;
        p += cnt;
    }
}

__device__ __forceinline__ bool run_start(const unsigned long long* __restrict__ endw, long long i)
{
    return i == 0 || ((endw[(i - 1) >> 6] >> ((i - 1) & 63)) & 1ull);
}

// the first Update of a cell allocates its patch (GridCellAt, :817-819);
// every thread of the patch stores the same byte
// (the flag is sticky: a thread that reads it set stores nothing -- thousands
// of cells of a patch would otherwise store to one byte, serialised at L2)
__device__ __forceinline__ void mark_patch(const RayMap& mp, unsigned long long local)
{
    const unsigned lx = (unsigned)(local % (unsigned)mp.w), ly = (unsigned)(local / (unsigned)mp.w);
    uint8_t* f = mp.palloc + (ly / (unsigned)mp.ps) * (unsigned)mp.npx + lx / (unsigned)mp.ps;
    if (!*f) *f = 1;
}

// k_apply: one thread per run of equal cells (the thread at the run's first
// key) continues the cell from its current value with the run's updates.
// The pass's maps (up to kApplyMapsLds) are staged in LDS first: the map of a
// run is then a binary search in LDS instead of a chain of dependent global
// loads on every run's critical path (the kernel is latency-bound).
constexpr int kApplyMapsLds = 64;
__global__ __launch_bounds__(256) void k_apply(const unsigned* __restrict__ keys, long long n, RunBits rb,
                                               const RayMap* __restrict__ maps, int nmaps,
                                               const BayesChains* __restrict__ ch, double p_hit, double p_miss,
                                               int ksh)
{
    __shared__ RayMap s_maps[kApplyMapsLds];
    const bool lds = nmaps <= kApplyMapsLds;
    if (lds) {
        static_assert(sizeof(RayMap) % 8 == 0, "RayMap copied as 8-byte words");
        constexpr int kw = (int)(sizeof(RayMap) / 8);
        const unsigned long long* src = (const unsigned long long*)maps;
        unsigned long long* dst = (unsigned long long*)s_maps;
        for (int k = threadIdx.x; k < nmaps * kw; k += blockDim.x) dst[k] = src[k];
        __syncthreads();
    }
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n || !run_start(rb.endw, i)) return;
    const unsigned cell = keys[i] >> ksh;
    const BayesK K(p_hit, p_miss);
    const RayMap mp = lds ? s_maps[find_map(s_maps, nmaps, cell)] : maps[find_map(maps, nmaps, cell)];
    const unsigned long long local = cell - mp.base;
    mark_patch(mp, local);
    uint32_t nh = 0, nm = 0;
    const double v = walk_run(i, mp.cells[local], nh, nm, rb, ch, K);
    mp.cells[local] = v;
    mp.hit[local] += nh;
    mp.miss[local] += nm;
}

// One step of the latest map's incremental rebuild: the
// window's scans keep their sorted key lists (one per ring slot, tagged keys,
// runs of one (cell, slot)); tbl[cell * kSlots + slot] locates a cell's run
// in a slot's list.  A cell touched by the entering scan E or the leaving
// scan L is recomputed from Unknown over the window's slots oldest first --
// the exact update sequence ConstructMapFromScans applies after Reset; every
// other cell's sequence, and so its value and counters, is unchanged.
struct SlotView {
    const unsigned* keys;
    RunBits rb;
};
struct WindowJob {
    SlotView slot[kSlots];
    SlotStamps st;
    int order[kSlots];              // the window's ring slots, oldest first
    int nwin;
    int eslot;                      // E's slot
    RayMap latest, local;           // latest map (cell base 0), local map (insert of E)
    long long nE, nloc;             // E's latest keys [0, nE), local keys [nE, nE + nloc) of slot[eslot]
    int lshift, ldx, ldy;           // lshift: E's local cells are its latest cells + (ldx, ldy), so the
                                    // local insert walks E's latest runs (nloc = nE, nothing emitted twice)
    const unsigned* lkeys;          // L's list: [lbeg, lbeg + nL) of lrb's array (nL = 0: no L)
    RunBits lrb;
    long long lbeg, nL;
    const unsigned long long* tbl;
};

// Cells with a long run in some slot (the cells around the window's sensors,
// crossed by many rays of every scan): one thread would walk each slot's run
// with a chain of dependent loads per word; they are queued instead
// (long_cells) and recomputed by k_apply_long, one wave per cell.
struct LongList {
    unsigned* count;     // cells queued (zeroed by the step's k_runmask before k_apply_window)
    unsigned* cells;
};

__device__ __forceinline__ unsigned long long readlane64(unsigned long long x, int l)
{
    const unsigned lo = __builtin_amdgcn_readlane((int)(unsigned)x, l);
    const unsigned hi = __builtin_amdgcn_readlane((int)(unsigned)(x >> 32), l);
    return ((unsigned long long)hi << 32) | lo;
}

// walk_run by a whole wave: the lanes hold 64 words of the run (from word
// w0, preloaded by the caller) and every lane follows the same (uniform) walk
// over them from registers; a run past them reloads
__device__ double walk_run_wave(long long i, double v, uint32_t& nh, uint32_t& nm, const RunBits& rb,
                                const BayesChains* __restrict__ ch, const BayesK& K, long long w0,
                                unsigned long long hwl, unsigned long long ewl)
{
    const int lane = (int)__lane_id();
    ChainState cs(v, ch);
    for (long long p = i;;) {
        const long long w = p >> 6;
        if (w0 < 0 || w - w0 >= 64) {
            w0 = w;
            const long long wl = w0 + lane;
            hwl = (wl < rb.nw) ? gload(rb.hitw + wl) : 0ull;
            ewl = (wl < rb.nw) ? gload(rb.endw + wl) : ~0ull;
        }
        const int sh = (int)(p & 63);
        const bool id_miss = K.miss_fixed && v == kPMin, id_hit = K.hit_fixed && v == kPMax;
        if (sh == 0 && (id_miss || id_hit)) {
            // whole words of identity updates (no run end, no hit -- resp.
            // miss -- in them): the lanes find the first word that is not,
            // one ballot for up to 64 words (cells next to a sensor see
            // thousands of misses at the fixed point)
            const int rel = (int)(w - w0);
            const bool stop = ewl != 0ull || (id_miss ? hwl != 0ull : ~hwl != 0ull);
            const unsigned long long b = __ballot(lane >= rel && stop);
            const int k = (b ? __ffsll((long long)b) - 1 : 64) - rel;
            if (k > 0) {
                if (id_miss) nm += 64u * (unsigned)k; else nh += 64u * (unsigned)k;
                p += 64LL * k;
                continue;
            }
        }
        const unsigned long long hm = readlane64(hwl, (int)(w - w0)) >> sh;
        const unsigned long long em = readlane64(ewl, (int)(w - w0)) >> sh;
        const int cnt = em ? __ffsll((long long)em) : 64 - sh;
        const unsigned long long inm = (cnt == 64) ? ~0ull : ((1ull << cnt) - 1ull);
        const unsigned long long h = hm & inm;
        nh += __popcll(h);
        nm += cnt - __popcll(h);
        v = apply_word(v, cs, h, inm & ~hm, cnt, ch, K);
        if (em) return v;
        p += cnt;
    }
}

__device__ void recompute_cell(const WindowJob& J, unsigned cell, const BayesChains* __restrict__ ch,
                               const BayesK& K, LongList ll)
{
    // the cell's run in every window slot, oldest first: one round of loads;
    // short runs are in the index itself, long ones are walked in their list
    const unsigned long long* e = J.tbl + (size_t)cell * kSlots;
    unsigned long long x[kSlots];
#pragma unroll
    for (int q = 0; q < kSlots; ++q) x[q] = (q < J.nwin) ? gload(e + J.order[q]) : 0ull;
    bool lng = false;
#pragma unroll
    for (int q = 0; q < kSlots; ++q)
        if (q < J.nwin && (unsigned)(x[q] >> 32) == J.st.s[J.order[q]] && ((unsigned)x[q] & kLongRun)) lng = true;
    {
        // one queue atomic per wave (hundreds of cells per step: same-address
        // device atomics serialise)
        const unsigned long long b = __ballot(lng);
        if (b) {
            const int lane = (int)__lane_id(), leader = __ffsll((long long)b) - 1;
            unsigned base = 0;
            if (lane == leader) base = atomicAdd(ll.count, (unsigned)__popcll(b));
            base = __shfl(base, leader);
            if (lng) ll.cells[base + (unsigned)__popcll(b & ((1ull << lane) - 1ull))] = cell;
        }
    }
    if (lng) return;
    // the slots' runs, oldest first, concatenated into 64-update words; each
    // word is applied with the chain state carried across slots (a cell that
    // saw only misses takes one chain look-up for the whole window)
    double v = 0.0;   // Reset (:290): Unknown
    ChainState cs(v, ch);
    uint32_t nh = 0, nm = 0;
    bool any = false;
    unsigned long long wb = 0;
    int wn = 0;
#pragma unroll
    for (int q = 0; q < kSlots; ++q) {
        if (q >= J.nwin) continue;
        const int s = J.order[q];
        if ((unsigned)(x[q] >> 32) != J.st.s[s]) continue;
        any = true;
        const unsigned en = (unsigned)x[q];
        const int len = (int)(en >> 26);
        const unsigned long long bits = en & ((1u << 26) - 1u);
        const int hits = __popcll(bits);
        nh += (uint32_t)hits;
        nm += (uint32_t)(len - hits);
        if (wn + len > 64) {
            const unsigned long long mk = (wn == 64) ? ~0ull : ((1ull << wn) - 1ull);
            v = apply_word(v, cs, wb, mk & ~wb, wn, ch, K);
            wb = 0, wn = 0;
        }
        wb |= bits << wn;
        wn += len;
    }
    if (wn > 0) {
        const unsigned long long mk = (wn == 64) ? ~0ull : ((1ull << wn) - 1ull);
        v = apply_word(v, cs, wb, mk & ~wb, wn, ch, K);
    }
    if (any) mark_patch(J.latest, cell);
    J.latest.cells[cell] = v;
    J.latest.hit[cell] = nh;
    J.latest.miss[cell] = nm;
}

__global__ __launch_bounds__(256) void k_apply_window(const WindowJob* __restrict__ jp,
                                                      const BayesChains* __restrict__ ch, double p_hit,
                                                      double p_miss, LongList ll)
{
    const WindowJob& J = *jp;
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    const BayesK K(p_hit, p_miss);
    const SlotView& E = J.slot[J.eslot];
    if (i < J.nE) {                                   // cells of E
        if (!run_start(E.rb.endw, i)) return;
        recompute_cell(J, E.keys[i] >> kTagShift, ch, K, ll);
    } else if (i < J.nE + J.nloc) {                   // E into the local map
        const long long p = J.lshift ? i - J.nE : i;
        if (!run_start(E.rb.endw, p)) return;
        const unsigned c = E.keys[p] >> kTagShift;
        const unsigned long long local =
            J.lshift ? (unsigned long long)((int)(c / (unsigned)J.latest.w) + J.ldy) * (unsigned)J.local.w +
                           (unsigned)((int)(c % (unsigned)J.latest.w) + J.ldx)
                     : c - J.local.base;
        mark_patch(J.local, local);
        uint32_t nh = 0, nm = 0;
        const double v = walk_run(p, J.local.cells[local], nh, nm, E.rb, ch, K);
        J.local.cells[local] = v;
        J.local.hit[local] += nh;
        J.local.miss[local] += nm;
    } else if (i < J.nE + J.nloc + J.nL) {            // cells of L not in E
        const long long p = J.lbeg + (i - J.nE - J.nloc);
        if (p != J.lbeg && !run_start(J.lrb.endw, p)) return;
        const unsigned cell = J.lkeys[p] >> kTagShift;
        const unsigned long long x = J.tbl[(size_t)cell * kSlots + J.eslot];
        if ((unsigned)(x >> 32) == J.st.s[J.eslot]) return;   // E's thread recomputes it
        recompute_cell(J, cell, ch, K, ll);
    }
}

// The queued cells, one wave per cell (every lane computes the same value).
__global__ __launch_bounds__(256) void k_apply_long(const WindowJob* __restrict__ jp,
                                                    const BayesChains* __restrict__ ch, double p_hit,
                                                    double p_miss, LongList ll)
{
    const WindowJob& J = *jp;
    const BayesK K(p_hit, p_miss);
    const int lane = (int)__lane_id();
    const unsigned nq = ll.count[0];
    const unsigned waves = gridDim.x * (blockDim.x / 64);
#ifdef LGS_PROBE
    const unsigned long long t_start = wall_clock64();
    unsigned n_cells = 0;
#endif
    for (unsigned k = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6); k < nq; k += waves) {
        const unsigned cell = ll.cells[k];
        const unsigned long long* e = J.tbl + (size_t)cell * kSlots;
        const unsigned long long xl = (lane < J.nwin) ? gload(e + J.order[lane]) : 0ull;
#ifdef LGS_PROBE
        unsigned long long t1 = 0, t2 = 0;
        if (blockIdx.x == 0 && threadIdx.x == 0) { (void)__builtin_amdgcn_readfirstlane((int)xl); t1 = wall_clock64(); }
#endif
        // the first 64 words of every slot's long run, all loads in flight at
        // once (one memory round trip for the cell, not one per slot)
        unsigned long long hw[kSlots], ew[kSlots];
#pragma unroll
        for (int q = 0; q < kSlots; ++q) {
            hw[q] = 0ull, ew[q] = ~0ull;
            if (q < J.nwin) {
                const int s = J.order[q];
                const unsigned long long x = readlane64(xl, q);
                if ((unsigned)(x >> 32) == J.st.s[s] && ((unsigned)x & kLongRun)) {
                    const long long wl = ((long long)((unsigned)x & ~kLongRun) >> 6) + lane;
                    const RunBits& rb = J.slot[s].rb;
                    if (wl < rb.nw) hw[q] = gload(rb.hitw + wl), ew[q] = gload(rb.endw + wl);
                }
            }
        }
#ifdef LGS_PROBE
        if (blockIdx.x == 0 && threadIdx.x == 0) { (void)__builtin_amdgcn_readfirstlane((int)(hw[0] ^ ew[J.nwin - 1])); t2 = wall_clock64(); }
#endif
        double v = 0.0;
        ChainState cs(v, ch);
        uint32_t nh = 0, nm = 0;
        bool any = false;
#pragma unroll
        for (int q = 0; q < kSlots; ++q) {
            if (q >= J.nwin) continue;
            const int s = J.order[q];
            const unsigned long long x = readlane64(xl, q);
            if ((unsigned)(x >> 32) != J.st.s[s]) continue;
            any = true;
            const unsigned en = (unsigned)x;
            if (en & kLongRun) {
                const long long p = (long long)(en & ~kLongRun);
                v = walk_run_wave(p, v, nh, nm, J.slot[s].rb, ch, K, p >> 6, hw[q], ew[q]);
                cs = ChainState(v, ch);
            } else {
                const int len = (int)(en >> 26);
                const unsigned long long bits = en & ((1u << 26) - 1u);
                const int hits = __popcll(bits);
                nh += (uint32_t)hits;
                nm += (uint32_t)(len - hits);
                v = apply_word(v, cs, bits, ((1ull << len) - 1ull) & ~bits, len, ch, K);
            }
        }
#ifdef LGS_PROBE
        ++n_cells;
        if (blockIdx.x == 0 && threadIdx.x == 0)
            printf("probe long cell %u: tbl %.2f us, preload %.2f us, walk %.2f us; hits %u misses %u\n", cell,
                   0.01 * (double)(t1 - t_start), 0.01 * (double)(t2 - t1), 0.01 * (double)(wall_clock64() - t2), nh, nm);
#endif
        if (lane == 0) {
            if (any) mark_patch(J.latest, cell);
            J.latest.cells[cell] = v;
            J.latest.hit[cell] = nh;
            J.latest.miss[cell] = nm;
        }
    }
#ifdef LGS_PROBE
    if (threadIdx.x == 0 && blockIdx.x == 0)
        printf("probe k_apply_long: cells %u waves %u, wave 0: %u cells in %.2f us\n", nq, waves, n_cells,
               0.01 * (double)(wall_clock64() - t_start));
#endif
}

// MapSaver::DrawMap (C/io/map_saver.cpp:276-313) for the W x H cells of the
// map (row stride `stride`) starting at cell (x0, y0): gray = (uint8)((1 - p)
// * 255) for 0 < p <= 1, else the background 192 (unallocated patches hold
// 0.0 and so render as the background too); rows flipped up-down if `flip`,
// as the PNG is written (:455-456).  One thread per 4 consecutive cells of a
// row.
__global__ __launch_bounds__(256) void k_render_gray(const double* __restrict__ cells, int stride, int x0c, int y0c,
                                                     int W, int H, int flip, uint8_t* __restrict__ img)
{
    const long long q = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    const int qw = (W + 3) / 4;
    if (q >= (long long)qw * H) return;
    const int y = (int)(q / qw), x0 = (int)(q % qw) * 4;
    uint8_t* row = img + (size_t)(flip ? H - 1 - y : y) * W;
    const double* src = cells + (size_t)(y0c + y) * stride + x0c;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int x = x0 + i;
        if (x >= W) break;
        const double v = src[x];
        row[x] = (v <= 0.0 || v > 1.0) ? (uint8_t)192 : (uint8_t)((1.0 - v) * 255.0);
    }
}

// Resize (:676-697) of the patch allocation flags: new patch (x, y) is old
// patch (x + pminx, y + pminy), or unallocated outside the old grid.
__global__ __launch_bounds__(256) void k_patch_remap(const uint8_t* __restrict__ src, int snpx, int snpy,
                                                     uint8_t* __restrict__ dst, int npx, int npy, int pminx,
                                                     int pminy)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= npx * npy) return;
    const int x = i % npx + pminx, y = i / npx + pminy;
    dst[i] = (x >= 0 && x < snpx && y >= 0 && y < snpy) ? src[(size_t)y * snpx + x] : (uint8_t)0;
}

// ---------------------------------------------------------------------------
// host: geometry restated from H/grid_map/grid_map.hpp
// ---------------------------------------------------------------------------
inline void world_to_cell(const lgs_map* m, double x, double y, int& ix, int& iy)
{
    // WorldCoordinateToGridCellIndex (:779-790)
    ix = (int)std::floor((x - m->min_x) / m->res);
    iy = (int)std::floor((y - m->min_y) / m->res);
}

inline int cell_to_patch(int idx, int ps) { return (idx < 0) ? (idx / ps - 1) : (idx / ps); }  // :905-915

// Cells, hit and miss counters of a map live in ONE allocation (cells at 0,
// hits at 8 n, misses at 12 n bytes), zeroed with one memset; d_cells owns it.
void map_alloc(lgs_map* m, int w, int h, double** cells, uint32_t** hit, uint32_t** miss)
{
    const size_t n = std::max<size_t>(1, (size_t)w * (size_t)h);
    void* p = nullptr;
    if (hipMalloc(&p, n * 16) != hipSuccess) throw Error(LGS_ERR_OOM, "hipMalloc failed for map");
    *cells = (double*)p;
    *hit = (uint32_t*)((char*)p + 8 * n);
    *miss = (uint32_t*)((char*)p + 12 * n);
    LGS_HIP_CHECK(hipMemsetAsync(p, 0, n * 16, m->ctx->stream));
}

void map_free(lgs_map* m)
{
    hipFree(m->d_cells);
    m->d_cells = nullptr;
    m->d_hit = m->d_miss = nullptr;
}

// Patch flags of a new map (all unallocated)
void palloc_init(lgs_map* m)
{
    const size_t n = std::max<size_t>(1, (size_t)m->npx * m->npy);
    if (hipMalloc(&m->d_palloc, n) != hipSuccess) throw Error(LGS_ERR_OOM, "hipMalloc failed for map patches");
    m->pcap = n;
    LGS_HIP_CHECK(hipMemsetAsync(m->d_palloc, 0, n, m->ctx->stream));
}

void palloc_free(lgs_map* m)
{
    hipFree(m->d_palloc);
    hipFree(m->d_palloc2);
    m->d_palloc = m->d_palloc2 = nullptr;
    m->pcap = m->pcap2 = 0;
}

void map_sync_view(lgs_map* m)
{
    m->view.ctx = m->ctx;
    m->view.device = m->device;
    m->view.d = m->d_cells;
    m->view.w = m->w;
    m->view.h = m->h;
    m->view.min_x = m->min_x;
    m->view.min_y = m->min_y;
    m->view.res = m->res;
    m->view.owned = false;
    m->view.map_view = true;
}

// Resize (:652-711): patches overlapping the new range keep their cells.
struct ResizeGeom {
    int pminx, pminy, npx, npy, w, h;
};

ResizeGeom resize_geom(const lgs_map* m, double minX, double minY, double maxX, double maxY)
{
    int cminx, cminy, cmaxx, cmaxy;
    world_to_cell(m, minX, minY, cminx, cminy);
    world_to_cell(m, maxX, maxY, cmaxx, cmaxy);
    const int ps = m->ps;
    ResizeGeom g;
    g.pminx = cell_to_patch(cminx, ps);
    g.pminy = cell_to_patch(cminy, ps);
    const int pmaxx = cell_to_patch(cmaxx, ps), pmaxy = cell_to_patch(cmaxy, ps);
    g.npx = std::max(0, pmaxx - g.pminx + 1);
    g.npy = std::max(0, pmaxy - g.pminy + 1);
    g.w = g.npx * ps;
    g.h = g.npy * ps;
    return g;
}

// Resize of the patch flags (before map_set_geom: m->npx/npy are the old
// counts).  A resize that keeps the patch grid leaves them in place.
void palloc_remap(lgs_map* m, const ResizeGeom& g)
{
    if (g.pminx == 0 && g.pminy == 0 && g.npx == m->npx && g.npy == m->npy) return;
    const size_t n = std::max<size_t>(1, (size_t)g.npx * g.npy);
    if (n > m->pcap2) {
        hipFree(m->d_palloc2);
        m->d_palloc2 = nullptr;
        m->pcap2 = 0;
        if (hipMalloc(&m->d_palloc2, 2 * n) != hipSuccess)
            throw Error(LGS_ERR_OOM, "hipMalloc failed for map patches");
        m->pcap2 = 2 * n;
    }
    if (g.npx * g.npy > 0)
        hipLaunchKernelGGL(k_patch_remap, dim3((unsigned)((g.npx * g.npy + 255) / 256)), dim3(256), 0,
                           m->ctx->stream, m->d_palloc, m->npx, m->npy, m->d_palloc2, g.npx, g.npy, g.pminx,
                           g.pminy);
    LGS_HIP_CHECK(hipGetLastError());
    std::swap(m->d_palloc, m->d_palloc2);
    std::swap(m->pcap, m->pcap2);
}

void map_set_geom(lgs_map* m, const ResizeGeom& g)
{
    m->npx = g.npx;
    m->npy = g.npy;
    m->w = g.w;
    m->h = g.h;
    m->min_x += (g.pminx * m->ps) * m->res;
    m->min_y += (g.pminy * m->ps) * m->res;
    map_sync_view(m);
}

void map_resize(lgs_map* m, double minX, double minY, double maxX, double maxY)
{
    const ResizeGeom g = resize_geom(m, minX, minY, maxX, maxY);
    const int ps = m->ps, nw = g.w, nh = g.h, pminx = g.pminx, pminy = g.pminy;
    double* cells;
    uint32_t *hit, *miss;
    map_alloc(m, nw, nh, &cells, &hit, &miss);
    const int x0 = std::max(0, pminx), y0 = std::max(0, pminy);
    const int x1 = std::min(m->npx, pminx + g.npx), y1 = std::min(m->npy, pminy + g.npy);
    if (x1 > x0 && y1 > y0) {
        const size_t cw = (size_t)(x1 - x0) * ps, ch = (size_t)(y1 - y0) * ps;
        const size_t ox = (size_t)x0 * ps, oy = (size_t)y0 * ps;
        const size_t nx = (size_t)(x0 - pminx) * ps, ny = (size_t)(y0 - pminy) * ps;
        hipStream_t st = m->ctx->stream;
        LGS_HIP_CHECK(hipMemcpy2DAsync(cells + ny * nw + nx, nw * sizeof(double),
                                       m->d_cells + oy * m->w + ox, m->w * sizeof(double),
                                       cw * sizeof(double), ch, hipMemcpyDeviceToDevice, st));
        LGS_HIP_CHECK(hipMemcpy2DAsync(hit + ny * nw + nx, nw * sizeof(uint32_t),
                                       m->d_hit + oy * m->w + ox, m->w * sizeof(uint32_t),
                                       cw * sizeof(uint32_t), ch, hipMemcpyDeviceToDevice, st));
        LGS_HIP_CHECK(hipMemcpy2DAsync(miss + ny * nw + nx, nw * sizeof(uint32_t),
                                       m->d_miss + oy * m->w + ox, m->w * sizeof(uint32_t),
                                       cw * sizeof(uint32_t), ch, hipMemcpyDeviceToDevice, st));
    }
    LGS_HIP_CHECK(hipStreamSynchronize(m->ctx->stream));
    map_free(m);
    m->d_cells = cells;
    m->d_hit = hit;
    m->d_miss = miss;
    m->cap = std::max<size_t>(1, (size_t)nw * nh);
    palloc_remap(m, g);
    map_set_geom(m, g);
}

// Resize followed by Reset (ConstructMapFromScans :288-290): every cell ends
// up zero, so nothing is copied and an allocation that is large enough is
// reused.
void map_resize_reset(lgs_map* m, double minX, double minY, double maxX, double maxY)
{
    const ResizeGeom g = resize_geom(m, minX, minY, maxX, maxY);
    const size_t need = std::max<size_t>(1, (size_t)g.w * g.h);
    hipStream_t st = m->ctx->stream;
    if (need > m->cap) {
        double* cells;
        uint32_t *hit, *miss;
        map_alloc(m, g.w, g.h, &cells, &hit, &miss);  // zeroed
        LGS_HIP_CHECK(hipStreamSynchronize(st));
        map_free(m);
        m->d_cells = cells;
        m->d_hit = hit;
        m->d_miss = miss;
        m->cap = need;
    } else {
        // the counters move to the offsets of the new cell count (one memset
        // zeroes cells, hits and misses)
        m->d_hit = (uint32_t*)((char*)m->d_cells + 8 * need);
        m->d_miss = (uint32_t*)((char*)m->d_cells + 12 * need);
        LGS_HIP_CHECK(hipMemsetAsync(m->d_cells, 0, need * 16, st));
    }
    palloc_remap(m, g);   // Reset keeps the patches allocated (grid_map_patch.hpp:194-203)
    map_set_geom(m, g);
}

bool map_inside(const lgs_map* m, double x, double y)
{
    int ix, iy;
    world_to_cell(m, x, y, ix, iy);
    return (ix >= 0 && ix < m->w) && (iy >= 0 && iy < m->h);
}

// Expand (:714-736)
void map_expand(lgs_map* m, double minX, double minY, double maxX, double maxY, double step)
{
    if (map_inside(m, minX, minY) && map_inside(m, maxX, maxY)) return;
    double minPX = m->min_x + m->res * 0, minPY = m->min_y + m->res * 0;
    double maxPX = m->min_x + m->res * m->w, maxPY = m->min_y + m->res * m->h;
    minPX = (minX < minPX) ? minX - step : minPX;
    minPY = (minY < minPY) ? minY - step : minPY;
    maxPX = (maxX > maxPX) ? maxX + step : maxPX;
    maxPY = (maxY > maxPY) ? maxY + step : maxPY;
    map_resize(m, minPX, minPY, maxPX, maxPY);
}

// the ray-cast passes' device error word: 1 a ray cell outside the map (k_emit),
// 2 the one-launch sort's grid barrier timed out (k_sort.hip)
inline const char* bad_message(int bad)
{
    return (bad & 2) ? "k_sort_wide: grid barrier timed out (cooperative tiles not co-resident)"
                     : "ray cell outside the map geometry";
}
inline double smin(double a, double b) { return (b < a) ? b : a; }  // std::min
inline double smax(double a, double b) { return (a < b) ? b : a; }  // std::max

struct ScanHits {
    lgs_pose2d sensor;
    std::vector<double> xy;  // hit points (x, y) of the usable beams, beam order
    // min x, min y, max x, max y of the sensor and the hit points
    double box[4];
};

// ComputeBoundingBoxAndScanPoints hit points (:335-380), glibc sin/cos
ScanHits scan_hits(const lgs_scan* s, lgs_pose2d robot, const lgs_builder_params* bp)
{
    ScanHits h;
    h.sensor = compound(robot, s->rel);
    const double minRange = smax(bp->usable_range_min, s->min_range);
    const double maxRange = smin(bp->usable_range_max, s->max_range);
    // the usable beams' angles, then their sincos four at a time (glibc bit
    // for bit, sincos_batch), then the points
    thread_local std::vector<double> th, rr, sn, cs;
    th.clear();
    rr.clear();
    for (int i = 0; i < s->n; ++i) {
        const double r = s->h_ranges[i];
        if (r >= maxRange || r <= minRange) continue;
        th.push_back(h.sensor.theta + s->h_angles[i]);
        rr.push_back(r);
    }
    const size_t m = th.size();
    sn.resize(m);
    cs.resize(m);
    sincos_batch(th.data(), (long long)m, sn.data(), cs.data());
    h.xy.resize(2 * m);
    for (size_t j = 0; j < m; ++j) {
        h.xy[2 * j] = h.sensor.x + rr[j] * cs[j];
        h.xy[2 * j + 1] = h.sensor.y + rr[j] * sn[j];
    }
    double b0 = h.sensor.x, b1 = h.sensor.y, b2 = h.sensor.x, b3 = h.sensor.y;
    for (size_t q = 0; q + 1 < h.xy.size(); q += 2) {
        b0 = smin(b0, h.xy[q]);
        b1 = smin(b1, h.xy[q + 1]);
        b2 = smax(b2, h.xy[q]);
        b3 = smax(b3, h.xy[q + 1]);
    }
    h.box[0] = b0, h.box[1] = b1, h.box[2] = b2, h.box[3] = b3;
    return h;
}

bool same_pose(lgs_pose2d a, lgs_pose2d b) { return std::memcmp(&a, &b, sizeof(a)) == 0; }

// scan_hits through the scan's one-entry cache (lgs_scan::hits_cache), keyed
// bitwise on the robot pose and the usable range.  Callers that may run in
// parallel over the same scan pass store = false and store afterwards.
typedef std::shared_ptr<const ScanHits> HitsPtr;
// (under the scan's cache_mu: contexts may update maps from one scan at once)
HitsPtr hits_lookup(const lgs_scan* s, const double* key)
{
    std::lock_guard<std::mutex> g(s->cache_mu);
    if (s->hits_cache && std::memcmp(key, s->hits_key, 5 * sizeof(double)) == 0)
        return std::static_pointer_cast<const ScanHits>(s->hits_cache);
    return nullptr;
}
void hits_store(const lgs_scan* s, const double* key, const HitsPtr& h)
{
    std::lock_guard<std::mutex> g(s->cache_mu);
    s->hits_cache = h;
    std::memcpy(s->hits_key, key, 5 * sizeof(double));
}
HitsPtr cached_hits(const lgs_scan* s, lgs_pose2d robot, const lgs_builder_params* bp, bool store)
{
    const double key[5] = { robot.x, robot.y, robot.theta, bp->usable_range_min, bp->usable_range_max };
    if (HitsPtr c = hits_lookup(s, key)) return c;
    HitsPtr h = std::make_shared<const ScanHits>(scan_hits(s, robot, bp));
    if (store) hits_store(s, key, h);
    return h;
}

// One map of a ray-cast pass and its scans (hit points in world coordinates).
struct MapJob {
    lgs_map* m;
    std::vector<HitsPtr> hs;
    std::vector<int> tags;   // per scan: slot tag of its keys (tagged passes; empty: 0)
};

// A tagged pass (the latest map's bootstrap, §4.4b): keys cell << 5 | slot
// << 1 | hit, one pass; the sorted keys stay in the pass's scratch for the
// caller (stream order) -- sorted[0, keys) by cell, jobs' maps in order.
struct TagPass {
    bool ok = false;                   // the pass ran tagged
    const unsigned* sorted = nullptr;
    long long keys = 0;
    long long job_keys[2] = {};
    long long tag_keys[kSlots] = {};   // keys of job 0 per slot tag
};

// Hit points of every job's scans (one parallel region over all of them) and
// each job's bounding box as ConstructMapFromScans accumulates it (:234-285)
// -- note topRight starts at numeric_limits<double>::min().  min/max of the
// per-scan boxes equals the reference's running min/max (no NaN reaches here).
void hits_and_boxes(std::vector<MapJob>& jobs, const std::vector<int>& first, const std::vector<int>& count,
                    const lgs_scan* const* scans, const lgs_pose2d* poses, const lgs_builder_params* bp,
                    std::vector<std::array<double, 4>>& boxes)
{
    // one computation per distinct (scan, pose): AppendScan's newest scan is
    // both the latest map's last scan and the local map's insert
    std::vector<std::pair<int, int>> work;
    std::vector<std::pair<int, int>> same;   // (job, k) -> the work item it shares
    std::unordered_map<const lgs_scan*, int> seen;
    for (size_t j = 0; j < jobs.size(); ++j) {
        jobs[j].hs.resize(count[j]);
        for (int k = 0; k < count[j]; ++k) {
            const int i = first[j] + k;
            int w = -1;
            const auto it = seen.find(scans[i]);
            if (it != seen.end()) {
                const int iq = first[work[it->second].first] + work[it->second].second;
                if (same_pose(poses[iq], poses[i])) w = it->second;
            }
            if (w < 0) {
                w = (int)work.size();
                work.emplace_back((int)j, k);
                seen.emplace(scans[i], w);
            }
            same.emplace_back((int)j, w);
        }
    }
    // cached hits first (a key compare each), then the missing ones -- on the
    // worker pool only when there are several (a frontend step computes one:
    // waking the pool would cost more than the scan's sincos)
    std::vector<int> todo;
    for (size_t w = 0; w < work.size(); ++w) {
        const int j = work[w].first, k = work[w].second;
        const lgs_scan* s = scans[first[j] + k];
        const lgs_pose2d p = poses[first[j] + k];
        const double key[5] = { p.x, p.y, p.theta, bp->usable_range_min, bp->usable_range_max };
        if (HitsPtr c = hits_lookup(s, key))
            jobs[j].hs[k] = c;
        else
            todo.push_back((int)w);
    }
    host_parallel_for((int)todo.size(), 2, [&](int t) {
        const int j = work[todo[t]].first, k = work[todo[t]].second;
        jobs[j].hs[k] = cached_hits(scans[first[j] + k], poses[first[j] + k], bp, false);
    });
    {
        size_t u = 0;
        for (size_t j = 0; j < jobs.size(); ++j)
            for (int k = 0; k < count[j]; ++k, ++u) {
                const auto& src = work[same[u].second];
                jobs[j].hs[k] = jobs[src.first].hs[src.second];
            }
    }
    boxes.assign(jobs.size(), std::array<double, 4>{DBL_MAX, DBL_MAX, DBL_MIN, DBL_MIN});
    for (size_t j = 0; j < jobs.size(); ++j)
        for (int k = 0; k < count[j]; ++k) {
            const ScanHits& h = *jobs[j].hs[k];
            const lgs_scan* s = scans[first[j] + k];
            const lgs_pose2d p = poses[first[j] + k];
            const double key[5] = { p.x, p.y, p.theta, bp->usable_range_min, bp->usable_range_max };
            hits_store(s, key, jobs[j].hs[k]);   // (serial: a scan may appear twice)
            auto& b = boxes[j];
            b[0] = smin(b[0], h.box[0]);
            b[1] = smin(b[1], h.box[1]);
            b[2] = smax(b[2], h.box[2]);
            b[3] = smax(b[3], h.box[3]);
        }
}

// Ray-cast every job's scans (already in its map's geometry), jobs in order,
// each job's scans in order.  The rays of all jobs share emit/sort/apply
// passes; a pass holds at most ctx->ray_chunk_keys keys and 2^31 cells of
// maps, and passes run in ray order, so each cell still sees its updates in
// the reference's order.
void raycast_maps(lgs_ctx* ctx, std::vector<MapJob>& jobs, const lgs_builder_params* bp, TagPass* tp = nullptr)
{
    hipStream_t st = ctx->stream;
    const auto t_rc0 = std::chrono::steady_clock::now();
    struct Unit {
        int job;
        int tag;
        const ScanHits* h;
        std::vector<int4> rays;
        std::vector<int> len;
        long long keys;
    };
    std::vector<Unit> units;
    for (int j = 0; j < (int)jobs.size(); ++j)
        for (size_t k = 0; k < jobs[j].hs.size(); ++k)
            if (jobs[j].hs[k]->xy.size() >= 2)
                units.push_back(Unit{j, jobs[j].tags.empty() ? 0 : jobs[j].tags[k], jobs[j].hs[k].get(), {}, {}, 0});
    if (tp) *tp = TagPass{};
    if (units.empty()) return;
    // sensor/hit cells and ray lengths (parallel over scans)
    host_parallel_for((int)units.size(), 2, [&](int u) {
        Unit& U = units[u];
        const lgs_map* m = jobs[U.job].m;
        const ScanHits& h = *U.h;
        int sx, sy;
        world_to_cell(m, h.sensor.x, h.sensor.y, sx, sy);
        const size_t nr = h.xy.size() / 2;
        U.rays.resize(nr);
        U.len.resize(nr);
        long long keys = 0;
        for (size_t k = 0; k < nr; ++k) {
            int hx, hy;
            world_to_cell(m, h.xy[2 * k], h.xy[2 * k + 1], hx, hy);
            U.rays[k] = make_int4(sx, sy, hx, hy);
            U.len[k] = std::max(std::abs(hx - sx), std::abs(hy - sy)) + 1;
            keys += U.len[k];
        }
        U.keys = keys;
    });
    long long total_keys = 0, total_rays = 0;
    unsigned long long total_cells = 0;
    for (size_t q = 0; q < units.size(); ++q) {
        total_keys += units[q].keys;
        total_rays += (long long)units[q].len.size();
        if (q == 0 || units[q].job != units[q - 1].job)
            total_cells += (unsigned long long)jobs[units[q].job].m->w * jobs[units[q].job].m->h;
    }
    const long long budget = std::max(1LL, std::min(ctx->ray_chunk_keys, 1LL << 30));
    // a tagged pass needs one pass and 27 cell bits; otherwise it runs untagged
    if (tp && !(total_keys <= budget && total_rays < (1LL << 30) && total_cells < (1ull << (32 - kTagShift))))
        tp = nullptr;
    const int ksh = tp ? kTagShift : 1;
    for (const MapJob& J : jobs)
        LGS_REQUIRE((size_t)J.m->w * J.m->h < (1ull << (32 - ksh)), "map too large for the cell bits of the keys");
    if (tp) {
        tp->ok = true;
        for (const Unit& U : units) {
            LGS_REQUIRE(U.job < 2 && U.tag < kSlots, "tagged pass: two maps, 16 slots");
            tp->job_keys[U.job] += U.keys;
            if (U.job == 0) tp->tag_keys[U.tag] += U.keys;
        }
    }
    // [0] rays leaving the map (int), [2..3] runs of equal cells applied (u64)
    int* d_bad = (int*)ctx->ensure(S_RAY4, 16);
    unsigned long long* d_runs = (unsigned long long*)(d_bad + 2);
    LGS_HIP_CHECK(hipMemsetAsync(d_bad, 0, 16, st));
    int apply_tok = -1;
    const BayesChains chains = make_chains(bp->prob_hit, bp->prob_miss);
    size_t u = 0, r = 0;
    int pass = 0;
    char* pin = nullptr;
    while (u < units.size()) {
        // plan one pass: rays [(u, r), (eu, er)) and the maps they touch
        std::vector<RayMap> maps;
        unsigned long long cells = 0;
        long long keys = 0, nr = 0;
        int cur = -1;
        size_t eu = u, er = r;
        if (pass == 0 && total_keys <= budget && total_rays < (1LL << 30) && total_cells < (1ull << (32 - ksh))) {
            // everything in one pass (the usual case): whole units
            for (size_t q = 0; q < units.size(); ++q)
                if (q == 0 || units[q].job != units[q - 1].job) {
                    const lgs_map* m = jobs[units[q].job].m;
                    maps.push_back(RayMap{cells, m->w, m->h, m->d_cells, m->d_hit, m->d_miss, m->d_palloc, m->ps, m->npx});
                    cells += (unsigned long long)m->w * m->h;
                }
            keys = total_keys, nr = total_rays, eu = units.size(), er = 0;
        }
        while (eu < units.size()) {
            const Unit& U = units[eu];
            if (er >= U.len.size()) {
                ++eu, er = 0;
                continue;
            }
            const long long L = U.len[er];
            if (nr > 0 && (keys + L > budget || nr >= (1LL << 30))) break;
            if (U.job != cur) {
                const lgs_map* m = jobs[U.job].m;
                const unsigned long long mc = (unsigned long long)m->w * m->h;
                if (nr > 0 && cells + mc > (1ull << (32 - ksh))) break;
                maps.push_back(RayMap{cells, m->w, m->h, m->d_cells, m->d_hit, m->d_miss, m->d_palloc, m->ps, m->npx});
                cells += mc;
                cur = U.job;
            }
            keys += L, ++nr, ++er;
        }
        const int nmaps = (int)maps.size();
        const bool multi = nmaps > 1 || tp;   // per-ray map | tag words
        // stage the map table, rays, key offsets and ray->map indices
        auto al = [](size_t b) { return (b + 63) & ~(size_t)63; };
        const size_t cb = al(sizeof(BayesChains));
        const size_t mb = cb + al(sizeof(RayMap) * nmaps), rb = al(sizeof(int4) * nr),
                     ob = al(sizeof(long long) * nr), ib = multi ? al(sizeof(int) * nr) : 0;
        if (pass > 0) ctx->sync();  // the previous pass's uploads have left the staging buffer
        pin = (char*)ctx->ensure_pinned(mb + rb + ob + ib + 64);
        std::memcpy(pin, &chains, sizeof(BayesChains));
        std::memcpy(pin + cb, maps.data(), sizeof(RayMap) * nmaps);
        int4* prays = (int4*)(pin + mb);
        long long* poffs = (long long*)(pin + mb + rb);
        int* pmap = (int*)(pin + mb + rb + ob);
        {
            // segments = the pass's part of each unit; their ray and key
            // offsets by a prefix over segments, then a parallel fill
            struct Seg {
                size_t unit, r0, r1;
                long long ray0, key0;
                int map;
                int tag;
            };
            std::vector<Seg> segs;
            long long ray0 = 0, key0 = 0;
            int mi = -1, cj = -1;
            for (size_t cu = u; cu < units.size() && ray0 < nr; ++cu) {
                const Unit& U = units[cu];
                const size_t r0 = (cu == u) ? r : 0;
                const size_t r1 = std::min(U.len.size(), r0 + (size_t)(nr - ray0));
                if (r1 <= r0) continue;
                if (U.job != cj) cj = U.job, ++mi;
                segs.push_back(Seg{cu, r0, r1, ray0, key0, mi, U.tag});
                long long kk = 0;
                if (r0 == 0 && r1 == U.len.size()) kk = U.keys;
                else
                    for (size_t q = r0; q < r1; ++q) kk += U.len[q];
                ray0 += (long long)(r1 - r0);
                key0 += kk;
            }
            host_parallel_for((int)segs.size(), 4, [&](int g) {
                const Seg& S = segs[g];
                const Unit& U = units[S.unit];
                long long k = S.ray0, off = S.key0;
                for (size_t q = S.r0; q < S.r1; ++q, ++k) {
                    prays[k] = U.rays[q];
                    poffs[k] = off;
                    if (multi) pmap[k] = S.map | (S.tag << 16);
                    off += U.len[q];
                }
            });
        }
        char* d_stage = (char*)ctx->ensure(S_RAY6, mb + rb + ob + ib);
        if (std::getenv("LGS_F2_TIMING"))
            std::fprintf(stderr, "f2 raycast host prep (cells + staging) %.1f us, %zu bytes staged\n",
                         std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t_rc0).count(),
                         mb + rb + ob + ib);
        LGS_HIP_CHECK(hipMemcpyAsync(d_stage, pin, mb + rb + ob + ib, hipMemcpyHostToDevice, st));
        const BayesChains* d_chains = (const BayesChains*)d_stage;
        const RayMap* d_maps = (const RayMap*)(d_stage + cb);
        const int4* d_rays = (const int4*)(d_stage + mb);
        const long long* d_offs = (const long long*)(d_stage + mb + rb);
        const int* d_rmap = multi ? (const int*)(d_stage + mb + rb + ob) : nullptr;
        unsigned* d_keys = (unsigned*)ctx->ensure(S_RAY2, sizeof(unsigned) * keys);
        unsigned* d_sorted = (unsigned*)ctx->ensure(S_RAY3, sizeof(unsigned) * keys);
        // algorithmic bytes: 4 B per emitted key (emit); 4 B per
        // key + 32 B per run of equal cells (cell, hit and miss counters read
        // and written once; the run count is added after the last pass)
        int tok = ctx->timing_begin(K_RAY_EMIT, 4.0 * (double)keys);
        hipLaunchKernelGGL(k_emit, dim3((unsigned)((nr + 3) / 4)), dim3(256), 0, st, d_rays, d_offs, d_rmap,
                           (int)nr, d_maps, d_keys, d_bad, ksh);
        ctx->timing_end(tok);
        LGS_HIP_CHECK(hipGetLastError());
        int cell_bits = 1;
        while (cell_bits < 32 && (1ull << cell_bits) < cells) ++cell_bits;
        unsigned* d_tmp = (unsigned*)ctx->ensure(S_RAY5, sizeof(unsigned) * keys);
        keysort(ctx, d_keys, d_sorted, d_tmp, keys, ksh, cell_bits, d_bad);
        tok = ctx->timing_begin(K_RAY_APPLY, 4.0 * (double)keys);
        if (tok >= 0) apply_tok = tok;
        const long long nw = (keys + 63) / 64;
        const long long nw2 = (nw + 63) / 64;
        unsigned long long* d_hitw =
            (unsigned long long*)ctx->ensure(S_RAY7, sizeof(unsigned long long) * (2 * nw + 3 * nw2));
        unsigned long long* d_endw = d_hitw + nw;
        unsigned long long* d_hit2 = d_endw + nw;
        unsigned long long* d_miss2 = d_hit2 + nw2;
        unsigned long long* d_end2 = d_miss2 + nw2;
        const unsigned blocks = (unsigned)((keys + 255) / 256);
        hipLaunchKernelGGL(k_runmask, dim3(blocks), dim3(256), 0, st, d_sorted, keys, ksh, d_hitw, d_endw,
                           RunIndex{});
        hipLaunchKernelGGL(k_runsummary, dim3((unsigned)((nw + 255) / 256)), dim3(256), 0, st, d_hitw, d_endw, nw,
                           d_hit2, d_miss2, d_end2);
        hipLaunchKernelGGL(k_apply, dim3(blocks), dim3(256), 0, st, d_sorted, keys,
                           RunBits{d_hitw, d_endw, d_hit2, d_miss2, d_end2, nw}, d_maps, nmaps, d_chains, bp->prob_hit,
                           bp->prob_miss, ksh);
        ctx->timing_end(tok);
        if (tok >= 0)
            hipLaunchKernelGGL(k_count_runs, dim3((unsigned)std::min<long long>((nw + 255) / 256, 512)), dim3(256), 0,
                               st, d_endw, nw, d_runs);
        LGS_HIP_CHECK(hipGetLastError());
        if (tp) {
            tp->sorted = d_sorted;
            tp->keys = keys;
        }
        u = eu, r = er;
        ++pass;
    }
    // (stream order: the copy into the staging buffer follows the uploads from it)
    LGS_HIP_CHECK(hipMemcpyAsync(pin, d_bad, 16, hipMemcpyDeviceToHost, st));
    ctx->sync();
    int bad = 0;
    unsigned long long runs = 0;
    std::memcpy(&bad, pin, sizeof(int));
    std::memcpy(&runs, pin + 8, sizeof(runs));
    if (apply_tok >= 0) ctx->pending[apply_tok].algo_bytes += 32.0 * (double)runs;
    if (ctx->profile) ctx->harvest();
    if (bad) throw Error(LGS_ERR_INTERNAL, bad_message(bad));
}

// ConstructMapFromScans of several maps (AfterLoopClosure; a global map) with
// the hit points, boxes, ray cells and key offsets formed on the device
// (k_hits, k_raycells): the host keeps the geometry
// (Resize) between the two device phases, from the boxes k_hits returns --
// identical values, so identical maps.  Returns false, with the maps as they
// were or resized and reset for the same boxes, when the pass does not fit
// one emit/sort/apply pass or an angle lies outside gl_sincos's domain: the
// caller then runs the host path.
bool construct_maps_device(lgs_ctx* ctx, lgs_map* const* maps, const int* first, const int* count, int n_maps,
                           const lgs_scan* const* scans, const lgs_pose2d* poses, const lgs_builder_params* bp)
{
    hipStream_t st = ctx->stream;
    std::vector<HitUnit> units;
    std::vector<int> unit_scan;
    long long beams = 0;
    for (int j = 0; j < n_maps; ++j)
        for (int k = 0; k < count[j]; ++k) {
            const int i = first[j] + k;
            const lgs_scan* sc = scans[i];
            HitUnit U{};
            const lgs_pose2d sp = compound(poses[i], sc->rel);   // :340-341
            U.n = sc->n;
            U.job = j;
            U.sx = sp.x, U.sy = sp.y, U.st = sp.theta;
            U.min_r = std::max(bp->usable_range_min, sc->min_range);
            U.max_r = std::min(bp->usable_range_max, sc->max_range);
            U.beam0 = beams;
            beams += sc->n;
            units.push_back(U);
            unit_scan.push_back(i);
        }
    const int nu = (int)units.size();
    if (nu == 0 || beams >= (1LL << 30)) return false;
    {
        std::vector<const lgs_scan*> sv;
        for (int i : unit_scan) sv.push_back(scans[i]);
        scans_to_device(ctx, sv.data(), (int)sv.size());
    }
    for (int u = 0; u < nu; ++u) {
        units[u].ranges = scans[unit_scan[u]]->d_ranges;
        units[u].angles = scans[unit_scan[u]]->d_angles;
    }
    auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
    const size_t o_hits = 0, o_rays = o_hits + al(16 * (size_t)beams), o_offs = o_rays + al(16 * (size_t)beams),
                 o_rmap = o_offs + al(8 * (size_t)beams), o_cnt = o_rmap + al(4 * (size_t)beams),
                 o_box = o_cnt + al(4 * (size_t)nu), o_ukeys = o_box + al(32 * (size_t)nu),
                 o_kbase = o_ukeys + al(8 * (size_t)nu), o_total = o_kbase + al(8 * (size_t)nu),
                 o_end = o_total + 256;
    char* d = (char*)ctx->ensure(S_RAY8, o_end);
    double2* d_hits = (double2*)(d + o_hits);
    int4* d_rays = (int4*)(d + o_rays);
    long long* d_offs = (long long*)(d + o_offs);
    int* d_rmap = (int*)(d + o_rmap);
    int* d_cnt = (int*)(d + o_cnt);
    double4* d_box = (double4*)(d + o_box);
    long long* d_ukeys = (long long*)(d + o_ukeys);
    long long* d_kbase = (long long*)(d + o_kbase);
    long long* d_total = (long long*)(d + o_total);
    int* d_bad = (int*)ctx->ensure(S_RAY4, 16);
    unsigned long long* d_runs = (unsigned long long*)(d_bad + 2);
    LGS_HIP_CHECK(hipMemsetAsync(d_bad, 0, 16, st));
    // phase 1: hit points, counts and boxes
    {
        Upload up(ctx);
        const size_t uo = up.append(units.data(), units.size());
        up.flush();
        hipLaunchKernelGGL(k_hits, dim3(nu), dim3(256), 0, st, up.at<HitUnit>(uo), d_hits, d_cnt, d_box, d_bad);
        LGS_HIP_CHECK(hipGetLastError());
    }
    std::vector<int> cnt(nu);
    std::vector<std::array<double, 4>> ubox(nu);
    int bad = 0;
    {
        char* pin = (char*)ctx->ensure_pinned(al(4 * (size_t)nu) + 32 * (size_t)nu + 16);
        LGS_HIP_CHECK(hipMemcpyAsync(pin, d_cnt, 4 * (size_t)nu, hipMemcpyDeviceToHost, st));
        LGS_HIP_CHECK(hipMemcpyAsync(pin + al(4 * (size_t)nu), d_box, 32 * (size_t)nu, hipMemcpyDeviceToHost, st));
        LGS_HIP_CHECK(hipMemcpyAsync(pin + al(4 * (size_t)nu) + 32 * (size_t)nu, d_bad, 4, hipMemcpyDeviceToHost, st));
        ctx->sync();
        std::memcpy(cnt.data(), pin, 4 * (size_t)nu);
        std::memcpy(ubox.data(), pin + al(4 * (size_t)nu), 32 * (size_t)nu);
        std::memcpy(&bad, pin + al(4 * (size_t)nu) + 32 * (size_t)nu, 4);
    }
    if (bad) return false;
    // the maps' boxes as ConstructMapFromScans accumulates them (:234-285;
    // topRight starts at numeric_limits<double>::min()), then Resize + Reset
    std::vector<std::array<double, 4>> box(n_maps, std::array<double, 4>{ DBL_MAX, DBL_MAX, DBL_MIN, DBL_MIN });
    for (int u = 0; u < nu; ++u) {
        auto& b = box[units[u].job];
        b[0] = smin(b[0], ubox[u][0]);
        b[1] = smin(b[1], ubox[u][1]);
        b[2] = smax(b[2], ubox[u][2]);
        b[3] = smax(b[3], ubox[u][3]);
    }
    for (int j = 0; j < n_maps; ++j) map_resize_reset(maps[j], box[j][0], box[j][1], box[j][2], box[j][3]);
    // phase 2: ray cells, ray -> map, key offsets
    std::vector<int> ray0(nu);
    long long nr = 0;
    for (int u = 0; u < nu; ++u) {
        ray0[u] = (int)nr;
        nr += cnt[u];
    }
    std::vector<RayMap> rm(n_maps);
    std::vector<MapGeo> geo(n_maps);
    unsigned long long cells = 0;
    for (int j = 0; j < n_maps; ++j) {
        const lgs_map* m = maps[j];
        rm[j] = RayMap{ cells, m->w, m->h, m->d_cells, m->d_hit, m->d_miss, m->d_palloc, m->ps, m->npx };
        geo[j] = MapGeo{ m->min_x, m->min_y, m->res };
        cells += (unsigned long long)m->w * m->h;
    }
    if (nr == 0 || nr >= (1LL << 30) || cells >= (1ull << 31)) return false;
    const bool multi = n_maps > 1;
    const BayesChains chains = make_chains(bp->prob_hit, bp->prob_miss);
    Upload up(ctx);
    const size_t uo = up.append(units.data(), units.size());
    const size_t go = up.append(geo.data(), geo.size());
    const size_t ro = up.append(ray0.data(), ray0.size());
    const size_t co = up.append(&chains, 1);
    const size_t mo = up.append(rm.data(), rm.size());
    up.flush();
    hipLaunchKernelGGL(k_raycells, dim3(nu), dim3(256), 0, st, up.at<HitUnit>(uo), (const double2*)d_hits, d_cnt,
                       up.at<MapGeo>(go), up.at<int>(ro), d_rays, d_offs, multi ? d_rmap : nullptr, d_ukeys);
    hipLaunchKernelGGL(k_unit_scan, dim3(1), dim3(256), 0, st, d_ukeys, nu, d_kbase, d_total);
    hipLaunchKernelGGL(k_addbase, dim3(nu), dim3(256), 0, st, d_cnt, up.at<int>(ro), d_kbase, d_offs);
    LGS_HIP_CHECK(hipGetLastError());
    long long keys = 0;
    {
        char* pin = (char*)ctx->ensure_pinned(16);
        LGS_HIP_CHECK(hipMemcpyAsync(pin, d_total, 8, hipMemcpyDeviceToHost, st));
        ctx->sync();
        std::memcpy(&keys, pin, 8);
    }
    const long long budget = std::max(1LL, std::min(ctx->ray_chunk_keys, 1LL << 30));
    if (keys > budget) return false;
    // phase 3: emit, sort, runs, apply -- raycast_maps' pass
    const RayMap* d_maps = up.at<RayMap>(mo);
    const BayesChains* d_chains = up.at<BayesChains>(co);
    unsigned* d_keys = (unsigned*)ctx->ensure(S_RAY2, sizeof(unsigned) * keys);
    unsigned* d_sorted = (unsigned*)ctx->ensure(S_RAY3, sizeof(unsigned) * keys);
    int tok = ctx->timing_begin(K_RAY_EMIT, 4.0 * (double)keys);
    hipLaunchKernelGGL(k_emit, dim3((unsigned)((nr + 3) / 4)), dim3(256), 0, st, d_rays, d_offs,
                       multi ? d_rmap : nullptr, (int)nr, d_maps, d_keys, d_bad, 1);
    ctx->timing_end(tok);
    LGS_HIP_CHECK(hipGetLastError());
    int cell_bits = 1;
    while (cell_bits < 32 && (1ull << cell_bits) < cells) ++cell_bits;
    unsigned* d_tmp = (unsigned*)ctx->ensure(S_RAY5, sizeof(unsigned) * keys);
    keysort(ctx, d_keys, d_sorted, d_tmp, keys, 1, cell_bits, d_bad);
    tok = ctx->timing_begin(K_RAY_APPLY, 4.0 * (double)keys);
    const long long nw = (keys + 63) / 64;
    const long long nw2 = (nw + 63) / 64;
    unsigned long long* d_hitw = (unsigned long long*)ctx->ensure(S_RAY7, sizeof(unsigned long long) * (2 * nw + 3 * nw2));
    unsigned long long* d_endw = d_hitw + nw;
    unsigned long long* d_hit2 = d_endw + nw;
    unsigned long long* d_miss2 = d_hit2 + nw2;
    unsigned long long* d_end2 = d_miss2 + nw2;
    const unsigned blocks = (unsigned)((keys + 255) / 256);
    hipLaunchKernelGGL(k_runmask, dim3(blocks), dim3(256), 0, st, d_sorted, keys, 1, d_hitw, d_endw, RunIndex{});
    hipLaunchKernelGGL(k_runsummary, dim3((unsigned)((nw + 255) / 256)), dim3(256), 0, st, d_hitw, d_endw, nw, d_hit2,
                       d_miss2, d_end2);
    hipLaunchKernelGGL(k_apply, dim3(blocks), dim3(256), 0, st, d_sorted, keys,
                       RunBits{ d_hitw, d_endw, d_hit2, d_miss2, d_end2, nw }, d_maps, n_maps, d_chains, bp->prob_hit,
                       bp->prob_miss, 1);
    ctx->timing_end(tok);
    if (tok >= 0)
        hipLaunchKernelGGL(k_count_runs, dim3((unsigned)std::min<long long>((nw + 255) / 256, 512)), dim3(256), 0, st,
                           d_endw, nw, d_runs);
    LGS_HIP_CHECK(hipGetLastError());
    char* pin = (char*)ctx->ensure_pinned(16);
    LGS_HIP_CHECK(hipMemcpyAsync(pin, d_bad, 16, hipMemcpyDeviceToHost, st));
    ctx->sync();
    unsigned long long runs = 0;
    std::memcpy(&bad, pin, sizeof(int));
    std::memcpy(&runs, pin + 8, sizeof(runs));
    if (tok >= 0) ctx->pending[tok].algo_bytes += 32.0 * (double)runs;
    if (ctx->profile) ctx->harvest();
    if (bad) throw Error(LGS_ERR_INTERNAL, bad_message(bad));
    return true;
}

void raycast(lgs_map* m, std::vector<HitsPtr>&& scans, const lgs_builder_params* bp)
{
    std::vector<MapJob> jobs(1);
    jobs[0].m = m;
    jobs[0].hs = std::move(scans);
    raycast_maps(m->ctx, jobs, bp);
}

// ---------------------------------------------------------------------------
// The latest map's incremental rebuild
//
// UpdateLatestMap (C/mapping/grid_map_builder.cpp:196-207) rebuilds the latest
// map from the last n scans after every scan: Resize to the scans' bounding box,
// Reset, then every scan's rays in order.  When the box keeps the map's
// geometry and the window only gained the new scan E (and lost its oldest L),
// the result differs from the previous latest map only in the cells E or L
// touches: every other cell sees the same update sequence from Unknown.  The
// window's scans therefore keep their sorted key lists on the device (tagged
// keys, one slot per scan), and a step casts E alone (plus its insert into the
// local map, one pass), sorts its keys, indexes its runs and recomputes the
// touched cells over the window's lists -- the other scans are neither re-cast
// nor re-sorted.  Any other change (geometry, window, parameters) rebuilds in
// full, which also re-seeds the lists.
// ---------------------------------------------------------------------------
struct KeyBuf {
    void* base = nullptr;
    long long cap = 0;
    unsigned* keys = nullptr;
    unsigned long long *hitw = nullptr, *endw = nullptr, *hit2 = nullptr, *miss2 = nullptr, *end2 = nullptr;
    KeyBuf() = default;
    KeyBuf(const KeyBuf&) = delete;
    KeyBuf& operator=(const KeyBuf&) = delete;
    ~KeyBuf()
    {
        if (base) hipFree(base);
    }
    long long nw = 0;
    RunBits bits() const { return RunBits{ hitw, endw, hit2, miss2, end2, nw }; }
};
typedef std::shared_ptr<KeyBuf> KeyBufPtr;

KeyBufPtr keybuf_new(long long cap)
{
    KeyBufPtr b = std::make_shared<KeyBuf>();
    const long long nw = (cap + 63) / 64 + 1, nw2 = (nw + 63) / 64 + 1;
    const size_t kb = ((size_t)cap * 4 + 255) & ~(size_t)255;
    if (hipMalloc(&b->base, kb + 8 * (size_t)(2 * nw + 3 * nw2)) != hipSuccess)
        throw Error(LGS_ERR_OOM, "hipMalloc failed for latest-map key lists");
    b->cap = cap;
    b->nw = nw;
    b->keys = (unsigned*)b->base;
    b->hitw = (unsigned long long*)((char*)b->base + kb);
    b->endw = b->hitw + nw;
    b->hit2 = b->endw + nw;
    b->miss2 = b->hit2 + nw2;
    b->end2 = b->miss2 + nw2;
    return b;
}

struct LatestSlot {
    unsigned long long uid = 0;
    lgs_pose2d pose{ 0, 0, 0 };
    unsigned stamp = 0;
    KeyBufPtr buf;
    long long beg = 0, end = 0;   // the scan's keys in buf
};

constexpr int kMaxWindow = kSlots - 1;              // E takes a free slot before L leaves
constexpr size_t kMaxTblCells = 4u << 20;           // index table: 128 B per latest-map cell

struct LatestCache {
    bool valid = false;
    int w = 0, h = 0;             // geometry the lists were cast in
    double min_x = 0, min_y = 0;
    double bpv[4] = {};           // usable range min/max, pHit, pMiss
    std::vector<int> window;      // ring slots, oldest first
    LatestSlot slot[kSlots];
    unsigned long long* d_tbl = nullptr;
    size_t tbl_cells = 0;
    unsigned* d_long = nullptr;   // k_apply_long queue: [0] count, [1] done, then cells
    long long long_cap = 0;
    std::vector<KeyBufPtr> pool, retired;
    int* h_bad = nullptr;         // mapped pinned word: a ray left the map (set by k_emit, never cleared)
    int* d_bad = nullptr;
    std::shared_ptr<WriterEvent> wev;   // end of the last step (the maps' pending writer)
    bool pending = false;
    char* pin = nullptr;
    size_t pin_cap = 0;
    long long n_incremental = 0, n_full = 0;
    ~LatestCache()
    {
        for (auto& s : slot) s.buf.reset();
        pool.clear();
        retired.clear();
        if (d_tbl) hipFree(d_tbl);
        if (d_long) hipFree(d_long);
        if (h_bad) hipHostFree(h_bad);
        if (pin) hipHostFree(pin);
    }
    // the previous step has finished: its error word is final, the staging
    // buffer is free, the lists it released can be reused
    void finish()
    {
        if (pending) {
            wev->wait();
            pending = false;
        }
        std::vector<KeyBufPtr> r;
        r.swap(retired);
        for (auto& b : r) {
            if (b.use_count() == 1) pool.push_back(std::move(b));
            else b.reset();
        }
        if (*h_bad) {
            const int bad = *h_bad;
            drop_lists();
            *h_bad = 0;
            throw Error(LGS_ERR_INTERNAL, bad_message(bad));
        }
    }
    KeyBufPtr acquire(long long need)
    {
        for (size_t i = 0; i < pool.size(); ++i)
            if (pool[i]->cap >= need) {
                KeyBufPtr b = std::move(pool[i]);
                pool.erase(pool.begin() + (long)i);
                return b;
            }
        if (pool.size() > 4) pool.erase(pool.begin());
        return keybuf_new(need + need / 2 + 4096);
    }
    void drop_lists()
    {
        valid = false;
        for (auto& s : slot) {
            if (s.buf) retired.push_back(std::move(s.buf));
            s = LatestSlot{};
        }
        window.clear();
    }
};

LatestCache& cache_of(lgs_map* m)
{
    if (!m->cache) {
        LatestCache* c = new LatestCache();
        c->wev = std::make_shared<WriterEvent>();
        if (hipHostMalloc((void**)&c->h_bad, 16, hipHostMallocMapped) != hipSuccess ||
            hipHostGetDevicePointer((void**)&c->d_bad, c->h_bad, 0) != hipSuccess ||
            hipHostMalloc((void**)&c->wev->flag, sizeof(unsigned), hipHostMallocCoherent) != hipSuccess) {
            delete c;
            throw Error(LGS_ERR_OOM, "latest-map cache allocation failed");
        }
        *c->h_bad = 0;
        *c->wev->flag = 0;
        m->cache = c;
    }
    return *m->cache;
}

// any other change of the map's cells invalidates its lists
void invalidate_cache(lgs_map* m)
{
    if (!m->cache) return;
    m->cache->finish();
    m->cache->drop_lists();
}


// The step's device work stays queued when the call returns: its completion
// word (k_writer_done after the work) tells the host; readers of the maps on
// other streams order after it (grid_acquire, WriterEvent).
// (no fence: the kernels before it on the stream have completed and released
// their writes at their ends; the word is the only thing the host reads, a
// system-scope store into uncached coherent memory)
__global__ void k_writer_done(unsigned* flag, unsigned gen)
{
    __hip_atomic_store(flag, gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
void record_writer(LatestCache& C, hipStream_t st, lgs_map* latest, lgs_map* local)
{
    static std::atomic<unsigned> counter{ 0 };
    unsigned gen = ++counter;
    if (gen == 0) gen = ++counter;   // 0: the word's initial value
    {
        std::lock_guard<std::mutex> lk(C.wev->mu);
        C.wev->st.store(st, std::memory_order_release);
        C.wev->gen.store(gen, std::memory_order_release);
    }
    hipLaunchKernelGGL(k_writer_done, dim3(1), dim3(1), 0, st, C.wev->flag, gen);
    LGS_HIP_CHECK(hipGetLastError());
    C.pending = true;
    latest->view.writer = C.wev;
    if (local) local->view.writer = C.wev;
}

// Sensor/hit cells of one scan's rays in a map's geometry (as raycast_maps),
// appended to rays/lens; returns the scan's key count.
long long scan_rays(const lgs_map* m, const ScanHits& h, std::vector<int4>& rays, std::vector<int>& lens)
{
    int sx, sy;
    world_to_cell(m, h.sensor.x, h.sensor.y, sx, sy);
    const size_t n2 = h.xy.size() & ~(size_t)1;
    std::vector<int> c(n2);
    cells_of_points(h.xy.data(), (long long)n2, m->min_x, m->min_y, m->res, c.data());
    long long keys = 0;
    for (size_t k = 0; k < n2; k += 2) {
        const int hx = c[k], hy = c[k + 1];
        rays.push_back(make_int4(sx, sy, hx, hy));
        const int L = std::max(std::abs(hx - sx), std::abs(hy - sy)) + 1;
        lens.push_back(L);
        keys += L;
    }
    return keys;
}

inline int bits_for(unsigned long long cells)
{
    int b = 1;
    while (b < 32 && (1ull << b) < cells) ++b;
    return b;
}

RayMap raymap_of(const lgs_map* m, unsigned long long base)
{
    return RayMap{ base, m->w, m->h, m->d_cells, m->d_hit, m->d_miss, m->d_palloc, m->ps, m->npx };
}

// LGS_STEP_TIMING=1: host wall time of the latest-map step's phases, averaged
// over every 500 steps, on stderr (diagnostics)
struct StepTiming {
    bool on = std::getenv("LGS_STEP_TIMING") != nullptr;
    std::chrono::steady_clock::time_point prev;
    double us[8] = {};
    double keys = 0, rays = 0, longq = 0;
    long long steps = 0;
    void start()
    {
        if (on) prev = std::chrono::steady_clock::now();
    }
    void lap(int k)
    {
        if (!on) return;
        const auto now = std::chrono::steady_clock::now();
        us[k] += std::chrono::duration<double, std::micro>(now - prev).count();
        prev = now;
    }
    void done()
    {
        if (!on || ++steps % 500) return;
        std::fprintf(stderr, "latest step host us: finish %.1f hits %.1f geom %.1f pre %.1f rays(latest) %.1f "
                     "rays(local)+shift %.1f stage %.1f launch %.1f; keys %.0f rays %.0f L-keys %.0f\n", us[0] / 500,
                     us[1] / 500, us[2] / 500, us[6] / 500, us[7] / 500, us[3] / 500, us[4] / 500, us[5] / 500,
                     keys / 500, rays / 500, longq / 500);
        for (double& u : us) u = 0;
        keys = rays = longq = 0;
    }
};
StepTiming& step_timing()
{
    static StepTiming t;
    return t;
}

// One incremental step: E = the window's newest scan; L = its oldest (evict).
void latest_step(lgs_ctx* ctx, LatestCache& C, lgs_map* latest, lgs_map* local, const lgs_scan* escan,
                 lgs_pose2d epose, const HitsPtr& E, bool evict, const lgs_builder_params* bp)
{
    hipStream_t st = ctx->stream;
    LatestSlot L;
    int es = -1;
    if (evict) {
        es = C.window.front();
        L = C.slot[es];
        C.window.erase(C.window.begin());
    } else {
        bool used[kSlots] = {};
        for (int q : C.window) used[q] = true;
        for (int q = 0; q < kSlots && es < 0; ++q)
            if (!used[q]) es = q;
    }
    // E's rays in the latest map's and the local map's geometry
    std::vector<int4> rays;
    std::vector<int> lens;
    rays.reserve(E->xy.size());
    lens.reserve(E->xy.size());
    StepTiming& tm = step_timing();
    tm.lap(6);
    const long long nE = scan_rays(latest, *E, rays, lens);
    const size_t nrE = rays.size();
    tm.lap(7);
    long long nloc = local ? scan_rays(local, *E, rays, lens) : 0;
    // the local map's cells of E's rays are usually its latest-map cells
    // shifted by whole cells (both maps keep the lattice of their common
    // origin): then E is cast and sorted once and the local insert walks the
    // same runs -- checked ray by ray with the host's own cell computations
    int lshift = 0, ldx = 0, ldy = 0;
    if (local && nrE > 0) {
        ldx = rays[nrE].x - rays[0].x;
        ldy = rays[nrE].y - rays[0].y;
        lshift = 1;
        for (size_t k = 0; k < nrE && lshift; ++k) {
            const int4 a = rays[k], b = rays[nrE + k];
            lshift = b.x == a.x + ldx && b.y == a.y + ldy && b.z == a.z + ldx && b.w == a.w + ldy;
        }
        if (lshift) {
            rays.resize(nrE);
            lens.resize(nrE);
        }
    }
    tm.lap(3);
    const long long keys = lshift ? nE : nE + nloc;
    const long long nr = (long long)rays.size();
    const unsigned long long lat_cells = (unsigned long long)latest->w * latest->h;
    const unsigned long long cells =
        lat_cells + ((local && !lshift) ? (unsigned long long)local->w * local->h : 0ull);
    LGS_REQUIRE(cells < (1ull << (32 - kTagShift)), "latest step: cell bits");
    KeyBufPtr buf = C.acquire(std::max(1LL, keys));
    const unsigned stamp = (unsigned)ctx->next_stamp();
    // staging: chains | maps[2] | job | rays | offsets | ray->(map, tag)
    auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
    const size_t o_maps = al(sizeof(BayesChains)), o_job = o_maps + al(2 * sizeof(RayMap));
    const size_t o_rays = o_job + al(sizeof(WindowJob)), o_offs = o_rays + al(sizeof(int4) * nr);
    const size_t o_rmap = o_offs + al(sizeof(long long) * nr), total = o_rmap + al(sizeof(int) * nr);
    if (C.pin_cap < total) {
        if (C.pin) hipHostFree(C.pin);
        C.pin = nullptr;
        C.pin_cap = 0;
        if (hipHostMalloc((void**)&C.pin, 2 * total, hipHostMallocCoherent) != hipSuccess)
            throw Error(LGS_ERR_OOM, "hipHostMalloc failed");
        C.pin_cap = 2 * total;
    }
    char* pin = C.pin;
    char* d_stage = (char*)ctx->ensure(S_RAY6, total);
    const BayesChains chains = make_chains(bp->prob_hit, bp->prob_miss);
    std::memcpy(pin, &chains, sizeof(chains));
    RayMap* pm = (RayMap*)(pin + o_maps);
    pm[0] = raymap_of(latest, 0);
    if (local) pm[1] = raymap_of(local, lat_cells);
    int4* prays = (int4*)(pin + o_rays);
    long long* poffs = (long long*)(pin + o_offs);
    int* prm = (int*)(pin + o_rmap);
    long long off = 0;
    for (long long k = 0; k < nr; ++k) {
        prays[k] = rays[k];
        poffs[k] = off;
        prm[k] = (k < (long long)nrE) ? (es << 16) : 1;
        off += lens[k];
    }
    // the window after this step, oldest first, and its stamps
    std::vector<int> order = C.window;
    order.push_back(es);
    WindowJob& J = *(WindowJob*)(pin + o_job);
    std::memset(&J, 0, sizeof(J));
    for (int q : order) {
        const KeyBuf* b = (q == es) ? buf.get() : C.slot[q].buf.get();
        J.slot[q] = SlotView{ b->keys, b->bits() };
        J.st.s[q] = (q == es) ? stamp : C.slot[q].stamp;
    }
    for (size_t q = 0; q < order.size(); ++q) J.order[q] = order[q];
    J.nwin = (int)order.size();
    J.eslot = es;
    J.latest = pm[0];
    if (local) J.local = pm[1];
    J.nE = nE;
    J.nloc = nloc;
    J.lshift = lshift;
    J.ldx = ldx;
    J.ldy = ldy;
    if (evict && L.buf) {
        J.lkeys = L.buf->keys;
        J.lrb = L.buf->bits();
        J.lbeg = L.beg;
        J.nL = L.end - L.beg;
    }
    J.tbl = C.d_tbl;
    fetch_async(ctx, d_stage, pin, total);
    tm.lap(4);
    unsigned* d_keys = (unsigned*)ctx->ensure(S_RAY2, sizeof(unsigned) * (size_t)std::max(1LL, keys));
    unsigned* d_tmp = (unsigned*)ctx->ensure(S_RAY3, sizeof(unsigned) * (size_t)std::max(1LL, keys));
    if (nr > 0) {
        int tok = ctx->timing_begin(K_RAY_EMIT, 4.0 * (double)keys);
        hipLaunchKernelGGL(k_emit, dim3((unsigned)((nr + 3) / 4)), dim3(256), 0, st, (const int4*)(d_stage + o_rays),
                           (const long long*)(d_stage + o_offs), (const int*)(d_stage + o_rmap), (int)nr,
                           (const RayMap*)(d_stage + o_maps), d_keys, C.d_bad, kTagShift);
        ctx->timing_end(tok);
        LGS_HIP_CHECK(hipGetLastError());
    }
    const long long nL = J.nL;
    if (nE + nL > C.long_cap) {
        if (C.d_long) LGS_HIP_CHECK(hipFree(C.d_long));
        C.d_long = nullptr;
        C.long_cap = 0;
        const long long cap = (nE + nL) * 2 + 4096;
        if (hipMalloc(&C.d_long, sizeof(unsigned) * (size_t)(cap + 2)) != hipSuccess)
            throw Error(LGS_ERR_OOM, "hipMalloc failed for the long-run queue");
        C.long_cap = cap;
    }
    const int tok = ctx->timing_begin(K_RAY_APPLY, 4.0 * (double)(keys + nL));
    if (keys == 0) LGS_HIP_CHECK(hipMemsetAsync(C.d_long, 0, sizeof(unsigned), st));   // (k_runmask clears it)
    if (keys > 0) {
        keysort(ctx, d_keys, buf->keys, d_tmp, keys, kTagShift, bits_for(cells), C.d_bad);
        RunIndex ix{ C.d_tbl, nE, J.st, C.d_long };
        const long long nw = (keys + 63) / 64;
        hipLaunchKernelGGL(k_runmask, dim3((unsigned)((keys + 255) / 256)), dim3(256), 0, st, buf->keys, keys, 1,
                           buf->hitw, buf->endw, ix);
        hipLaunchKernelGGL(k_runsummary, dim3((unsigned)((nw + 255) / 256)), dim3(256), 0, st, buf->hitw, buf->endw,
                           nw, buf->hit2, buf->miss2, buf->end2);
    }
    const long long nthreads = nE + nloc + nL;
    if (tm.on) tm.keys += (double)keys, tm.rays += (double)nr, tm.longq += (double)nL;
    const LongList ll{ C.d_long, C.d_long + 2 };
    if (nthreads > 0) {
        hipLaunchKernelGGL(k_apply_window, dim3((unsigned)((nthreads + 255) / 256)), dim3(256), 0, st,
                           (const WindowJob*)(d_stage + o_job), (const BayesChains*)d_stage, bp->prob_hit,
                           bp->prob_miss, ll);
        hipLaunchKernelGGL(k_apply_long, dim3(512), dim3(256), 0, st, (const WindowJob*)(d_stage + o_job),
                           (const BayesChains*)d_stage, bp->prob_hit, bp->prob_miss, ll);
    }
    ctx->timing_end(tok);
    LGS_HIP_CHECK(hipGetLastError());
    record_writer(C, st, latest, local);
    tm.lap(5);
    tm.done();
    if (evict) C.retired.push_back(std::move(L.buf));
    C.slot[es] = LatestSlot{ escan->uid, epose, stamp, buf, 0, nE };
    C.window.push_back(es);
    ++C.n_incremental;
    if (ctx->profile) {
        C.finish();
        ctx->harvest();
    }
}

// GridMapBuilder::UpdateLatestMap's ConstructMapFromScans over scans[0, n)
// (:196-207, :227-332) and, with `local`, UpdateGridMap's insert of the newest
// scan into the local map (:149-186) -- AppendScan (:48-59).  The two maps are
// independent, so both ray-casts share one device pass.
void latest_rebuild(lgs_ctx* ctx, lgs_map* latest, lgs_map* local, const lgs_scan* const* scans,
                    const lgs_pose2d* poses, int n, const lgs_builder_params* bp)
{
    LatestCache& C = cache_of(latest);
    step_timing().start();
    C.finish();
    step_timing().lap(0);
    latest->ctx = ctx;
    if (local) local->ctx = ctx;
    std::vector<MapJob> jobs(local ? 2 : 1);
    jobs[0].m = latest;
    if (local) jobs[1].m = local;
    std::vector<std::array<double, 4>> box;
    if (local) hits_and_boxes(jobs, { 0, n - 1 }, { n, 1 }, scans, poses, bp, box);
    else hits_and_boxes(jobs, { 0 }, { n }, scans, poses, bp, box);
    step_timing().lap(1);
    if (local) {
        // the insert's box is the scan's own (sensor included, :346-352), not
        // ConstructMapFromScans' running box with its DBL_MIN start
        const double* bx = jobs[1].hs[0]->box;
        map_expand(local, bx[0], bx[1], bx[2], bx[3], 5.0);                // :157-158
    }
    const ResizeGeom g = resize_geom(latest, box[0][0], box[0][1], box[0][2], box[0][3]);
    const double bpv[4] = { bp->usable_range_min, bp->usable_range_max, bp->prob_hit, bp->prob_miss };
    const bool same_geom = g.pminx == 0 && g.pminy == 0 && g.npx == latest->npx && g.npy == latest->npy &&
                           C.w == latest->w && C.h == latest->h && C.min_x == latest->min_x &&
                           C.min_y == latest->min_y;
    // the new window = the cached one plus scans[n - 1], less its oldest scan (evict)
    const int k = (int)C.window.size();
    bool evict = false, shift_ok = false;
    if (C.valid && n <= kMaxWindow && (n == k || n == k + 1)) {
        evict = n == k;
        shift_ok = true;
        for (int i = 0; i + 1 < n && shift_ok; ++i) {
            const LatestSlot& sl = C.slot[C.window[i + (evict ? 1 : 0)]];
            shift_ok = sl.uid == scans[i]->uid && same_pose(sl.pose, poses[i]);
        }
    }
    if (shift_ok && same_geom && std::memcmp(bpv, C.bpv, sizeof(bpv)) == 0) {
        step_timing().lap(2);
        latest_step(ctx, C, latest, local, scans[n - 1], poses[n - 1], jobs[0].hs[n - 1], evict, bp);
        return;
    }
    // full rebuild: Resize + Reset (:288-290), every scan; re-seeds the lists
    C.drop_lists();
    map_resize_reset(latest, box[0][0], box[0][1], box[0][2], box[0][3]);
    const size_t lat_cells = (size_t)latest->w * latest->h;
    const unsigned long long cells = lat_cells + (local ? (unsigned long long)local->w * local->h : 0ull);
    const bool tagged = n <= kMaxWindow && lat_cells <= kMaxTblCells && cells < (1ull << (32 - kTagShift));
    ++C.n_full;
    if (!tagged) {
        raycast_maps(ctx, jobs, bp);
        return;
    }
    jobs[0].tags.resize((size_t)n);
    for (int i = 0; i < n; ++i) jobs[0].tags[i] = i;
    if (local) jobs[1].tags.assign(1, 0);
    TagPass tp;
    raycast_maps(ctx, jobs, bp, &tp);   // synchronises
    if (!tp.ok) return;                 // too many keys for one pass: no lists
    hipStream_t st = ctx->stream;
    if (C.tbl_cells < lat_cells) {
        if (C.d_tbl) LGS_HIP_CHECK(hipFree(C.d_tbl));
        C.d_tbl = nullptr;
        C.tbl_cells = 0;
        if (hipMalloc(&C.d_tbl, sizeof(unsigned long long) * kSlots * lat_cells) != hipSuccess)
            throw Error(LGS_ERR_OOM, "hipMalloc failed for the latest-map index");
        LGS_HIP_CHECK(hipMemsetAsync(C.d_tbl, 0, sizeof(unsigned long long) * kSlots * lat_cells, st));
        C.tbl_cells = lat_cells;
    }
    const long long nlat = tp.job_keys[0];
    KeyBufPtr boot = C.acquire(std::max(1LL, nlat));
    SlotStamps stamps{};
    long long beg = 0;
    C.window.clear();
    for (int i = 0; i < n; ++i) {
        stamps.s[i] = (unsigned)ctx->next_stamp();
        C.slot[i] = LatestSlot{ scans[i]->uid, poses[i], stamps.s[i], boot, beg, beg + tp.tag_keys[i] };
        beg += tp.tag_keys[i];
        C.window.push_back(i);
    }
    if (nlat > 0) {
        // the window's lists: the latest map's sorted keys partitioned by slot
        // (stable: each slot's keys stay in cell order), runs of (cell, slot)
        keysort(ctx, tp.sorted, boot->keys, nullptr, nlat, 1, 4, C.d_bad);
        const long long nw = (nlat + 63) / 64;
        hipLaunchKernelGGL(k_runmask, dim3((unsigned)((nlat + 255) / 256)), dim3(256), 0, st, boot->keys, nlat, 1,
                           boot->hitw, boot->endw, RunIndex{ C.d_tbl, nlat, stamps });
        hipLaunchKernelGGL(k_runsummary, dim3((unsigned)((nw + 255) / 256)), dim3(256), 0, st, boot->hitw,
                           boot->endw, nw, boot->hit2, boot->miss2, boot->end2);
        LGS_HIP_CHECK(hipGetLastError());
    }
    *C.h_bad = 0;
    C.w = latest->w;
    C.h = latest->h;
    C.min_x = latest->min_x;
    C.min_y = latest->min_y;
    std::memcpy(C.bpv, bpv, sizeof(bpv));
    C.valid = true;
    record_writer(C, st, latest, local);
}

}  // namespace

extern "C" int lgs_map_create(lgs_ctx* ctx, double res, int ps, int ncx, int ncy, double cx, double cy,
                              lgs_map** out)
{
    if (!ctx || !out) return LGS_ERR_INVALID_ARG;
    *out = nullptr;
    return guarded(ctx, [&] {
        LGS_REQUIRE(res > 0.0 && ps > 0, "invalid map resolution / patch size");
        LGS_HIP_CHECK(hipSetDevice(ctx->device));
        // GridMap(res, patchSize, numCellsX, numCellsY, centerPos) (:337-391)
        lgs_map* m = new lgs_map();
        m->ctx = ctx;
        m->device = ctx->device;
        m->res = res;
        m->ps = ps;
        ncx = std::max(0, ncx);
        ncy = std::max(0, ncy);
        m->npx = (int)std::ceil((double)ncx / (double)ps);
        m->npy = (int)std::ceil((double)ncy / (double)ps);
        m->w = m->npx * ps;
        m->h = m->npy * ps;
        const double offX = (m->w % 2 == 0) ? (double)(m->w / 2) : ((double)(m->w / 2) + 0.5);
        const double offY = (m->h % 2 == 0) ? (double)(m->h / 2) : ((double)(m->h / 2) + 0.5);
        m->min_x = cx - offX * res;
        m->min_y = cy - offY * res;
        try {
            map_alloc(m, m->w, m->h, &m->d_cells, &m->d_hit, &m->d_miss);
            m->cap = std::max<size_t>(1, (size_t)m->w * m->h);
            palloc_init(m);
        } catch (...) {
            map_free(m);
            palloc_free(m);
            delete m;
            throw;
        }
        map_sync_view(m);
        *out = m;
    });
}

extern "C" void lgs_map_destroy(lgs_map* m)
{
    if (!m) return;
    hipSetDevice(m->device);
    if (m->cache) {
        if (m->cache->pending) {
            try {
                m->cache->wev->wait();
            } catch (...) {
                hipStreamSynchronize(m->cache->wev->st.load());
            }
        }
        delete m->cache;
        m->cache = nullptr;
    }
    map_free(m);
    palloc_free(m);
    delete m;
}

extern "C" int lgs_map_get_geometry(const lgs_map* m, lgs_map_geometry* g)
{
    if (!m || !g) return LGS_ERR_INVALID_ARG;
    g->resolution = m->res;
    g->patch_size = m->ps;
    g->num_patches_x = m->npx;
    g->num_patches_y = m->npy;
    g->num_cells_x = m->w;
    g->num_cells_y = m->h;
    g->min_x = m->min_x;
    g->min_y = m->min_y;
    return LGS_OK;
}

extern "C" int lgs_map_grid(lgs_map* m, lgs_grid** out)
{
    if (!m || !out) return LGS_ERR_INVALID_ARG;
    *out = &m->view;
    return LGS_OK;
}

extern "C" int lgs_map_update_scan(lgs_ctx* ctx, lgs_map* m, const lgs_scan* scan, lgs_pose2d robot,
                                   const lgs_builder_params* bp)
{
    if (!ctx || !m || !scan || !bp) return LGS_ERR_INVALID_ARG;
    return guarded(ctx, [&] {
        LGS_HIP_CHECK(hipSetDevice(ctx->device));
        m->ctx = ctx;
        invalidate_cache(m);
        std::vector<HitsPtr> hs(1, cached_hits(scan, robot, bp, true));
        // bounding box starts at the sensor position (:346-352)
        const double* bx = hs[0]->box;
        map_expand(m, bx[0], bx[1], bx[2], bx[3], 5.0);  // :157-158 (default enlargeStep)
        raycast(m, std::move(hs), bp);
    });
}

extern "C" int lgs_map_construct_from_scans(lgs_ctx* ctx, lgs_map* m, const lgs_scan* const* scans,
                                            const lgs_pose2d* poses, int n,
                                            const lgs_builder_params* bp)
{
    if (!ctx || !m || !bp || n < 0 || (n > 0 && (!scans || !poses))) return LGS_ERR_INVALID_ARG;
    return guarded(ctx, [&] {
        LGS_HIP_CHECK(hipSetDevice(ctx->device));
        m->ctx = ctx;
        latest_rebuild(ctx, m, nullptr, scans, poses, n, bp);   // :227-332
    });
}

extern "C" int lgs_map_append_scan(lgs_ctx* ctx, lgs_map* local, lgs_map* latest, const lgs_scan* const* scans,
                                   const lgs_pose2d* poses, int n, const lgs_builder_params* bp)
{
    if (!ctx || !local || !latest || local == latest || !scans || !poses || !bp || n < 1)
        return LGS_ERR_INVALID_ARG;
    return guarded(ctx, [&] {
        LGS_HIP_CHECK(hipSetDevice(ctx->device));
        // GridMapBuilder::AppendScan (:48-59) = UpdateGridMap's insert of the
        // newest scan into the local map (:149-186) + UpdateLatestMap's
        // ConstructMapFromScans over the last n scans (:196-207)
        invalidate_cache(local);
        latest_rebuild(ctx, latest, local, scans, poses, n, bp);
    });
}

extern "C" int lgs_maps_construct_from_scans(lgs_ctx* ctx, lgs_map* const* maps, const int* idx_min,
                                             const int* idx_max, int n_maps, const lgs_scan* const* scans,
                                             const lgs_pose2d* poses, int n_nodes,
                                             const lgs_builder_params* bp)
{
    if (!ctx || !bp || n_maps < 0 || n_nodes < 0) return LGS_ERR_INVALID_ARG;
    if (n_maps > 0 && (!maps || !idx_min || !idx_max || !scans || !poses)) return LGS_ERR_INVALID_ARG;
    for (int i = 0; i < n_maps; ++i) {
        if (!maps[i] || idx_min[i] < 0 || idx_min[i] > idx_max[i] || idx_max[i] >= n_nodes)
            return LGS_ERR_INVALID_ARG;
        for (int j = 0; j < i; ++j)
            if (maps[j] == maps[i]) return LGS_ERR_INVALID_ARG;
    }
    return guarded(ctx, [&] {
        LGS_HIP_CHECK(hipSetDevice(ctx->device));
        for (int i = 0; i < n_maps; ++i) invalidate_cache(maps[i]);
        // AfterLoopClosure (:66-74): ConstructMapFromScans per local map; the
        // geometry of each is fixed before any ray is cast, so the ray-casts
        // of all maps run as one pass over the maps in order
        std::vector<MapJob> jobs(n_maps);
        std::vector<int> first(n_maps), count(n_maps);
        for (int i = 0; i < n_maps; ++i) {
            maps[i]->ctx = ctx;
            jobs[i].m = maps[i];
            first[i] = idx_min[i];
            count[i] = idx_max[i] - idx_min[i] + 1;
        }
        // LGS_F2_TIMING=1: host phases of each call on stderr (diagnostics)
        static const bool timing = std::getenv("LGS_F2_TIMING") != nullptr;
        const auto t0 = std::chrono::steady_clock::now();
        if (ctx->device_hits && construct_maps_device(ctx, maps, first.data(), count.data(), n_maps, scans, poses, bp)) {
            if (timing)
                std::fprintf(stderr, "f2 call us (device hits): %.1f\n",
                             std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
            return;
        }
        std::vector<std::array<double, 4>> box;
        hits_and_boxes(jobs, first, count, scans, poses, bp, box);
        const auto t1 = std::chrono::steady_clock::now();
        for (int i = 0; i < n_maps; ++i) map_resize_reset(maps[i], box[i][0], box[i][1], box[i][2], box[i][3]);
        const auto t2 = std::chrono::steady_clock::now();
        raycast_maps(ctx, jobs, bp);
        if (timing) {
            const auto t3 = std::chrono::steady_clock::now();
            auto us = [](auto a, auto b) { return std::chrono::duration<double, std::micro>(b - a).count(); };
            std::fprintf(stderr, "f2 call us: hits %.1f resize %.1f raycast(+sync) %.1f\n", us(t0, t1), us(t1, t2),
                         us(t2, t3));
        }
    });
}

extern "C" int lgs_map_construct_global(lgs_ctx* ctx, double res, int ps, const lgs_scan* const* scans,
                                        const lgs_pose2d* poses, int n, const lgs_builder_params* bp,
                                        lgs_map** out)
{
    if (!ctx || !bp || !out || n < 0 || (n > 0 && (!scans || !poses))) return LGS_ERR_INVALID_ARG;
    *out = nullptr;
    lgs_map* m = nullptr;
    // GridMapType gridMap { res, patchSize, 0, 0, Point2D(0, 0) } (:89-90)
    int rc = lgs_map_create(ctx, res, ps, 0, 0, 0.0, 0.0, &m);
    if (rc != LGS_OK) return rc;
    // :91, with the hit points and ray cells on the device (the map is new:
    // no latest-map window to keep)
    bool done = false;
    if (ctx->device_hits && n > 0) {
        rc = guarded(ctx, [&] {
            LGS_HIP_CHECK(hipSetDevice(ctx->device));
            m->ctx = ctx;
            const int f = 0;
            done = construct_maps_device(ctx, &m, &f, &n, 1, scans, poses, bp);
        });
        if (rc != LGS_OK) {
            lgs_map_destroy(m);
            return rc;
        }
    }
    if (!done) rc = lgs_map_construct_from_scans(ctx, m, scans, poses, n, bp);
    if (rc != LGS_OK) {
        lgs_map_destroy(m);
        return rc;
    }
    *out = m;
    return LGS_OK;
}

extern "C" int lgs_map_render_gray(lgs_ctx* ctx, const lgs_map* m, uint8_t* image)
{
    if (!ctx || !m || !image) return LGS_ERR_INVALID_ARG;
    return guarded(ctx, [&] {
        const size_t n = (size_t)m->w * m->h;
        if (!n) return;
        LGS_HIP_CHECK(hipSetDevice(ctx->device));
        grid_acquire(ctx, &m->view);
        hipStream_t st = ctx->stream;
        uint8_t* d_img = (uint8_t*)ctx->ensure(S_RAY2, n);
        const long long threads = (long long)((m->w + 3) / 4) * m->h;
        hipLaunchKernelGGL(k_render_gray, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, st, m->d_cells,
                           m->w, 0, 0, m->w, m->h, 1, d_img);
        LGS_HIP_CHECK(hipGetLastError());
        LGS_HIP_CHECK(hipMemcpyAsync(image, d_img, n, hipMemcpyDeviceToHost, st));
        LGS_HIP_CHECK(hipStreamSynchronize(st));
    });
}

extern "C" int lgs_map_download(lgs_ctx* ctx, const lgs_map* m, double* cells, uint32_t* hit,
                                uint32_t* miss)
{
    if (!ctx || !m) return LGS_ERR_INVALID_ARG;
    return guarded(ctx, [&] {
        const size_t n = (size_t)m->w * m->h;
        if (!n) return;
        hipStream_t st = ctx->stream;
        grid_acquire(ctx, &m->view);
        if (cells)
            LGS_HIP_CHECK(hipMemcpyAsync(cells, m->d_cells, n * sizeof(double), hipMemcpyDeviceToHost, st));
        if (hit)
            LGS_HIP_CHECK(hipMemcpyAsync(hit, m->d_hit, n * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
        if (miss)
            LGS_HIP_CHECK(hipMemcpyAsync(miss, m->d_miss, n * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
        LGS_HIP_CHECK(hipStreamSynchronize(st));
    });
}

extern "C" int lgs_map_render_gray_region(lgs_ctx* ctx, const lgs_map* m, int x0, int y0, int w, int h,
                                          int flip_rows, uint8_t* image)
{
    if (!ctx || !m || !image || x0 < 0 || y0 < 0 || w < 0 || h < 0 || x0 + (long long)w > m->w ||
        y0 + (long long)h > m->h)
        return LGS_ERR_INVALID_ARG;
    return guarded(ctx, [&] {
        const size_t n = (size_t)w * h;
        if (!n) return;
        LGS_HIP_CHECK(hipSetDevice(ctx->device));
        grid_acquire(ctx, &m->view);
        hipStream_t st = ctx->stream;
        uint8_t* d_img = (uint8_t*)ctx->ensure(S_RAY2, n);
        const long long threads = (long long)((w + 3) / 4) * h;
        hipLaunchKernelGGL(k_render_gray, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, st, m->d_cells,
                           m->w, x0, y0, w, h, flip_rows ? 1 : 0, d_img);
        LGS_HIP_CHECK(hipGetLastError());
        LGS_HIP_CHECK(hipMemcpyAsync(image, d_img, n, hipMemcpyDeviceToHost, st));
        LGS_HIP_CHECK(hipStreamSynchronize(st));
    });
}

extern "C" int lgs_map_download_patches(lgs_ctx* ctx, const lgs_map* m, uint8_t* flags)
{
    if (!ctx || !m || !flags) return LGS_ERR_INVALID_ARG;
    return guarded(ctx, [&] {
        const size_t n = (size_t)m->npx * m->npy;
        if (!n) return;
        LGS_HIP_CHECK(hipSetDevice(ctx->device));
        grid_acquire(ctx, &m->view);
        LGS_HIP_CHECK(hipMemcpyAsync(flags, m->d_palloc, n, hipMemcpyDeviceToHost, ctx->stream));
        LGS_HIP_CHECK(hipStreamSynchronize(ctx->stream));
    });
}

extern "C" int lgs_map_actual_size(lgs_ctx* ctx, const lgs_map* m, int* num_allocated, int* out)
{
    if (!ctx || !m || !num_allocated || !out) return LGS_ERR_INVALID_ARG;
    std::vector<uint8_t> f((size_t)m->npx * m->npy);
    const int rc = f.empty() ? LGS_OK : lgs_map_download_patches(ctx, m, f.data());
    if (rc != LGS_OK) return rc;
    // GridMap::ComputeActualMapSize (H/grid_map/grid_map.hpp:969-1015)
    int pminx = INT_MAX, pminy = INT_MAX, pmaxx = INT_MIN, pmaxy = INT_MIN, n = 0;
    for (int y = 0; y < m->npy; ++y)
        for (int x = 0; x < m->npx; ++x)
            if (f[(size_t)y * m->npx + x]) {
                ++n;
                pminx = std::min(pminx, x);
                pminy = std::min(pminy, y);
                pmaxx = std::max(pmaxx, x);
                pmaxy = std::max(pmaxy, y);
            }
    *num_allocated = n;
    for (int i = 0; i < 12; ++i) out[i] = 0;
    if (!n) return LGS_OK;
    const int ps = m->ps;
    out[0] = pminx, out[1] = pminy, out[2] = pmaxx + 1, out[3] = pmaxy + 1;                 // patchIdxMin/Max
    out[4] = pminx * ps, out[5] = pminy * ps, out[6] = pmaxx * ps + ps, out[7] = pmaxy * ps + ps;  // :918-929
    out[8] = out[2] - out[0], out[9] = out[3] - out[1];                                     // mapSizeInPatches
    out[10] = out[6] - out[4], out[11] = out[7] - out[5];                                   // mapSizeInGridCells
    return LGS_OK;
}

extern "C" int lgs_debug_map_rebuilds(const lgs_map* m, long long* incremental, long long* full)
{
    if (!m || !incremental || !full) return LGS_ERR_INVALID_ARG;
    *incremental = m->cache ? m->cache->n_incremental : 0;
    *full = m->cache ? m->cache->n_full : 0;
    return LGS_OK;
}
