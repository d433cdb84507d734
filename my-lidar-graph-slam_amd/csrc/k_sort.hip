// k_sort.hip -- K3 sort: stable LSD radix sort of the ray-cast keys on MI355X.
//
// The ordered Bayes update (C/mapping/grid_map_builder.cpp:170-186 and
// :292-329) needs every cell's updates in ray order.  k_emit writes one 32-bit
// key per visited cell in ray order; a STABLE sort on the cell bits of the keys
// makes each cell's updates one contiguous run that keeps that order.
//
//   k_sort_hist   one read of the keys: the digit histograms of every pass
//                 (LDS, then device-scope atomics); the last workgroup turns
//                 them into each pass's exclusive digit offsets and clears the
//                 accumulators for the next sort (the control block stays zero
//                 between sorts, no memset per call)
//   k_sort_pass   one launch per digit (<= 8 bits): tiles of 256 x KPT keys
//                 taken in ticket order; per wave a stable rank of each key
//                 among equal digits (LDS peer masks), per tile the digit
//                 counts published as aggregates and turned into inclusive
//                 prefixes by a decoupled look-back over earlier tiles (status
//                 words tagged with a per-pass stamp: no clearing); keys are
//                 reordered by digit in LDS and written out in digit runs
//
// Each workgroup only waits on tiles with lower tickets, which belong to
// workgroups that started before it, so the look-back always drains.
//
//   k_sort_wide   sorts that fit the device at once: every pass in one
//                 launch, 8192-key tiles, digits of up to 10 bits, ranks from
//                 per-wave LDS peer masks, grid barriers around the count
//                 exchange (a config-4 step's ~160k keys, 20 cell bits: 20
//                 workgroups, 2 passes)
#include "lgs_internal.hpp"

#include <algorithm>

namespace {

constexpr int kSortThreads = 256;
constexpr int kSortRadix = 256;        // bins per pass (digits of at most 8 bits)
constexpr int kSortMaxPasses = 4;
// control block (unsigned words, S_RAY0): zero between sorts
constexpr int kHistLanes = 8;                                // accumulator copies (workgroup % 8): less contention
constexpr int kCtlHist = 0;                                  // [lane][pass][256] accumulators
constexpr int kCtlDone = kHistLanes * kSortMaxPasses * kSortRadix;   // workgroups finished k_sort_hist
constexpr int kCtlTicket = kCtlDone + 1;                     // [pass] tile tickets
constexpr int kCtlBar = kCtlDone + 8;                        // k_sort_wide grid barrier, workgroups done
constexpr int kCtlOffs = kCtlDone + 64;                      // [pass][256] exclusive digit offsets
constexpr int kCtlWords = kCtlOffs + kSortMaxPasses * kSortRadix;

constexpr unsigned long long kFlagAgg = 1ull << 30, kFlagPrefix = 2ull << 30;
constexpr int kHistRun = 16;          // consecutive keys per thread in k_sort_hist
constexpr int kLookback = 16;         // predecessor tiles read at once in the look-back
constexpr unsigned long long kCountMask = (1ull << 30) - 1;

__device__ __forceinline__ unsigned ld_agent(const unsigned* p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ __launch_bounds__(kSortThreads) void k_sort_hist(const unsigned* __restrict__ keys, long long n, int lo,
                                                            int dbits, int bits, int passes,
                                                            unsigned* __restrict__ ctl)
{
    __shared__ unsigned h[kSortMaxPasses][kSortRadix];
    __shared__ int last;
    const int tid = threadIdx.x;
    for (int p = 0; p < passes; ++p) h[p][tid] = 0;
    __syncthreads();
    // each thread counts kHistRun consecutive keys per chunk; equal digits of
    // neighbouring keys (ray-ordered keys share their high digits) are
    // counted in a register and added to LDS once per run
    const long long stride = (long long)gridDim.x * kSortThreads * kHistRun;
    for (long long i0 = ((long long)blockIdx.x * kSortThreads + tid) * kHistRun; i0 < n; i0 += stride) {
        const int m = (int)min((long long)kHistRun, n - i0);
        unsigned k[kHistRun];
#pragma unroll
        for (int q = 0; q < kHistRun; ++q) k[q] = (q < m) ? keys[i0 + q] : 0u;
        for (int p = 0; p < passes; ++p) {
            const int sh = lo + p * dbits;
            const unsigned mask = (1u << min(dbits, bits - p * dbits)) - 1u;
            unsigned cur = (k[0] >> sh) & mask, cnt = 0;
#pragma unroll
            for (int q = 0; q < kHistRun; ++q) {
                const unsigned d = (k[q] >> sh) & mask;
                if (q < m && d != cur) {
                    atomicAdd(&h[p][cur], cnt);
                    cur = d, cnt = 0;
                }
                cnt += (q < m) ? 1u : 0u;
            }
            atomicAdd(&h[p][cur], cnt);
        }
    }
    __syncthreads();
    unsigned* acc = ctl + kCtlHist + (blockIdx.x % kHistLanes) * kSortMaxPasses * kSortRadix;
    for (int p = 0; p < passes; ++p)
        if (h[p][tid]) __hip_atomic_fetch_add(acc + p * kSortRadix + tid, h[p][tid], __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT);
    __threadfence();
    __syncthreads();
    if (tid == 0)
        last = __hip_atomic_fetch_add(ctl + kCtlDone, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) ==
               gridDim.x - 1;
    __syncthreads();
    if (!last) return;
    __threadfence();
    // last workgroup: exclusive scan of each pass's histogram (one wave per
    // pass, 4 digits per lane), then clear the accumulators and counters
    const int w = tid >> 6, lane = tid & 63;
    if (w < passes) {
        unsigned v[4], s = 0;
        for (int j = 0; j < 4; ++j) {
            v[j] = 0;
            for (int l = 0; l < kHistLanes; ++l)
                v[j] += ld_agent(ctl + kCtlHist + (l * kSortMaxPasses + w) * kSortRadix + lane * 4 + j);
            s += v[j];
        }
        unsigned incl = s;
        for (int o = 1; o < 64; o <<= 1) {
            const unsigned t = __shfl_up(incl, o);
            if (lane >= o) incl += t;
        }
        unsigned run = incl - s;
        for (int j = 0; j < 4; ++j) {
            ctl[kCtlOffs + w * kSortRadix + lane * 4 + j] = run;
            run += v[j];
        }
    }
    __syncthreads();
    for (int l = 0; l < kHistLanes; ++l)
        for (int p = 0; p < passes; ++p)
            __hip_atomic_store(ctl + kCtlHist + (l * kSortMaxPasses + p) * kSortRadix + tid, 0u, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
    if (tid <= kSortMaxPasses)
        __hip_atomic_store(ctl + kCtlDone + tid, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int KPT>
__global__ __launch_bounds__(kSortThreads) void k_sort_pass(const unsigned* __restrict__ in,
                                                            unsigned* __restrict__ out, long long n, int shift,
                                                            int nb, const unsigned* __restrict__ offs,
                                                            unsigned long long* __restrict__ status,
                                                            unsigned* __restrict__ ticket, unsigned stamp)
{
    constexpr int TILE = kSortThreads * KPT;
    __shared__ unsigned keys_s[TILE];
    __shared__ unsigned wcnt[4][kSortRadix];
    __shared__ unsigned dstart[kSortRadix];
    __shared__ unsigned gbase[kSortRadix];
    __shared__ unsigned wsum[4];
    __shared__ unsigned tile_s;
    __shared__ unsigned long long wmask[4][kSortRadix];   // per-wave peer masks (k_sort_wide)
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    const unsigned mask = (1u << nb) - 1u;
    wcnt[0][tid] = wcnt[1][tid] = wcnt[2][tid] = wcnt[3][tid] = 0;
    wmask[0][tid] = wmask[1][tid] = wmask[2][tid] = wmask[3][tid] = 0ull;
    if (tid == 0) tile_s = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    const long long tile = tile_s;
    const long long t0 = tile * TILE;
    // wave w ranks tile positions [w * 64 KPT, (w + 1) * 64 KPT) in order
    unsigned k[KPT], rank[KPT];
    const long long p0 = t0 + (long long)w * 64 * KPT + lane;
#pragma unroll
    for (int i = 0; i < KPT; ++i) {
        const long long p = p0 + 64 * i;
        k[i] = (p < n) ? in[p] : 0u;
    }
    const unsigned long long me = 1ull << lane, lt = me - 1ull;
    unsigned long long* mw = wmask[w];
#pragma unroll
    for (int i = 0; i < KPT; ++i) {
        const bool valid = p0 + 64 * i < n;
        const unsigned d = (k[i] >> shift) & mask;
        unsigned long long peers = 0;
        if (valid) {
            __hip_atomic_fetch_or(&mw[d], me, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            peers = __hip_atomic_load(&mw[d], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        const unsigned base = valid ? wcnt[w][d] : 0u;
        rank[i] = base + (unsigned)__popcll(peers & lt);
        if (valid && !(peers & lt)) {
            wcnt[w][d] = base + (unsigned)__popcll(peers);
            __hip_atomic_store(&mw[d], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
    }
    __syncthreads();
    // per digit: exclusive prefix over the waves, tile total, publication
    const int d = tid;
    const unsigned c0 = wcnt[0][d], c1 = wcnt[1][d], c2 = wcnt[2][d], c3 = wcnt[3][d];
    const unsigned tot = c0 + c1 + c2 + c3;
    wcnt[0][d] = 0;
    wcnt[1][d] = c0;
    wcnt[2][d] = c0 + c1;
    wcnt[3][d] = c0 + c1 + c2;
    const unsigned long long tag = (unsigned long long)stamp << 32;
    unsigned long long* st = status + (size_t)tile * kSortRadix + d;
    __hip_atomic_store(st, tag | (tile == 0 ? kFlagPrefix : kFlagAgg) | tot, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
    // tile-local digit starts: exclusive scan of tot over the 256 digits
    unsigned incl = tot;
    for (int o = 1; o < 64; o <<= 1) {
        const unsigned t = __shfl_up(incl, o);
        if (lane >= o) incl += t;
    }
    if (lane == 63) wsum[w] = incl;
    // decoupled look-back over the earlier tiles
    // (kLookback predecessors per round, loads in flight together; a round
    // consumes tiles up to the first one not yet published)
    unsigned excl = 0;
    if (tile > 0) {
        long long j = tile - 1;
        for (bool done = false; !done;) {
            unsigned long long v[kLookback];
#pragma unroll
            for (int q = 0; q < kLookback; ++q)
                v[q] = (j - q >= 0) ? __hip_atomic_load(status + (size_t)(j - q) * kSortRadix + d, __ATOMIC_RELAXED,
                                                        __HIP_MEMORY_SCOPE_AGENT)
                                    : 0ull;
            int used = 0;
            bool stop = false;   // at the first unpublished tile, or after a prefix
#pragma unroll
            for (int q = 0; q < kLookback; ++q) {
                const bool ready = (v[q] >> 32) == stamp && (v[q] & (kFlagAgg | kFlagPrefix));
                if (!stop && ready) {
                    excl += (unsigned)(v[q] & kCountMask);
                    used = q + 1;
                    done = (v[q] & kFlagPrefix) != 0;
                }
                stop = stop || !ready || done;
            }
            j -= used;
            if (!done && used == 0) __builtin_amdgcn_s_sleep(1);
        }
        __hip_atomic_store(st, tag | kFlagPrefix | (excl + tot), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    gbase[d] = offs[d] + excl;
    __syncthreads();
    unsigned wo = 0;
    for (int q = 0; q < w; ++q) wo += wsum[q];
    dstart[d] = wo + incl - tot;
    __syncthreads();
    // reorder the tile by digit in LDS (stable), then write digit runs
#pragma unroll
    for (int i = 0; i < KPT; ++i)
        if (p0 + 64 * i < n) {
            const unsigned dd = (k[i] >> shift) & mask;
            keys_s[dstart[dd] + wcnt[w][dd] + rank[i]] = k[i];
        }
    __syncthreads();
    const int nvalid = (int)min((long long)TILE, n - t0);
    for (int j = tid; j < nvalid; j += kSortThreads) {
        const unsigned key = keys_s[j];
        const unsigned dd = (key >> shift) & mask;
        out[gbase[dd] + (unsigned)j - dstart[dd]] = key;
    }
}

// Small sorts (every tile resident at once): all passes in ONE launch.  Each
// workgroup ranks its tile as k_sort_pass does, stores its digit counts,
// waits at a grid barrier, reads every tile's counts (digit totals and the
// counts of the tiles before it: the same offsets a histogram and a look-back
// give), scatters, and waits again before the next pass reads the keys.
// Stores are released and loads acquired at agent scope around each barrier
// (the tiles live on different XCDs, each with its own L2).
__device__ __forceinline__ void grid_barrier(unsigned* bar, unsigned target)
{
    __syncthreads();
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        __hip_atomic_fetch_add(bar, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        while (__hip_atomic_load(bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target)
            __builtin_amdgcn_s_sleep(1);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }
    __syncthreads();
}

// Wide tiles for the cooperative sort: 512 threads x 16 keys (8192 keys per
// tile), digits of up to 10 bits.  A config-4 step's ~160k keys are then 20
// tiles and 20 cell bits take 2 passes -- the cross-XCD barriers and count
// exchange, not the key traffic, are the cost of a small sort.
//
// Ranking: a key's peers (the lanes of its wave with the same digit) come
// from a per-wave LDS mask table -- every lane ORs its lane bit into
// mask[digit], reads the word back and the lowest peer clears it -- instead
// of one ballot per digit bit (10 ballots and 64-bit selects per key made the
// ranking VALU-bound: 12.8 of a pass's ~27 us on 10 CUs).  A wave's LDS
// instructions execute in order, so the read sees every lane's OR and the
// next key's ORs see the clear.
constexpr int kWideThreads = 512, kWideKPT = 16, kWideTile = kWideThreads * kWideKPT;
template <int RB>
__global__ __launch_bounds__(kWideThreads) void k_sort_wide(const unsigned* __restrict__ in,
                                                            unsigned* __restrict__ out, unsigned* __restrict__ tmp,
                                                            long long n, int lo, int dbits, int bits, int passes,
                                                            unsigned* __restrict__ counts,
                                                            unsigned* __restrict__ bar)
{
    constexpr int NT = kWideThreads, NW = NT / 64, KPT = kWideKPT, TILE = kWideTile;
    constexpr int R = 1 << RB;
    constexpr int Q = R >= NT ? R / NT : 1;   // digits per digit-owning thread
    constexpr int ND = R / Q;                 // digit-owning threads (whole waves)
    static_assert(ND % 64 == 0 && ND <= NT, "digit threads");
    __shared__ unsigned keys_s[TILE];
    __shared__ unsigned wcnt[NW][R];
    __shared__ unsigned long long wmask[NW][R];
    __shared__ unsigned dstart[R];
    __shared__ unsigned gbase[R];
    __shared__ unsigned wsa[NW], wsb[NW];
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    const unsigned ntiles = gridDim.x, tile = blockIdx.x;
    const long long t0 = (long long)tile * TILE;
    const long long p0 = t0 + (long long)w * 64 * KPT + lane;
    const unsigned long long me = 1ull << lane, lt = me - 1ull;
    const bool dig = tid < ND;
    const int d0 = tid * Q;   // this thread's first digit
    unsigned nbar = 0;
    LGS_PROBE_DECL;
    LGS_PROBE_MARK();
    for (int i = tid; i < NW * R; i += NT) (&wmask[0][0])[i] = 0ull;
    for (int p = 0; p < passes; ++p) {
        const unsigned* src = (p == 0) ? in : (((passes - p) % 2 == 1) ? tmp : out);
        unsigned* dst = ((passes - 1 - p) % 2 == 0) ? out : tmp;
        const int shift = lo + p * dbits;
        const int nb = min(dbits, bits - p * dbits);
        const unsigned mask = (1u << nb) - 1u;
        for (int i = tid; i < NW * R; i += NT) (&wcnt[0][0])[i] = 0;
        __syncthreads();
        unsigned k[KPT], rank[KPT];
#pragma unroll
        for (int i = 0; i < KPT; ++i) {
            const long long q = p0 + 64 * i;
            k[i] = (q < n) ? src[q] : 0u;
        }
#ifdef LGS_PROBE
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
        LGS_PROBE_MARK();
        unsigned* cw = wcnt[w];
        unsigned long long* mw = wmask[w];
#pragma unroll
        for (int i = 0; i < KPT; ++i) {
            const bool valid = p0 + 64 * i < n;
            const unsigned d = (k[i] >> shift) & mask;
            unsigned long long peers = 0;
            if (valid) {
                __hip_atomic_fetch_or(&mw[d], me, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                peers = __hip_atomic_load(&mw[d], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
            const unsigned base = valid ? cw[d] : 0u;
            rank[i] = base + (unsigned)__popcll(peers & lt);
            if (valid && !(peers & lt)) {   // the lowest peer: the digit's count, and clear the mask
                cw[d] = base + (unsigned)__popcll(peers);
                __hip_atomic_store(&mw[d], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
        }
        __syncthreads();
        LGS_PROBE_MARK();
        // this thread's digits: exclusive prefix over the waves, the tile's
        // counts (published), the tile-local digit starts
        unsigned* cp = counts + (size_t)p * ntiles * R;
        unsigned tot[Q], tsum = 0, incl = 0;
        if (dig) {
#pragma unroll
            for (int j = 0; j < Q; ++j) {
                unsigned c = 0;
#pragma unroll
                for (int q = 0; q < NW; ++q) {
                    const unsigned v = wcnt[q][d0 + j];
                    wcnt[q][d0 + j] = c;
                    c += v;
                }
                tot[j] = c;
                tsum += c;
                cp[(size_t)tile * R + d0 + j] = c;
            }
            incl = tsum;
            for (int o = 1; o < 64; o <<= 1) {
                const unsigned t = __shfl_up(incl, o);
                if (lane >= o) incl += t;
            }
            if (lane == 63) wsa[w] = incl;
        }
        __syncthreads();
        if (dig) {
            unsigned run = incl - tsum;
            for (int q = 0; q < w; ++q) run += wsa[q];
#pragma unroll
            for (int j = 0; j < Q; ++j) {
                dstart[d0 + j] = run;
                run += tot[j];
            }
        }
        __syncthreads();
        LGS_PROBE_MARK();
        // reorder the tile by digit in LDS (tile-local offsets: before the
        // barrier, so the keys and ranks need not live across it)
#pragma unroll
        for (int i = 0; i < KPT; ++i)
            if (p0 + 64 * i < n) {
                const unsigned dd = (k[i] >> shift) & mask;
                keys_s[dstart[dd] + cw[dd] + rank[i]] = k[i];
            }
        LGS_PROBE_MARK();
        grid_barrier(bar, ++nbar * ntiles);
        LGS_PROBE_MARK();
        // digit totals over all tiles and the counts of the tiles before this one
        unsigned all[Q], before[Q], asum = 0, incl2 = 0;
        if (dig) {
#pragma unroll
            for (int j = 0; j < Q; ++j) all[j] = before[j] = 0;
            constexpr int B = 16 / Q;   // tiles per round: 16 loads in flight
            for (unsigned tc = 0; tc < ntiles; tc += B) {
                unsigned c[Q][B];
#pragma unroll
                for (int q = 0; q < B; ++q)
#pragma unroll
                    for (int j = 0; j < Q; ++j) c[j][q] = (tc + q < ntiles) ? cp[(size_t)(tc + q) * R + d0 + j] : 0u;
#pragma unroll
                for (int q = 0; q < B; ++q)
#pragma unroll
                    for (int j = 0; j < Q; ++j) {
                        all[j] += c[j][q];
                        before[j] += (tc + q < tile) ? c[j][q] : 0u;
                    }
            }
#pragma unroll
            for (int j = 0; j < Q; ++j) asum += all[j];
            incl2 = asum;
            for (int o = 1; o < 64; o <<= 1) {
                const unsigned t = __shfl_up(incl2, o);
                if (lane >= o) incl2 += t;
            }
            if (lane == 63) wsb[w] = incl2;
        }
        __syncthreads();
        if (dig) {
            unsigned run = incl2 - asum;
            for (int q = 0; q < w; ++q) run += wsb[q];
#pragma unroll
            for (int j = 0; j < Q; ++j) {
                gbase[d0 + j] = run + before[j];
                run += all[j];
            }
        }
        __syncthreads();
        LGS_PROBE_MARK();
        const int nvalid = (int)max(0LL, min((long long)TILE, n - t0));
        for (int j = tid; j < nvalid; j += NT) {
            const unsigned key = keys_s[j];
            const unsigned dd = (key >> shift) & mask;
            dst[gbase[dd] + (unsigned)j - dstart[dd]] = key;
        }
        if (p + 1 < passes) grid_barrier(bar, ++nbar * ntiles);
        LGS_PROBE_MARK();
    }
    LGS_PROBE_PRINT("k_sort_wide");
    __syncthreads();
    if (tid == 0 &&
        __hip_atomic_fetch_add(bar + 1, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == ntiles - 1) {
        __hip_atomic_store(bar, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(bar + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

}  // namespace

namespace lgs {

// Workgroups of k_sort_wide the device holds at once (all its tiles must be
// resident: they wait for each other), with a margin for other streams' work.
long long coop_capacity(lgs_ctx* ctx)
{
    static long long cap[64] = {};
    const int dev = ctx->device;
    if (dev < 0 || dev >= 64) return 0;
    if (!cap[dev]) {
        int per_cu = 0, cus = 0;
        LGS_HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_sort_wide<10>, kWideThreads, 0));
        LGS_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
        cap[dev] = std::max(1LL, (long long)per_cu * cus / 2);
    }
    return cap[dev];
}

// Stable sort of n 32-bit keys on bits [lo, lo + bits).  `tmp` (n keys) is
// needed when the sort takes two or more passes; in, tmp and out are distinct.
void keysort(lgs_ctx* ctx, const unsigned* in, unsigned* out, unsigned* tmp, long long n, int lo, int bits)
{
    hipStream_t st = ctx->stream;
    LGS_REQUIRE(n >= 0 && n < (1LL << 30), "keysort: at most 2^30 keys");
    LGS_REQUIRE(lo >= 0 && bits >= 0 && lo + bits <= 32, "keysort: bit range");
    if (n == 0) return;
    if (bits == 0) {
        LGS_HIP_CHECK(hipMemcpyAsync(out, in, sizeof(unsigned) * (size_t)n, hipMemcpyDeviceToDevice, st));
        return;
    }
    const bool fresh = ctx->buf[S_RAY0] == nullptr;
    unsigned* ctl = (unsigned*)ctx->ensure(S_RAY0, sizeof(unsigned) * kCtlWords);
    if (fresh) LGS_HIP_CHECK(hipMemsetAsync(ctl, 0, sizeof(unsigned) * kCtlWords, st));
    // one launch (k_sort_wide) when every tile can be resident at once
    // (measured per device)
    {
        // wide tiles, digits of up to 10 bits (8 when that takes as many passes)
        const int wp = bits > 16 ? (bits + 9) / 10 : (bits + 7) / 8;
        const int wd = (bits + wp - 1) / wp;
        const long long ctiles = (n + kWideTile - 1) / kWideTile;
        if (ctiles <= coop_capacity(ctx) && (wp == 1 || tmp)) {
            const int rb = wd > 8 ? 10 : 8;
            unsigned* counts = (unsigned*)ctx->ensure(S_RAY1, sizeof(unsigned) * (size_t)ctiles * (1u << rb) * wp);
            if (rb == 10)
                hipLaunchKernelGGL(HIP_KERNEL_NAME(k_sort_wide<10>), dim3((unsigned)ctiles), dim3(kWideThreads), 0, st,
                                   in, out, tmp, n, lo, wd, bits, wp, counts, ctl + kCtlBar);
            else
                hipLaunchKernelGGL(HIP_KERNEL_NAME(k_sort_wide<8>), dim3((unsigned)ctiles), dim3(kWideThreads), 0, st,
                                   in, out, tmp, n, lo, wd, bits, wp, counts, ctl + kCtlBar);
            LGS_HIP_CHECK(hipGetLastError());
            return;
        }
    }
    const int passes = (bits + 7) / 8;
    const int dbits = (bits + passes - 1) / passes;
    // 4096-key tiles (a short look-back chain); 1024-key tiles only for sorts
    // too small to give 64 workgroups
    const bool big = n >= 64LL * 4096;
    const int tile = kSortThreads * (big ? 16 : 4);
    const long long tiles = (n + tile - 1) / tile;
    unsigned long long* status = (unsigned long long*)ctx->ensure(
        S_RAY1, sizeof(unsigned long long) * (size_t)tiles * kSortRadix * (size_t)passes);
    const unsigned hist_blocks =
        (unsigned)std::min<long long>((n + kSortThreads * kHistRun - 1) / (kSortThreads * kHistRun), 2048);
    hipLaunchKernelGGL(k_sort_hist, dim3(hist_blocks), dim3(kSortThreads), 0, st, in, n, lo, dbits, bits, passes,
                       ctl);
    LGS_HIP_CHECK(hipGetLastError());
    for (int p = 0; p < passes; ++p) {
        const unsigned* src = (p == 0) ? in : (((passes - p) % 2 == 1) ? tmp : out);
        unsigned* dst = ((passes - 1 - p) % 2 == 0) ? out : tmp;
        LGS_REQUIRE(dst != nullptr && src != nullptr, "keysort: tmp buffer needed for several passes");
        const int nb = std::min(dbits, bits - p * dbits);
        const unsigned stamp = (unsigned)ctx->next_stamp();
        unsigned long long* stp = status + (size_t)p * tiles * kSortRadix;
        if (big)
            hipLaunchKernelGGL(k_sort_pass<16>, dim3((unsigned)tiles), dim3(kSortThreads), 0, st, src, dst, n,
                               lo + p * dbits, nb, ctl + kCtlOffs + p * kSortRadix, stp, ctl + kCtlTicket + p, stamp);
        else
            hipLaunchKernelGGL(k_sort_pass<4>, dim3((unsigned)tiles), dim3(kSortThreads), 0, st, src, dst, n,
                               lo + p * dbits, nb, ctl + kCtlOffs + p * kSortRadix, stp, ctl + kCtlTicket + p, stamp);
        LGS_HIP_CHECK(hipGetLastError());
    }
}

}  // namespace lgs

// Diagnostics entry (tests): stable sort of host keys on bits [lo, lo + bits)
// through the device path.
extern "C" int lgs_debug_keysort(lgs_ctx* ctx, const unsigned* keys, unsigned* out, long long n, int lo, int bits)
{
    using namespace lgs;
    if (!ctx || n < 0 || (n > 0 && (!keys || !out))) return LGS_ERR_INVALID_ARG;
    return guarded(ctx, [&] {
        LGS_HIP_CHECK(hipSetDevice(ctx->device));
        if (n == 0) return;
        unsigned* d = nullptr;
        LGS_HIP_CHECK(hipMalloc(&d, sizeof(unsigned) * 3 * (size_t)n));
        try {
            LGS_HIP_CHECK(hipMemcpyAsync(d, keys, sizeof(unsigned) * (size_t)n, hipMemcpyHostToDevice, ctx->stream));
            keysort(ctx, d, d + n, d + 2 * n, n, lo, bits);
            LGS_HIP_CHECK(hipMemcpyAsync(out, d + n, sizeof(unsigned) * (size_t)n, hipMemcpyDeviceToHost, ctx->stream));
            ctx->sync();
        } catch (...) {
            hipFree(d);
            throw;
        }
        LGS_HIP_CHECK(hipFree(d));
    });
}
