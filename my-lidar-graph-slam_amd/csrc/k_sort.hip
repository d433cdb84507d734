// k_sort.hip -- K3 sort: stable LSD radix sort of the ray-cast keys on MI355X.
//
// The ordered Bayes update (C/mapping/grid_map_builder.cpp:170-186 and
// :292-329) needs every cell's updates in ray order.  k_emit writes one 32-bit
// key per visited cell in ray order; a STABLE sort on the cell bits of the keys
// makes each cell's updates one contiguous run that keeps that order.
//
//   large sorts   one pass per 8-bit digit, reduce-then-scan: per-tile digit
//                 counts (k_sort_up), a device scan of the digit-major count
//                 array (k_scan_chunks + k_scan_top), then per tile stable
//                 ranks (per-wave LDS peer masks), an LDS reorder by digit and
//                 digit runs written at their offsets (k_sort_down)
//
//   k_sort_wide   sorts that fit the device at once: every pass in one
//                 launch, 8192-key tiles, digits of up to 10 bits, ranks from
//                 per-wave LDS peer masks, grid barriers around the count
//                 exchange (a config-4 step's ~160k keys, 20 cell bits: 20
//                 workgroups, 2 passes)
#include "lgs_internal.hpp"

#include <algorithm>
#include <cstring>
#include <mutex>
#include <utility>
#include <vector>

namespace {

constexpr int kSortThreads = 256;
constexpr int kSortRadix = 256;        // bins per pass (digits of at most 8 bits)
// control words (S_RAY0): k_sort_wide's grid barrier [arrived, done, abort],
// zero between sorts (the last workgroup out resets them)
constexpr int kCtlBar = 0;
constexpr int kCtlWords = 8;

// Large sorts, one digit pass = three steps with no chain between tiles
// (a decoupled look-back propagates prefixes tile to tile at a cross-XCD
// round trip per window of predecessors: ~0.33 ms per pass of 20M keys):
//   k_sort_up     per 4096-key tile the digit counts, stored digit-major
//                 (counts[d * tiles + tile])
//   k_scan_chunks exclusive scan of 4096-entry chunks of that array in place,
//   k_scan_top    and of the chunk totals: offset(d, tile) = chunk scan +
//                 scanned chunk total -- every digit's start in the output
//                 plus the keys of that digit in the tiles before this one
//   k_sort_down   per tile: stable ranks (per-wave LDS peer masks), the tile
//                 reordered by digit in LDS, digit runs written at the offsets
constexpr int kTileKPT = 16, kTile = kSortThreads * kTileKPT;   // 4096 keys per tile
constexpr int kScanChunk = kSortThreads * 16;                   // 4096 counts per scan chunk

// one key's stable rank among the earlier keys of its wave with the same
// digit; wcnt/mw: the wave's digit counts and peer masks (see k_sort_wide)
__device__ __forceinline__ unsigned wave_rank(bool valid, unsigned d, unsigned* __restrict__ wcnt,
                                              unsigned long long* __restrict__ mw, unsigned long long me,
                                              unsigned long long lt)
{
    unsigned long long peers = 0;
    if (valid) {
        __hip_atomic_fetch_or(&mw[d], me, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        peers = __hip_atomic_load(&mw[d], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    const unsigned base = valid ? wcnt[d] : 0u;
    if (valid && !(peers & lt)) {
        wcnt[d] = base + (unsigned)__popcll(peers);
        __hip_atomic_store(&mw[d], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    return base + (unsigned)__popcll(peers & lt);
}

__global__ __launch_bounds__(kSortThreads) void k_sort_up(const unsigned* __restrict__ in, long long n, int shift,
                                                          int nb, unsigned* __restrict__ counts, unsigned ntiles)
{
    __shared__ unsigned wcnt[4][kSortRadix];
    __shared__ unsigned long long wmask[4][kSortRadix];
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    const unsigned mask = (1u << nb) - 1u;
    wcnt[0][tid] = wcnt[1][tid] = wcnt[2][tid] = wcnt[3][tid] = 0;
    wmask[0][tid] = wmask[1][tid] = wmask[2][tid] = wmask[3][tid] = 0ull;
    __syncthreads();
    const long long p0 = (long long)blockIdx.x * kTile + (long long)w * 64 * kTileKPT + lane;
    unsigned k[kTileKPT];
#pragma unroll
    for (int i = 0; i < kTileKPT; ++i) {
        const long long p = p0 + 64 * i;
        k[i] = (p < n) ? in[p] : 0u;
    }
    const unsigned long long me = 1ull << lane, lt = me - 1ull;
#pragma unroll
    for (int i = 0; i < kTileKPT; ++i)
        (void)wave_rank(p0 + 64 * i < n, (k[i] >> shift) & mask, wcnt[w], wmask[w], me, lt);
    __syncthreads();
    counts[(size_t)tid * ntiles + blockIdx.x] = wcnt[0][tid] + wcnt[1][tid] + wcnt[2][tid] + wcnt[3][tid];
}

// exclusive scan of the 256 values of the block (thread order); *total: their sum
__device__ __forceinline__ unsigned block_scan256(unsigned v, unsigned* ws4, unsigned* total)
{
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    unsigned incl = v;
    for (int o = 1; o < 64; o <<= 1) {
        const unsigned t = __shfl_up(incl, o);
        if (lane >= o) incl += t;
    }
    if (lane == 63) ws4[w] = incl;
    __syncthreads();
    unsigned wo = 0;
    for (int q = 0; q < w; ++q) wo += ws4[q];
    if (total) *total = ws4[0] + ws4[1] + ws4[2] + ws4[3];
    return wo + incl - v;
}

__global__ __launch_bounds__(kSortThreads) void k_scan_chunks(unsigned* __restrict__ a, long long m,
                                                              unsigned* __restrict__ csum)
{
    __shared__ unsigned ws4[4];
    const long long b0 = (long long)blockIdx.x * kScanChunk + (long long)threadIdx.x * 16;
    unsigned v[16], s = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        v[i] = (b0 + i < m) ? a[b0 + i] : 0u;
        s += v[i];
    }
    unsigned tot = 0;
    unsigned run = block_scan256(s, ws4, &tot);
#pragma unroll
    for (int i = 0; i < 16; ++i)
        if (b0 + i < m) {
            a[b0 + i] = run;
            run += v[i];
        }
    if (threadIdx.x == 0) csum[blockIdx.x] = tot;
}

// one workgroup: exclusive scan of the chunk totals, in place
__global__ __launch_bounds__(kSortThreads) void k_scan_top(unsigned* __restrict__ csum, int nc)
{
    __shared__ unsigned ws4[4];
    unsigned carry = 0;
    for (int c0 = 0; c0 < nc; c0 += kSortThreads * 16) {
        const int b0 = c0 + (int)threadIdx.x * 16;
        unsigned v[16], s = 0;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            v[i] = (b0 + i < nc) ? csum[b0 + i] : 0u;
            s += v[i];
        }
        unsigned tot = 0;
        unsigned run = carry + block_scan256(s, ws4, &tot);
#pragma unroll
        for (int i = 0; i < 16; ++i)
            if (b0 + i < nc) {
                csum[b0 + i] = run;
                run += v[i];
            }
        carry += tot;
        __syncthreads();
    }
}

__global__ __launch_bounds__(kSortThreads) void k_sort_down(const unsigned* __restrict__ in,
                                                            unsigned* __restrict__ out, long long n, int shift,
                                                            int nb, const unsigned* __restrict__ offs,
                                                            const unsigned* __restrict__ csum, unsigned ntiles)
{
    __shared__ unsigned keys_s[kTile];
    __shared__ unsigned wcnt[4][kSortRadix];
    __shared__ unsigned long long wmask[4][kSortRadix];
    __shared__ unsigned dstart[kSortRadix];
    __shared__ unsigned gbase[kSortRadix];
    __shared__ unsigned ws4[4];
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    const unsigned mask = (1u << nb) - 1u;
    const unsigned tile = blockIdx.x;
    wcnt[0][tid] = wcnt[1][tid] = wcnt[2][tid] = wcnt[3][tid] = 0;
    wmask[0][tid] = wmask[1][tid] = wmask[2][tid] = wmask[3][tid] = 0ull;
    {
        const size_t q = (size_t)tid * ntiles + tile;   // digit tid's offset for this tile
        gbase[tid] = offs[q] + csum[q / kScanChunk];
    }
    __syncthreads();
    const long long t0 = (long long)tile * kTile;
    const long long p0 = t0 + (long long)w * 64 * kTileKPT + lane;
    unsigned k[kTileKPT], rank[kTileKPT];
#pragma unroll
    for (int i = 0; i < kTileKPT; ++i) {
        const long long p = p0 + 64 * i;
        k[i] = (p < n) ? in[p] : 0u;
    }
    const unsigned long long me = 1ull << lane, lt = me - 1ull;
#pragma unroll
    for (int i = 0; i < kTileKPT; ++i)
        rank[i] = wave_rank(p0 + 64 * i < n, (k[i] >> shift) & mask, wcnt[w], wmask[w], me, lt);
    __syncthreads();
    // digit tid: exclusive prefix over the waves and the tile-local start
    const int d = tid;
    const unsigned c0 = wcnt[0][d], c1 = wcnt[1][d], c2 = wcnt[2][d], c3 = wcnt[3][d];
    const unsigned tot = c0 + c1 + c2 + c3;
    wcnt[0][d] = 0;
    wcnt[1][d] = c0;
    wcnt[2][d] = c0 + c1;
    wcnt[3][d] = c0 + c1 + c2;
    dstart[d] = block_scan256(tot, ws4, nullptr);
    __syncthreads();
#pragma unroll
    for (int i = 0; i < kTileKPT; ++i)
        if (p0 + 64 * i < n) {
            const unsigned dd = (k[i] >> shift) & mask;
            keys_s[dstart[dd] + wcnt[w][dd] + rank[i]] = k[i];
        }
    __syncthreads();
    const int nvalid = (int)min((long long)kTile, n - t0);
    for (int j = tid; j < nvalid; j += kSortThreads) {
        const unsigned key = keys_s[j];
        const unsigned dd = (key >> shift) & mask;
        out[gbase[dd] + (unsigned)j - dstart[dd]] = key;
    }
}

// Small sorts (every tile resident at once): all passes in ONE launch.  Each
// workgroup ranks its tile as k_sort_down does, stores its digit counts,
// waits at a grid barrier, reads every tile's counts (digit totals and the
// counts of the tiles before it: the same offsets a histogram and a look-back
// give), scatters, and waits again before the next pass reads the keys.
// Stores are released and loads acquired at agent scope around each barrier
// (the tiles live on different XCDs, each with its own L2).
// The wait is bounded (`ticks` of s_memrealtime, 100 MHz; LGS_OPT_SORT_BARRIER_US):
// a tile that waits longer -- its peers cannot all be resident -- raises the
// abort word, every tile leaves, and the caller's error word reads 2 (a loud
// failure instead of a hung GPU; the host reservation below keeps it from
// happening within one process).
__device__ __forceinline__ bool grid_barrier(unsigned* bar, unsigned target, unsigned long long ticks)
{
    __shared__ int s_ok;
    __syncthreads();
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        __hip_atomic_fetch_add(bar, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        int ok = 1;
        while (__hip_atomic_load(bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
            if (__hip_atomic_load(bar + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ||
                __builtin_amdgcn_s_memrealtime() - t0 >= ticks) {
                __hip_atomic_store(bar + 2, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                ok = 0;
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        s_ok = ok;
    }
    __syncthreads();
    return s_ok != 0;
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
                                                            unsigned* __restrict__ bar, int* __restrict__ err,
                                                            unsigned long long ticks, unsigned* done_flag,
                                                            unsigned done_gen)
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
        if (!grid_barrier(bar, ++nbar * ntiles, ticks)) break;
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
        if (p + 1 < passes && !grid_barrier(bar, ++nbar * ntiles, ticks)) break;
        LGS_PROBE_MARK();
    }
    LGS_PROBE_PRINT("k_sort_wide");
    __syncthreads();
    if (tid == 0) {
        if (__hip_atomic_load(bar + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) && err) *err = 2;
        if (__hip_atomic_fetch_add(bar + 1, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == ntiles - 1) {
            __hip_atomic_store(bar, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(bar + 2, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(bar + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            // every tile is past its last wait: the host may reuse the reservation
            __threadfence_system();
            *(volatile unsigned*)done_flag = done_gen;
        }
    }
}

}  // namespace

namespace lgs {

// Co-residency of k_sort_wide across the process: its tiles wait for each
// other, so the tiles of every k_sort_wide in flight on a device -- from any
// lgs_ctx, on any stream -- must fit the device at once.  Each launch
// reserves its tiles against the device's capacity (half its occupancy: a
// margin for other streams' and processes' work) and holds them until the
// launch's last workgroup has written the launch's generation into its slot
// of a coherent pinned flag array (r05: an event recorded after each launch
// cost a ~5 us gap before the next kernel of a config-4 step); a sort that
// does not fit beside the others takes the reduce-then-scan passes.
// Reserve and launch happen under the device's lock.
struct CoopDevice {
    static constexpr int kSlots = 64;
    std::mutex mu;
    long long cap = 0, used = 0;
    unsigned* flags = nullptr;   // coherent pinned; slot s = generation of the last launch done in it
    unsigned gen = 0;
    struct Live {
        int slot;
        unsigned gen;
        long long tiles;
    };
    std::vector<Live> live;   // launch order
    std::vector<int> free_slots;
    bool done(const Live& l) const { return __atomic_load_n(&flags[l.slot], __ATOMIC_ACQUIRE) == l.gen; }
    void release(size_t i)
    {
        used -= live[i].tiles;
        free_slots.push_back(live[i].slot);
        live.erase(live.begin() + (ptrdiff_t)i);
    }
    // every completed launch (when the capacity is short)
    void reclaim()
    {
        for (size_t i = 0; i < live.size();) {
            if (done(live[i])) release(i);
            else ++i;
        }
    }
    // the oldest launches, while completed
    void reclaim_front()
    {
        while (!live.empty() && done(live.front())) release(0);
    }
};
CoopDevice g_coop[64];

// Launches the one-launch sort when its tiles fit beside the device's other
// cooperative launches; false: not launched (take the multi-pass sort).
template <typename Launch>
bool coop_launch(lgs_ctx* ctx, long long tiles, Launch&& launch)
{
    const int dev = ctx->device;
    if (dev < 0 || dev >= 64) return false;
    CoopDevice& D = g_coop[dev];
    std::lock_guard<std::mutex> lk(D.mu);
    if (!D.cap) {
        int per_cu = 0, cus = 0;
        LGS_HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_sort_wide<10>, kWideThreads, 0));
        LGS_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
        LGS_HIP_CHECK(hipHostMalloc((void**)&D.flags, sizeof(unsigned) * CoopDevice::kSlots, hipHostMallocCoherent));
        std::memset(D.flags, 0, sizeof(unsigned) * CoopDevice::kSlots);
        for (int i = CoopDevice::kSlots - 1; i >= 0; --i) D.free_slots.push_back(i);
        D.cap = std::max(1LL, (long long)per_cu * cus / 2);
    }
    const long long cap = ctx->coop_tiles >= 0 ? std::min(D.cap, ctx->coop_tiles) : D.cap;
    if (tiles > cap) return false;
    D.reclaim_front();
    if (D.used + tiles > cap || D.free_slots.empty()) D.reclaim();
    if (D.used + tiles > cap || D.free_slots.empty()) return false;
    const int slot = D.free_slots.back();
    if (++D.gen == 0) ++D.gen;   // 0: a slot never used
    launch(D.flags + slot, D.gen);
    LGS_HIP_CHECK(hipGetLastError());
    D.free_slots.pop_back();
    D.used += tiles;
    D.live.push_back(CoopDevice::Live{ slot, D.gen, tiles });
    return true;
}

// Stable sort of n 32-bit keys on bits [lo, lo + bits).  `tmp` (n keys) is
// needed when the sort takes two or more passes; in, tmp and out are distinct.
// `err` (device-visible, may be null): set to 2 if the one-launch sort's grid
// barrier timed out (its output is then invalid).
void keysort(lgs_ctx* ctx, const unsigned* in, unsigned* out, unsigned* tmp, long long n, int lo, int bits, int* err)
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
        if (wp == 1 || tmp) {
            const int rb = wd > 8 ? 10 : 8;
            unsigned* counts = (unsigned*)ctx->ensure(S_RAY1, sizeof(unsigned) * (size_t)ctiles * (1u << rb) * wp);
            const unsigned long long ticks = (unsigned long long)ctx->sort_barrier_us * 100ull;   // 100 MHz
            const bool done = coop_launch(ctx, ctiles, [&](unsigned* flag, unsigned gen) {
                if (rb == 10)
                    hipLaunchKernelGGL(HIP_KERNEL_NAME(k_sort_wide<10>), dim3((unsigned)ctiles), dim3(kWideThreads), 0,
                                       st, in, out, tmp, n, lo, wd, bits, wp, counts, ctl + kCtlBar, err, ticks, flag,
                                       gen);
                else
                    hipLaunchKernelGGL(HIP_KERNEL_NAME(k_sort_wide<8>), dim3((unsigned)ctiles), dim3(kWideThreads), 0,
                                       st, in, out, tmp, n, lo, wd, bits, wp, counts, ctl + kCtlBar, err, ticks, flag,
                                       gen);
            });
            if (done) return;
        }
    }
    // reduce-then-scan passes of 8-bit digits
    const int passes = (bits + 7) / 8;
    const int dbits = (bits + passes - 1) / passes;
    const long long tiles = (n + kTile - 1) / kTile;
    const long long m = tiles * kSortRadix;
    const long long nc = (m + kScanChunk - 1) / kScanChunk;
    unsigned* counts = (unsigned*)ctx->ensure(S_RAY1, sizeof(unsigned) * (size_t)(m + nc));
    unsigned* csum = counts + m;
    for (int p = 0; p < passes; ++p) {
        const unsigned* src = (p == 0) ? in : (((passes - p) % 2 == 1) ? tmp : out);
        unsigned* dst = ((passes - 1 - p) % 2 == 0) ? out : tmp;
        LGS_REQUIRE(dst != nullptr && src != nullptr, "keysort: tmp buffer needed for several passes");
        const int nb = std::min(dbits, bits - p * dbits), sh = lo + p * dbits;
        hipLaunchKernelGGL(k_sort_up, dim3((unsigned)tiles), dim3(kSortThreads), 0, st, src, n, sh, nb, counts,
                           (unsigned)tiles);
        hipLaunchKernelGGL(k_scan_chunks, dim3((unsigned)nc), dim3(kSortThreads), 0, st, counts, m, csum);
        hipLaunchKernelGGL(k_scan_top, dim3(1), dim3(kSortThreads), 0, st, csum, (int)nc);
        hipLaunchKernelGGL(k_sort_down, dim3((unsigned)tiles), dim3(kSortThreads), 0, st, src, dst, n, sh, nb,
                           (const unsigned*)counts, (const unsigned*)csum, (unsigned)tiles);
        LGS_HIP_CHECK(hipGetLastError());
    }
}

}  // namespace lgs

// Diagnostics entry (tests): stable sort of host keys on bits [lo, lo + bits)
// through the device path; LGS_ERR_INTERNAL if the one-launch sort's grid
// barrier timed out.
extern "C" int lgs_debug_keysort(lgs_ctx* ctx, const unsigned* keys, unsigned* out, long long n, int lo, int bits)
{
    using namespace lgs;
    if (!ctx || n < 0 || (n > 0 && (!keys || !out))) return LGS_ERR_INVALID_ARG;
    return guarded(ctx, [&] {
        LGS_HIP_CHECK(hipSetDevice(ctx->device));
        if (n == 0) return;
        unsigned* d = nullptr;
        LGS_HIP_CHECK(hipMalloc(&d, sizeof(unsigned) * (3 * (size_t)n + 1)));
        int err = 0;
        try {
            int* d_err = (int*)(d + 3 * n);
            LGS_HIP_CHECK(hipMemsetAsync(d_err, 0, sizeof(int), ctx->stream));
            LGS_HIP_CHECK(hipMemcpyAsync(d, keys, sizeof(unsigned) * (size_t)n, hipMemcpyHostToDevice, ctx->stream));
            keysort(ctx, d, d + n, d + 2 * n, n, lo, bits, d_err);
            LGS_HIP_CHECK(hipMemcpyAsync(out, d + n, sizeof(unsigned) * (size_t)n, hipMemcpyDeviceToHost, ctx->stream));
            LGS_HIP_CHECK(hipMemcpyAsync(&err, d_err, sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
            ctx->sync();
        } catch (...) {
            hipFree(d);
            throw;
        }
        LGS_HIP_CHECK(hipFree(d));
        if (err) throw Error(LGS_ERR_INTERNAL, "k_sort_wide: grid barrier timed out (cooperative tiles not co-resident)");
    });
}
