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
//                 among equal digits (digit-bit ballots), per tile the digit
//                 counts published as aggregates and turned into inclusive
//                 prefixes by a decoupled look-back over earlier tiles (status
//                 words tagged with a per-pass stamp: no clearing); keys are
//                 reordered by digit in LDS and written out in digit runs
//
// Each workgroup only waits on tiles with lower tickets, which belong to
// workgroups that started before it, so the look-back always drains.
#include "lgs_internal.hpp"

#include <algorithm>

namespace {

constexpr int kSortThreads = 256;
constexpr int kSortRadix = 256;        // bins per pass (digits of at most 8 bits)
constexpr int kSortMaxPasses = 4;
// control block (unsigned words, S_RAY0): zero between sorts
constexpr int kCtlHist = 0;                                  // [pass][256] accumulators
constexpr int kCtlDone = kSortMaxPasses * kSortRadix;        // workgroups finished k_sort_hist
constexpr int kCtlTicket = kCtlDone + 1;                     // [pass] tile tickets
constexpr int kCtlOffs = 2 * kSortMaxPasses * kSortRadix;    // [pass][256] exclusive digit offsets
constexpr int kCtlWords = 3 * kSortMaxPasses * kSortRadix;

constexpr unsigned long long kFlagAgg = 1ull << 30, kFlagPrefix = 2ull << 30;
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
    const long long stride = (long long)gridDim.x * kSortThreads;
    for (long long i = (long long)blockIdx.x * kSortThreads + tid; i < n; i += stride) {
        const unsigned k = keys[i];
        for (int p = 0; p < passes; ++p) {
            const int sh = lo + p * dbits;
            const int nb = min(dbits, bits - p * dbits);
            atomicAdd(&h[p][(k >> sh) & ((1u << nb) - 1u)], 1u);
        }
    }
    __syncthreads();
    for (int p = 0; p < passes; ++p)
        if (h[p][tid]) __hip_atomic_fetch_add(ctl + kCtlHist + p * kSortRadix + tid, h[p][tid], __ATOMIC_RELAXED,
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
            v[j] = ld_agent(ctl + kCtlHist + w * kSortRadix + lane * 4 + j);
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
    for (int p = 0; p < passes; ++p)
        __hip_atomic_store(ctl + kCtlHist + p * kSortRadix + tid, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
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
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    const unsigned mask = (1u << nb) - 1u;
    wcnt[0][tid] = wcnt[1][tid] = wcnt[2][tid] = wcnt[3][tid] = 0;
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
    const unsigned long long lt = (1ull << lane) - 1ull;
#pragma unroll
    for (int i = 0; i < KPT; ++i) {
        const bool valid = p0 + 64 * i < n;
        const unsigned d = (k[i] >> shift) & mask;
        unsigned long long peers = __ballot(valid);
        for (int b = 0; b < nb; ++b) {
            const bool bit = (d >> b) & 1u;
            const unsigned long long m = __ballot(valid && bit);
            peers &= bit ? m : ~m;
        }
        const unsigned base = wcnt[w][d];
        rank[i] = base + (unsigned)__popcll(peers & lt);
        if (valid && !(peers & lt)) wcnt[w][d] = base + (unsigned)__popcll(peers);
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
    unsigned excl = 0;
    if (tile > 0) {
        long long j = tile - 1;
        for (;;) {
            const unsigned long long v = __hip_atomic_load(status + (size_t)j * kSortRadix + d, __ATOMIC_RELAXED,
                                                           __HIP_MEMORY_SCOPE_AGENT);
            if ((v >> 32) != stamp || !(v & (kFlagAgg | kFlagPrefix))) {
                __builtin_amdgcn_s_sleep(1);
                continue;
            }
            excl += (unsigned)(v & kCountMask);
            if (v & kFlagPrefix) break;
            --j;
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

}  // namespace

namespace lgs {

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
    const int passes = (bits + 7) / 8;
    const int dbits = (bits + passes - 1) / passes;
    const bool fresh = ctx->buf[S_RAY0] == nullptr;
    unsigned* ctl = (unsigned*)ctx->ensure(S_RAY0, sizeof(unsigned) * kCtlWords);
    if (fresh) LGS_HIP_CHECK(hipMemsetAsync(ctl, 0, sizeof(unsigned) * kCtlWords, st));
    // small sorts: 1024-key tiles (enough workgroups to fill the chip); large: 4096
    const bool big = n >= (1LL << 21);
    const int tile = kSortThreads * (big ? 16 : 4);
    const long long tiles = (n + tile - 1) / tile;
    unsigned long long* status = (unsigned long long*)ctx->ensure(
        S_RAY1, sizeof(unsigned long long) * (size_t)tiles * kSortRadix * (size_t)passes);
    const unsigned hist_blocks = (unsigned)std::min<long long>(std::max<long long>(1, n / 8192), 1024);
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
