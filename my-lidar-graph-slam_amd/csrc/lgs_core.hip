// lgs_core.hip -- context, device arena, grids, scans and the coarse-map
// precompute kernel (K2) of the MI355X hot-path library.
//
// K2 restates PrecomputeGridMap (C/mapping/grid_map_builder.cpp:518-536):
// SlidingWindowMaxRow (:403-434) then SlidingWindowMaxCol (:437-468), each a
// forward window max out[i] = max(in[s(i) .. s(i)+w-1]) with s(i) = min(i, n-w)
// (the tail repeats the last full window, H/util.hpp:250-252) and 0.0 read past
// the end when n < w.  Max is exact, so the separable pair equals one 2-D
// window max over zero-padded input; it is computed here from an LDS tile.
#include "lgs_internal.hpp"

#include <atomic>
#include <condition_variable>
#include <cstring>
#include <mutex>
#include <thread>

#include <pthread.h>

using namespace lgs;

// ---------------------------------------------------------------------------
// context + arena
// ---------------------------------------------------------------------------
void* lgs_ctx::ensure(int slot, size_t bytes)
{
    if (bytes == 0) bytes = 16;
    if (buf_bytes[slot] >= bytes) return buf[slot];
    if (buf[slot]) {
        LGS_HIP_CHECK(hipStreamSynchronize(stream));
        LGS_HIP_CHECK(hipFree(buf[slot]));
        buf[slot] = nullptr;
        buf_bytes[slot] = 0;
    }
    size_t want = bytes + bytes / 4;  // grow with headroom
    void* p = nullptr;
    hipError_t e = hipMalloc(&p, want);
    if (e != hipSuccess) throw Error(LGS_ERR_OOM, "hipMalloc failed for scratch slot");
    buf[slot] = p;
    buf_bytes[slot] = want;
    return p;
}

void* lgs_ctx::ensure_aux(int i, size_t bytes)
{
    if ((int)aux.size() <= i) {
        aux.resize((size_t)i + 1, nullptr);
        aux_bytes.resize((size_t)i + 1, 0);
    }
    if (bytes == 0) bytes = 16;
    if (aux_bytes[i] >= bytes) return aux[i];
    if (aux[i]) {
        LGS_HIP_CHECK(hipStreamSynchronize(stream));
        LGS_HIP_CHECK(hipFree(aux[i]));
        aux[i] = nullptr;
        aux_bytes[i] = 0;
    }
    const size_t want = bytes + bytes / 2;
    if (hipMalloc(&aux[i], want) != hipSuccess) throw Error(LGS_ERR_OOM, "hipMalloc failed for an auxiliary buffer");
    aux_bytes[i] = want;
    return aux[i];
}

void* lgs_ctx::ensure_pinned(size_t bytes)
{
    if (pinned_bytes >= bytes) return pinned;
    if (pinned) {
        LGS_HIP_CHECK(hipStreamSynchronize(stream));
        LGS_HIP_CHECK(hipHostFree(pinned));
        pinned = nullptr;
        pinned_bytes = 0;
    }
    size_t want = bytes + bytes / 4;
    LGS_HIP_CHECK(hipHostMalloc(&pinned, want, hipHostMallocDefault));
    pinned_bytes = want;
    return pinned;
}

void* lgs_ctx::ensure_pinned_in(size_t bytes)
{
    if (pinned_in_bytes >= bytes) return pinned_in;
    if (pinned_in) {
        LGS_HIP_CHECK(hipStreamSynchronize(stream));
        LGS_HIP_CHECK(hipHostFree(pinned_in));
        pinned_in = nullptr;
        pinned_in_bytes = 0;
    }
    size_t want = bytes + bytes / 4;
    LGS_HIP_CHECK(hipHostMalloc(&pinned_in, want, hipHostMallocDefault));
    pinned_in_bytes = want;
    return pinned_in;
}

namespace {
void* grow_pinned(hipStream_t stream, void*& p, size_t& have, size_t bytes, bool coherent)
{
    if (have >= bytes) return p;
    if (p) {
        LGS_HIP_CHECK(hipStreamSynchronize(stream));
        LGS_HIP_CHECK(hipHostFree(p));
        p = nullptr;
        have = 0;
    }
    size_t want = bytes + bytes / 4;
    // coherent where k_fetch reads it: uncached on the device, fresh on every launch
    LGS_HIP_CHECK(hipHostMalloc(&p, want, coherent ? hipHostMallocCoherent : hipHostMallocDefault));
    have = want;
    return p;
}

__global__ __launch_bounds__(256) void k_fetch(FetchList L)
{
    const FetchSeg& s = L.s[blockIdx.y];   // one segment per grid row
    const unsigned long long n16 = s.bytes / 16;
    const unsigned long long g = (unsigned long long)blockIdx.x * 256 + threadIdx.x;
    const uint4* __restrict__ a = (const uint4*)s.src;
    uint4* __restrict__ b = (uint4*)s.dst;
    for (unsigned long long i = g; i < n16; i += (unsigned long long)gridDim.x * 256) b[i] = a[i];
    if (n16 * 16 + g < s.bytes) s.dst[n16 * 16 + g] = s.src[n16 * 16 + g];   // the tail bytes
}
}  // namespace

namespace lgs {
FetchSeg fetch_seg(void* dst, const void* src, size_t bytes)
{
    LGS_REQUIRE(((uintptr_t)dst & 15) == 0 && ((uintptr_t)src & 15) == 0, "fetch: 16-byte alignment");
    void* dsrc = nullptr;
    LGS_HIP_CHECK(hipHostGetDevicePointer(&dsrc, const_cast<void*>(src), 0));
    return FetchSeg{ (const unsigned char*)dsrc, (unsigned char*)dst, (unsigned long long)bytes };
}

void fetch_list(lgs_ctx* ctx, const std::vector<FetchSeg>& segs)
{
    for (size_t k0 = 0; k0 < segs.size(); k0 += kFetchSegs) {
        FetchList L{};
        unsigned long long mx = 0;
        int n = 0;
        for (size_t k = k0; k < segs.size() && n < kFetchSegs; ++k)
            if (segs[k].bytes) {
                L.s[n++] = segs[k];
                mx = std::max(mx, segs[k].bytes / 16);
            }
        if (!n) continue;
        const unsigned blocks = (unsigned)std::max<unsigned long long>(1, std::min<unsigned long long>((mx + 255) / 256, 64));
        hipLaunchKernelGGL(k_fetch, dim3(blocks, (unsigned)n), dim3(256), 0, ctx->stream, L);
        LGS_HIP_CHECK(hipGetLastError());
    }
}

void fetch_async(lgs_ctx* ctx, void* dst, const void* src, size_t bytes)
{
    if (bytes == 0) return;
    fetch_list(ctx, { fetch_seg(dst, src, bytes) });
}
}  // namespace lgs

void* lgs_ctx::ensure_pinned_up(size_t bytes)
{
    return bank ? grow_pinned(stream, pinned_up_b, pinned_up_b_bytes, bytes, true)
                : grow_pinned(stream, pinned_up, pinned_up_bytes, bytes, true);
}

int* lgs_ctx::tedge_buffer(size_t n)
{
    // kTedgeCtrs wrap-around counters (k_match_small) ahead of the stamps:
    // both are zero in their rest state, so one memset at allocation serves
    const int slot = banked(S_TEDGE);
    int* p = (int*)ensure(slot, sizeof(int) * (kTedgeCtrs + std::max<size_t>(n, 1)));
    if (buf_bytes[slot] != tedge_zeroed[bank]) {
        LGS_HIP_CHECK(hipMemsetAsync(p, 0, buf_bytes[slot], stream));
        tedge_zeroed[bank] = buf_bytes[slot];
    }
    return p + kTedgeCtrs;
}

int* lgs_ctx::small_counters(size_t n)
{
    return tedge_buffer(n) - kTedgeCtrs;
}

void* lgs_ctx::ensure_pinned_rec(size_t bytes)
{
    // coherent: k_post writes the records (and their flag) here directly
    return grow_pinned(stream, pinned_rec[bank], pinned_rec_bytes[bank], bytes, true);
}

namespace lgs {
const char* const kKernelNames[K_NUM_KERNELS] = { "k_project", "k_coarse", "k_seed", "k_select",
                                                  "k_fine", "k_replay", "k_cost", "k_precompute",
                                                  "k_linsolve", "k_ray_emit", "k_ray_apply",
                                                  "k_super", "k_super_planes", "k_bb_score", "k_bb_expand",
                                                  "k_coarse_aux", "k_match_small" };
}

int lgs_ctx::next_stamp()
{
    static std::atomic<int> counter{ 0 };
    int s = counter.fetch_add(1, std::memory_order_relaxed) + 1;
    if (s <= 0) {   // 2^31 stamps: restart above 0 (tags compare 32 bits)
        counter.store(1);
        s = 1;
    }
    return s;
}

void lgs_ctx::sync()
{
    if (!spin_sync) {
        LGS_HIP_CHECK(hipStreamSynchronize(stream));
    } else {
        for (;;) {
            const hipError_t e = hipStreamQuery(stream);
            if (e == hipSuccess) break;
            if (e != hipErrorNotReady) LGS_HIP_CHECK(e);
        }
    }
    up_busy[0] = up_busy[1] = false;
}

int lgs_ctx::timing_begin(int kernel, double algo_bytes)
{
    if (!profile || !((profile_mask >> kernel) & 1u)) return -1;
    if (dev_timing && dts_dev && dts_used < kDtsSlots) {
        // device-timed: a slot of the chunk's words, no events
        PendingTiming t{ kernel, nullptr, nullptr, algo_bytes };
        t.batch = timing_batch;
        t.hw = dts_host + (size_t)dts_used * 2 * kDtsSub;
        t.tag = (unsigned long long)dts_gen << 40;
        ++dts_used;
        pending.push_back(t);
        return (int)pending.size() - 1;
    }
    hipEvent_t ev[2];
    for (int i = 0; i < 2; ++i) {
        if (!event_pool.empty()) {
            ev[i] = event_pool.back();
            event_pool.pop_back();
        } else {
            LGS_HIP_CHECK(hipEventCreate(&ev[i]));
        }
    }
    LGS_HIP_CHECK(hipEventRecord(ev[0], stream));
    PendingTiming t{ kernel, ev[0], ev[1], algo_bytes };
    t.batch = timing_batch;
    pending.push_back(t);
    return (int)pending.size() - 1;
}

void lgs_ctx::timing_end(int token)
{
    if (token < 0 || !pending[token].b) return;   // device-timed: nothing to record
    LGS_HIP_CHECK(hipEventRecord(pending[token].b, stream));
}

namespace {
// A device-timed launch's span from its words' host copy (first workgroup
// start to last workgroup end, s_memrealtime at 100 MHz); false if no
// workgroup of this generation stamped both (e.g. a launch skipped).  *t0,
// *t1: the ticks.
bool dts_span_ms(const PendingTiming& p, float& ms, unsigned long long* t0p = nullptr,
                 unsigned long long* t1p = nullptr)
{
    unsigned long long t0 = ~0ull, t1 = 0;
    bool any0 = false, any1 = false;
    for (int s = 0; s < kDtsSub; ++s) {
        const unsigned long long w0 = __atomic_load_n(p.hw + 2 * s, __ATOMIC_ACQUIRE);
        const unsigned long long w1 = __atomic_load_n(p.hw + 2 * s + 1, __ATOMIC_ACQUIRE);
        if ((w0 & ~kDtsMask) == p.tag) {
            t0 = std::min(t0, kDtsMask - (w0 & kDtsMask));
            any0 = true;
        }
        if ((w1 & ~kDtsMask) == p.tag) {
            t1 = std::max(t1, w1 & kDtsMask);
            any1 = true;
        }
    }
    if (!any0 || !any1 || t1 < t0) return false;   // (t1 < t0: the 40-bit clock wrapped, ~3 h)
    ms = (float)((double)(t1 - t0) * 1e-5);
    if (t0p) *t0p = t0;
    if (t1p) *t1p = t1;
    return true;
}
}  // namespace

void lgs_ctx::harvest()
{
    harvest_upto(LLONG_MAX);
}

void lgs_ctx::harvest_upto(long long b)
{
    size_t k = 0;
    long long prev_batch = -1;
    unsigned long long prev_end = 0;   // the end tick of the chunk's previous device-timed launch
    for (; k < pending.size() && pending[k].batch <= b; ++k) {
        PendingTiming& p = pending[k];
        float ms = 0.f;
        double disp = 0.0;
        if (p.hw) {
            unsigned long long t0 = 0, t1 = 0;
            if (!dts_span_ms(p, ms, &t0, &t1)) continue;
            const bool chained = prev_batch == p.batch && prev_end <= t1 && prev_end != 0;
            disp = chained ? (double)(t1 - std::min(prev_end, t0)) * 1e-5 : (double)ms;
            prev_batch = p.batch;
            prev_end = t1;
        } else {
            LGS_HIP_CHECK(hipEventSynchronize(p.b));
            LGS_HIP_CHECK(hipEventElapsedTime(&ms, p.a, p.b));
            event_pool.push_back(p.a);
            event_pool.push_back(p.b);
            disp = ms;
        }
        stat_launches[p.kernel] += 1;
        stat_ms[p.kernel] += ms;
        stat_bytes[p.kernel] += p.algo_bytes;
        stat_disp_ms[p.kernel] += disp;
    }
    pending.erase(pending.begin(), pending.begin() + (long)k);
}

void lgs_ctx::wait_event(hipEvent_t ev)
{
    if (!spin_sync) {
        LGS_HIP_CHECK(hipEventSynchronize(ev));
        return;
    }
    for (;;) {
        const hipError_t e = hipEventQuery(ev);
        if (e == hipSuccess) return;
        if (e != hipErrorNotReady) LGS_HIP_CHECK(e);
    }
}

void lgs_ctx::release()
{
    if (stream) hipStreamSynchronize(stream);
    if (hi) hipStreamSynchronize(hi);
    for (int i = 0; i < S_NUM_SLOTS; ++i) {
        if (buf[i]) hipFree(buf[i]);
        buf[i] = nullptr;
        buf_bytes[i] = 0;
    }
    if (pinned) hipHostFree(pinned);
    pinned = nullptr;
    for (void* q : aux)
        if (q) hipFree(q);
    aux.clear();
    aux_bytes.clear();
    if (zero) hipFree(zero);
    zero = nullptr;
    for (int b = 0; b < 2; ++b) {
        if (dts_buf[b]) hipFree(dts_buf[b]);
        dts_buf[b] = nullptr;
    }
    for (auto& p : pending) {
        if (!p.a) continue;   // device-timed
        hipEventDestroy(p.a);
        hipEventDestroy(p.b);
    }
    pending.clear();
    for (auto e : event_pool) hipEventDestroy(e);
    event_pool.clear();
    for (auto& e : bank_ev) {
        if (e) hipEventDestroy(e);
        e = nullptr;
    }
    if (pinned_up) hipHostFree(pinned_up);
    pinned_up = nullptr;
    if (pinned_in) hipHostFree(pinned_in);
    pinned_in = nullptr;
    if (pinned_up_b) hipHostFree(pinned_up_b);
    pinned_up_b = nullptr;
    for (int b = 0; b < 2; ++b) {
        if (pinned_rec[b]) hipHostFree(pinned_rec[b]);
        pinned_rec[b] = nullptr;
        if (pinned_scan[b]) hipHostFree(pinned_scan[b]);
        pinned_scan[b] = nullptr;
        if (scan_ev[b]) hipEventDestroy(scan_ev[b]);
        scan_ev[b] = nullptr;
    }
    if (stream) hipStreamDestroy(stream);
    stream = nullptr;
    if (hi) hipStreamDestroy(hi);
    hi = nullptr;
    for (auto& e : split_ev) {
        if (e) hipEventDestroy(e);
        e = nullptr;
    }
}

extern "C" int lgs_abi_version(void) { return LGS_ABI_VERSION; }

extern "C" int lgs_ctx_create(int device, lgs_ctx** out)
{
    if (!out) return LGS_ERR_INVALID_ARG;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return LGS_ERR_NO_DEVICE;
    if (device < 0 || device >= n) return LGS_ERR_INVALID_ARG;
    lgs_ctx* ctx = new lgs_ctx();
    ctx->device = device;
    if (hipSetDevice(device) != hipSuccess ||
        hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess ||
        hipMalloc(&ctx->zero, 32 * sizeof(double)) != hipSuccess ||
        hipMemsetAsync(ctx->zero, 0, 32 * sizeof(double), ctx->stream) != hipSuccess ||
        hipStreamSynchronize(ctx->stream) != hipSuccess) {
        delete ctx;
        return LGS_ERR_HIP;
    }
    int lo = 0, hi = 0;
    if (hipDeviceGetStreamPriorityRange(&lo, &hi) != hipSuccess ||
        hipStreamCreateWithPriority(&ctx->hi, hipStreamNonBlocking, hi) != hipSuccess ||
        hipEventCreateWithFlags(&ctx->split_ev[0], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&ctx->split_ev[1], hipEventDisableTiming) != hipSuccess) {
        ctx->release();
        delete ctx;
        return LGS_ERR_HIP;
    }
    *out = ctx;
    return LGS_OK;
}

extern "C" void lgs_ctx_destroy(lgs_ctx* ctx)
{
    if (!ctx) return;
    hipSetDevice(ctx->device);
    ctx->release();
    delete ctx;
}

extern "C" const char* lgs_ctx_last_error(const lgs_ctx* ctx)
{
    return ctx ? ctx->last_error.c_str() : "null context";
}

extern "C" int lgs_ctx_synchronize(lgs_ctx* ctx)
{
    if (!ctx) return LGS_ERR_INVALID_ARG;
    return guarded(ctx, [&] { ctx->sync(); });
}

extern "C" int lgs_ctx_kernel_stats(lgs_ctx* ctx, lgs_kernel_stat* out, int cap)
{
    if (!ctx) return -LGS_ERR_INVALID_ARG;
    int rc = guarded(ctx, [&] {
        ctx->sync();
        ctx->harvest();
    });
    if (rc != LGS_OK) return -rc;
    int n = 0;
    for (int k = 0; k < K_NUM_KERNELS; ++k) {
        if (ctx->stat_launches[k] == 0) continue;
        if (out && n < cap) {
            std::memset(&out[n], 0, sizeof(out[n]));
            std::strncpy(out[n].name, kKernelNames[k], sizeof(out[n].name) - 1);
            out[n].launches = ctx->stat_launches[k];
            out[n].total_ms = ctx->stat_ms[k];
            out[n].algo_bytes = ctx->stat_bytes[k];
            out[n].dispatch_ms = ctx->stat_disp_ms[k];
        }
        ++n;
    }
    return n;
}

extern "C" int lgs_ctx_reset_stats(lgs_ctx* ctx)
{
    if (!ctx) return LGS_ERR_INVALID_ARG;
    return guarded(ctx, [&] {
        ctx->sync();
        ctx->harvest();
        for (int k = 0; k < K_NUM_KERNELS; ++k) {
            ctx->stat_launches[k] = 0;
            ctx->stat_ms[k] = 0;
            ctx->stat_bytes[k] = 0;
            ctx->stat_disp_ms[k] = 0;
        }
        ctx->count_matches = ctx->count_coarse_blocks = ctx->count_coarse_blocks_dense = ctx->count_pruned = 0;
    });
}

extern "C" int lgs_ctx_match_counters(lgs_ctx* ctx, int64_t* out4)
{
    if (!ctx || !out4) return LGS_ERR_INVALID_ARG;
    out4[0] = ctx->count_matches;
    out4[1] = ctx->count_coarse_blocks;
    out4[2] = ctx->count_coarse_blocks_dense;
    out4[3] = ctx->count_pruned;
    return LGS_OK;
}

extern "C" void* lgs_ctx_stream(lgs_ctx* ctx) { return ctx ? (void*)ctx->stream : nullptr; }

extern "C" int lgs_ctx_set_option(lgs_ctx* ctx, int option, double value)
{
    if (!ctx) return LGS_ERR_INVALID_ARG;
    switch (option) {
    case LGS_OPT_GUARD_EPS: ctx->guard_eps = value; return LGS_OK;
    case LGS_OPT_FORCE_DENSE: ctx->force_dense = value != 0.0; return LGS_OK;
    case LGS_OPT_INJECT_INDEX: ctx->inject_index = value != 0.0; return LGS_OK;
    case LGS_OPT_PROFILE:
        ctx->profile = value != 0.0;
        ctx->profile_mask = ~0u;
        return LGS_OK;
    case LGS_OPT_SPIN_SYNC: ctx->spin_sync = value != 0.0; return LGS_OK;
    case LGS_OPT_PROFILE_MASK:
        ctx->profile_mask = (unsigned)value;
        ctx->profile = ctx->profile_mask != 0;
        return LGS_OK;
    case LGS_OPT_SUPER_PRUNE: ctx->super_prune = value != 0.0; return LGS_OK;
    case LGS_OPT_LANES_MIN_BATCH: ctx->lanes_min_batch = (int)value; return LGS_OK;
    case LGS_OPT_RAY_CHUNK_KEYS:
        if (!(value >= 1.0)) return LGS_ERR_INVALID_ARG;
        ctx->ray_chunk_keys = (long long)std::min(value, (double)(1LL << 30));
        return LGS_OK;
    case LGS_OPT_SKIP_MASK: ctx->skip_mask = (unsigned)value; return LGS_OK;
    case LGS_OPT_POISON_WS: ctx->poison_ws = value != 0.0; return LGS_OK;
    case LGS_OPT_PEER_COPY: ctx->peer_staged = value != 0.0; return LGS_OK;
    case LGS_OPT_PRUNE_MIN_SUPER: ctx->prune_min_super = (int)value; return LGS_OK;
    case LGS_OPT_COOP_TILES: ctx->coop_tiles = (long long)value; return LGS_OK;
    case LGS_OPT_FINE_STAGED: ctx->fine_staged = value != 0.0; return LGS_OK;
    case LGS_OPT_SMALL_WINDOW: ctx->small_window = value != 0.0; return LGS_OK;
    case LGS_OPT_POST_RECORDS: ctx->post_records = value != 0.0; return LGS_OK;
    case LGS_OPT_FUSED_PLANES: ctx->fused_planes = value != 0.0; return LGS_OK;
    case LGS_OPT_PRIORITY_TAIL: ctx->prio_tail = value != 0.0; return LGS_OK;
    case LGS_OPT_DEVICE_TIMING: ctx->dev_timing = value != 0.0; return LGS_OK;
    case LGS_OPT_HV_FULL: ctx->hv_full = value != 0.0; return LGS_OK;
    case LGS_OPT_SPLIT_CHUNKS: ctx->split_chunks = value != 0.0; return LGS_OK;
    case LGS_OPT_DEVICE_HITS: ctx->device_hits = value != 0.0; return LGS_OK;
    case LGS_OPT_ZERO_TILES: ctx->zero_tiles = value != 0.0; return LGS_OK;
    case LGS_OPT_LEAN_PROJECT: ctx->lean_project = value != 0.0; return LGS_OK;
    case LGS_OPT_SEED_WIDE:
        if (!(value >= 0.0 && value <= 16.0)) return LGS_ERR_INVALID_ARG;
        ctx->seed_wide = (int)value;
        return LGS_OK;
    case LGS_OPT_SORT_BARRIER_US:
        if (value < 0) return LGS_ERR_INVALID_ARG;
        ctx->sort_barrier_us = (long long)value;
        return LGS_OK;
    case LGS_OPT_LINSOLVE_SPLIT: ctx->linsolve_split = value != 0.0; return LGS_OK;
    case LGS_OPT_HANDOFF_SPIN_US:
        if (value < 0.0) return LGS_ERR_INVALID_ARG;
        ctx->handoff_spin_us = (long long)value;
        return LGS_OK;
    case LGS_OPT_GUARD_CAP:
        ctx->guard_cap = (int)value;
        if (ctx->guard_cap < 0) ctx->guard_cap = 0;
        if (ctx->guard_cap > kGuardInline) ctx->guard_cap = kGuardInline;
        return LGS_OK;
    default: ctx->last_error = "unknown option"; return LGS_ERR_INVALID_ARG;
    }
}

// ---------------------------------------------------------------------------
// grids
// ---------------------------------------------------------------------------
__global__ void k_fill(double* __restrict__ d, size_t n, double v)
{
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    size_t stride = (size_t)gridDim.x * blockDim.x;
    for (; i < n; i += stride) d[i] = v;
}

extern "C" int lgs_grid_create(lgs_ctx* ctx, int w, int h, double min_x, double min_y,
                               double res, lgs_grid** out)
{
    if (!ctx || !out) return LGS_ERR_INVALID_ARG;
    *out = nullptr;
    return guarded(ctx, [&] {
        LGS_REQUIRE(w >= 0 && h >= 0 && res > 0.0, "invalid grid geometry");
        LGS_HIP_CHECK(hipSetDevice(ctx->device));
        lgs_grid* g = new lgs_grid();
        g->ctx = ctx;
        g->device = ctx->device;
        g->w = w;
        g->h = h;
        g->min_x = min_x;
        g->min_y = min_y;
        g->res = res;
        g->owned = true;
        size_t bytes = (size_t)w * (size_t)h * sizeof(double);
        if (bytes == 0) bytes = sizeof(double);
        if (hipMalloc(&g->d, bytes) != hipSuccess) {
            delete g;
            throw Error(LGS_ERR_OOM, "hipMalloc failed for grid");
        }
        LGS_HIP_CHECK(hipMemsetAsync(g->d, 0, bytes, ctx->stream));
        ctx->sync();
        *out = g;
    });
}

extern "C" int lgs_grid_wrap(lgs_ctx* ctx, double* dev, int w, int h, double min_x,
                             double min_y, double res, lgs_grid** out)
{
    if (!ctx || !out) return LGS_ERR_INVALID_ARG;
    *out = nullptr;
    return guarded(ctx, [&] {
        LGS_REQUIRE(dev != nullptr && w >= 0 && h >= 0 && res > 0.0, "invalid grid view");
        lgs_grid* g = new lgs_grid();
        g->ctx = ctx;
        g->device = ctx->device;
        g->d = dev;
        g->w = w;
        g->h = h;
        g->min_x = min_x;
        g->min_y = min_y;
        g->res = res;
        g->owned = false;
        *out = g;
    });
}

extern "C" void lgs_grid_destroy(lgs_grid* g)
{
    if (!g || g->map_view) return;  // map views live and die with their lgs_map
    // hipFree synchronises with the device; the creating context may already
    // be gone, so it is not touched here.
    if (g->owned && g->d) {
        hipSetDevice(g->device);
        hipFree(g->d);
    }
    delete g;
}

extern "C" int lgs_grid_upload(lgs_ctx* ctx, lgs_grid* g, const double* host)
{
    if (!ctx || !g || !host) return LGS_ERR_INVALID_ARG;
    return guarded(ctx, [&] {
        LGS_REQUIRE(!g->map_view, "cannot upload into a map's grid view");
        size_t bytes = (size_t)g->w * (size_t)g->h * sizeof(double);
        if (!bytes) return;
        grid_acquire(ctx, g);
        LGS_HIP_CHECK(hipMemcpyAsync(g->d, host, bytes, hipMemcpyHostToDevice, ctx->stream));
        ctx->sync();
    });
}

namespace {
// Dense grid from staged raw patch cells: one thread per cell, x fastest;
// slot[p] = staging index of patch p or -1 (unallocated: Unknown 0.0).  The
// value is one 8-byte load at value_offset of the cell (the vptr half of a
// 16-byte BinaryBayesGridCell is never read).
__global__ __launch_bounds__(256) void k_patch_ingest(double* __restrict__ grid, int W, int H, int ps, int npx,
                                                      const int* __restrict__ slot,
                                                      const unsigned char* __restrict__ cells, int cell_bytes,
                                                      int value_offset)
{
    const int x = blockIdx.x * blockDim.x + threadIdx.x;
    if (x >= W) return;
    for (int y = blockIdx.y; y < H; y += gridDim.y) {   // rows grid-stride (gridDim.y <= 65535)
        const int s = slot[(y / ps) * npx + x / ps];
        double v = 0.0;
        if (s >= 0) {
            const size_t c = (size_t)s * ps * ps + (size_t)(y % ps) * ps + (x % ps);
            v = *(const double*)(cells + c * cell_bytes + value_offset);
        }
        grid[(size_t)y * W + x] = v;
    }
}
}  // namespace

extern "C" int lgs_grid_upload_patches(lgs_ctx* ctx, lgs_grid* g, const void* const* patches, int npx, int npy,
                                       int ps, int cell_bytes, int value_offset)
{
    if (!ctx || !g || (!patches && npx * npy > 0)) return LGS_ERR_INVALID_ARG;
    return guarded(ctx, [&] {
        // a map's view: its cells change only through the map (counters, patch flags)
        LGS_REQUIRE(!g->map_view, "cannot upload into a map's grid view");
        LGS_REQUIRE(npx >= 0 && npy >= 0 && ps >= 1, "invalid patch geometry");
        LGS_REQUIRE((long long)npx * ps == g->w && (long long)npy * ps == g->h,
                    "grid size must be npx*patch_size x npy*patch_size");
        LGS_REQUIRE(cell_bytes >= 8 && cell_bytes % 8 == 0 && value_offset >= 0 && value_offset % 8 == 0 &&
                        value_offset + 8 <= cell_bytes,
                    "cell_bytes / value_offset must describe an aligned fp64 inside each cell");
        if (!g->w || !g->h) return;
        LGS_HIP_CHECK(hipSetDevice(ctx->device));
        grid_acquire(ctx, g);   // after any pending asynchronous writer of g
        const int np = npx * npy;
        const size_t patch_bytes = (size_t)ps * ps * cell_bytes;
        // slot table first (16-byte padded), then the allocated patches in table order
        const size_t b_slot = ((size_t)np * sizeof(int) + 15) / 16 * 16;
        std::vector<int> slot(np);
        std::vector<int> order;
        for (int p = 0; p < np; ++p) {
            slot[p] = patches[p] ? (int)order.size() : -1;
            if (patches[p]) order.push_back(p);
        }
        const int na = (int)order.size();
        const size_t total = b_slot + (size_t)na * patch_bytes;
        char* h = (char*)ctx->ensure_pinned_in(total);
        char* d = (char*)ctx->ensure(S_INGEST, total);
        std::memcpy(h, slot.data(), (size_t)np * sizeof(int));
        LGS_HIP_CHECK(hipMemcpyAsync(d, h, b_slot, hipMemcpyHostToDevice, ctx->stream));
        // host copies of chunk c (parallel over patches) overlap the DMA of chunk c - 1
        constexpr size_t kChunkBytes = 2u << 20;
        const int per_chunk = (int)std::max<size_t>(1, kChunkBytes / patch_bytes);
        for (int c0 = 0; c0 < na; c0 += per_chunk) {
            const int c1 = std::min(na, c0 + per_chunk);
            host_parallel_for(c1 - c0, 1, [&](int k) {
                std::memcpy(h + b_slot + (size_t)(c0 + k) * patch_bytes, patches[order[c0 + k]], patch_bytes);
            });
            LGS_HIP_CHECK(hipMemcpyAsync(d + b_slot + (size_t)c0 * patch_bytes, h + b_slot + (size_t)c0 * patch_bytes,
                                         (size_t)(c1 - c0) * patch_bytes, hipMemcpyHostToDevice, ctx->stream));
        }
        hipLaunchKernelGGL(k_patch_ingest, dim3((g->w + 255) / 256, std::min(g->h, 65535)), dim3(256), 0, ctx->stream,
                           g->d, g->w, g->h, ps, npx, (const int*)d, (const unsigned char*)(d + b_slot), cell_bytes, value_offset);
        LGS_HIP_CHECK(hipGetLastError());
        ctx->sync();
    });
}

extern "C" int lgs_grid_download(lgs_ctx* ctx, const lgs_grid* g, double* host)
{
    if (!ctx || !g || !host) return LGS_ERR_INVALID_ARG;
    return guarded(ctx, [&] {
        size_t bytes = (size_t)g->w * (size_t)g->h * sizeof(double);
        if (!bytes) return;
        grid_acquire(ctx, g);
        LGS_HIP_CHECK(hipMemcpyAsync(host, g->d, bytes, hipMemcpyDeviceToHost, ctx->stream));
        ctx->sync();
    });
}

extern "C" int lgs_grid_fill(lgs_ctx* ctx, lgs_grid* g, double v)
{
    if (!ctx || !g) return LGS_ERR_INVALID_ARG;
    return guarded(ctx, [&] {
        size_t n = (size_t)g->w * (size_t)g->h;
        if (!n) return;
        unsigned blocks = (unsigned)std::min<size_t>((n + 255) / 256, 4096);
        hipLaunchKernelGGL(k_fill, dim3(blocks), dim3(256), 0, ctx->stream, g->d, n, v);
        LGS_HIP_CHECK(hipGetLastError());
    });
}

extern "C" int lgs_grid_info(const lgs_grid* g, int* w, int* h, double* min_x, double* min_y,
                             double* res)
{
    if (!g) return LGS_ERR_INVALID_ARG;
    if (w) *w = g->w;
    if (h) *h = g->h;
    if (min_x) *min_x = g->min_x;
    if (min_y) *min_y = g->min_y;
    if (res) *res = g->res;
    return LGS_OK;
}

extern "C" double* lgs_grid_device_ptr(lgs_grid* g) { return g ? g->d : nullptr; }

// ---------------------------------------------------------------------------
// K2: coarse-map precompute (2-D forward window max), LDS tiled
// ---------------------------------------------------------------------------
namespace {

constexpr int kTileX = 64;
constexpr int kTileY = 32;
constexpr int kMaxWinTiled = 32;

// window start of output i over n cells with window w (SlidingWindowMax)
__device__ __forceinline__ int win_start(int i, int n, int w) { return (n >= w) ? min(i, n - w) : 0; }

__device__ __forceinline__ double dmax(double a, double b) { return (a < b) ? b : a; }

// One workgroup computes a kTileX x kTileY block of outputs.  The input
// footprint [sx0, sx1) x [sy0, sy1) is staged in LDS (zero outside the grid),
// then the y-pass (SlidingWindowMaxRow) and x-pass (SlidingWindowMaxCol) run
// from LDS.
// pg.Wqp > 0: the output is written directly into the interior of the padded
// phase-plane layout of k_rtcsm.hip (plane ry*w + rx, row y/w + M, column
// x/w + M; requires W, H multiples of w).
__device__ __forceinline__ void precompute_tile(const double* __restrict__ in, double* __restrict__ out, int W,
                                                int H, int w, const PlaneGeom& pg, int bx, int by)
{
    extern __shared__ double lds[];
    const int x0 = bx * kTileX, y0 = by * kTileY;
    const int x1 = min(x0 + kTileX, W), y1 = min(y0 + kTileY, H);
    const int sx0 = win_start(x0, W, w), sy0 = win_start(y0, H, w);
    const int sx1 = win_start(x1 - 1, W, w) + w, sy1 = win_start(y1 - 1, H, w) + w;
    const int fw = sx1 - sx0, fh = sy1 - sy0;  // footprint (<= tile + w - 1)
    double* tile = lds;                          // [fh][fw]
    double* m1 = lds + fh * fw;                  // [y1-y0][fw]
    const int tid = threadIdx.x;
    for (int k0 = tid; k0 < fh * fw; k0 += 8 * (int)blockDim.x) {   // 8 loads in flight per thread
        double v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int k = k0 + j * (int)blockDim.x;
            const int yy = sy0 + k / fw, xx = sx0 + k % fw;
            v[j] = (k < fh * fw && xx < W && yy < H) ? in[(size_t)yy * W + xx] : 0.0;
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int k = k0 + j * (int)blockDim.x;
            if (k < fh * fw) tile[k] = v[j];
        }
    }
    __syncthreads();
    const int oh = y1 - y0;
    for (int k = tid; k < oh * fw; k += blockDim.x) {
        const int oy = k / fw, cx = k % fw;
        const int s = win_start(y0 + oy, H, w) - sy0;
        double m = tile[s * fw + cx];
        for (int j = 1; j < w; ++j) m = dmax(m, tile[(s + j) * fw + cx]);
        m1[oy * fw + cx] = m;
    }
    __syncthreads();
    const int ow = x1 - x0;
    for (int k = tid; k < oh * ow; k += blockDim.x) {
        const int oy = k / ow, ox = k % ow;
        const int s = win_start(x0 + ox, W, w) - sx0;
        double m = m1[oy * fw + s];
        for (int j = 1; j < w; ++j) m = dmax(m, m1[oy * fw + s + j]);
        const int x = x0 + ox, y = y0 + oy;
        if (pg.Wqp > 0) {
            const int qx = x / w, qy = y / w, rx = x - qx * w, ry = y - qy * w;
            out[(ry * w + rx) * pg.pstride + (long long)(qy + pg.M) * pg.Wqp + qx + pg.M] = m;
        } else {
            out[(size_t)y * W + x] = m;
        }
    }
}

__global__ __launch_bounds__(256) void k_precompute_tiled(const double* __restrict__ in,
                                                          double* __restrict__ out, int W,
                                                          int H, int w, PlaneGeom pg)
{
    precompute_tile(in, out, W, H, w, pg, blockIdx.x, blockIdx.y);
}

// Batched precompute straight into the padded phase planes (W, H multiples of
// the window LR <= 8).  A tile is kPQX coarse columns x kPTY fine rows.
//  1. y pass (SlidingWindowMaxRow) in registers: a thread owns footprint
//     columns, loads its column's kPTY + LR - 1 values once (all loads issued
//     before any max) and writes the kPTY window maxima to LDS;
//  2. x pass (SlidingWindowMaxCol) from LDS, each thread producing TWO
//     consecutive coarse columns of one plane row and writing them with one
//     16-byte store (padded plane rows are even, so the pair is aligned); the
//     lanes of a wave walk a plane row, so a wave writes 512-byte runs.
// Same values as the reference's passes (max is exact).
// tile rows: 8 for a batch's maps (r05: with zero tiles most workgroups only
// read their footprint, and the shorter tiles' smaller LDS rows let more of
// them run per CU); a lone map (one job) takes 4-row tiles, more workgroups
// for its ~250 tiles (latency, not bandwidth, bounds a single 1000 x 1000 map)
#ifndef LGS_PTY_BATCH
#define LGS_PTY_BATCH 8   // measured (64 config-2 maps, zero tiles on): 32: 0.374 ms, 16: 0.189, 8: 0.150, 4: 0.173
#endif
#ifndef LGS_PTY_LONE
#define LGS_PTY_LONE 4   // measured (lone config-2 map): 16: 16.4 us, 8: 13.3, 4: 11.5
#endif
// coarse columns per tile: the footprint (kPQX * LR + LR - 1 fine columns) fits
// the 256 threads of the y pass, and kPQX is even (column pairs)
constexpr int pqx_of(int LR) { return ((257 - LR) / LR) & ~1; }
template <int LR>
constexpr int pqx() { return pqx_of(LR); }
typedef double d2a16 __attribute__((ext_vector_type(2)));
template <int LR, int kPTY = 16>
__global__ __launch_bounds__(256) void k_precompute_planes(const PrecompJob* __restrict__ jobs, DevTs dts)
{
    const DtsScope dts_scope(dts);
    const int gx = gridDim.x, gy = gridDim.y, nwg = gx * gy * gridDim.z;
    const int b = blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z);
    const int xcd = b & 7, q = nwg >> 3, r = nwg & 7;
    const int l = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (b >> 3);
#ifdef LGS_NO_XCD
    const int bx = blockIdx.x, by = blockIdx.y, bz = blockIdx.z;
    (void)l;
#else
    // wave-uniform by construction: readfirstlane lets the job descriptor be
    // read with scalar loads (the divisions put them in vector registers)
    const int bx = __builtin_amdgcn_readfirstlane(l % gx), by = __builtin_amdgcn_readfirstlane((l / gx) % gy),
              bz = __builtin_amdgcn_readfirstlane(l / (gx * gy));
#endif
    const PrecompJob& j = jobs[bz];
    const int W = j.W, H = j.H;
    constexpr int kPQX = pqx<LR>();
    const int x0 = bx * kPQX * LR, y0 = by * kPTY;
    if (x0 >= W || y0 >= H) return;   // past this job's map (uniform)
    const int x1 = min(x0 + kPQX * LR, W), y1 = min(y0 + kPTY, H);
    const int sx0 = win_start(x0, W, LR), sy0 = win_start(y0, H, LR);
    const int sx1 = win_start(x1 - 1, W, LR) + LR;
    const int fw = sx1 - sx0;
    const int oh = y1 - y0;
    constexpr int FW = kPQX * LR + LR - 1;
    static_assert(FW <= 256, "one footprint column per thread");
    constexpr int FH = kPTY + LR - 1;
    __shared__ double m1[kPTY][FW];
    const double* __restrict__ in = j.in;
    const int tid = threadIdx.x;
    int nz = 0;   // a footprint value of this thread is not +0
    for (int c = tid; c < fw; c += 256) {   // one column per thread (FW <= 256)
        const int xx = sx0 + c;
        double v[FH];
#pragma unroll
        for (int k = 0; k < FH; ++k) {
            const int yy = sy0 + k;
            v[k] = (xx < W && yy < H) ? gload(in + ((size_t)yy * W + xx)) : 0.0;   // reads past the end are 0
        }
#pragma unroll
        for (int k = 0; k < FH; ++k) nz |= __double_as_longlong(v[k]) != 0;
        // window maxima of every start row (static register indices), then row
        // oy takes the window starting at win_start(y0 + oy) - sy0 =
        // min(oy + d, st) (the tail repeats the last full window)
        double wm[kPTY];
#pragma unroll
        for (int k = 0; k < kPTY; ++k) {
            double m = v[k];
#pragma unroll
            for (int i = 1; i < LR; ++i) m = dmax(m, v[k + i]);
            wm[k] = m;
        }
        const int d = y0 - sy0, st = max(0, H - LR - sy0);
        if (d == 0 && st >= kPTY - 1) {   // interior tiles (uniform): row oy's window starts at oy
#pragma unroll
            for (int oy = 0; oy < kPTY; ++oy)
                if (oy < oh) m1[oy][c] = wm[oy];
        } else {
#pragma unroll
            for (int oy = 0; oy < kPTY; ++oy) {
                const int s = min(oy + d, st);
                double m = wm[0];
#pragma unroll
                for (int k = 1; k < kPTY; ++k) m = (k == s) ? wm[k] : m;
                if (oy < oh) m1[oy][c] = m;
            }
        }
    }
    // zero tiles: an all-(+0) footprint gives +0 in every plane and fp16
    // output of the tile; when the set's word says the tile already holds
    // them (its previous build read an all-zero footprint too), nothing is
    // stored -- an unknown map's empty patches cost their reads only
    unsigned* zw = j.zt ? j.zt + (by * gx + bx) : nullptr;   // uniform per workgroup
    if (zw) {
        const unsigned zprev = *zw;              // every thread reads it before the barrier,
        const int anynz = __syncthreads_or(nz);  // thread 0 rewrites it after
        if (!anynz && zprev == 1u) return;
        if (tid == 0 && zprev != (anynz ? 0u : 1u)) *zw = anynz ? 0u : 1u;
    } else {
        __syncthreads();
    }
    const PlaneGeom& pg = j.pg;
    const int nq = (x1 - x0) / LR;        // coarse columns of this tile (W is a multiple of LR)
    const int np = (nq + 1) >> 1;         // column pairs
    double* __restrict__ out = j.out;
    for (int k = tid; k < oh * LR * (kPQX / 2); k += 256) {   // (row, plane column, pair), pair fastest
        const int oy = k / (LR * (kPQX / 2)), rem = k % (LR * (kPQX / 2));
        const int rx = rem / (kPQX / 2), p = rem % (kPQX / 2);
        if (p >= np) continue;
        const int qxl = 2 * p;
        const int xa = x0 + qxl * LR + rx;
        const double* ca = &m1[oy][win_start(xa, W, LR) - sx0];
        double ma = ca[0];
#pragma unroll
        for (int i = 1; i < LR; ++i) ma = dmax(ma, ca[i]);
        const int y = y0 + oy, qy = y / LR, ry = y - qy * LR;
        const long long o = (ry * LR + rx) * pg.pstride + (long long)(qy + pg.M) * pg.Wqp + (x0 / LR + qxl) + pg.M;
        double* dst = out + o;
        if (qxl + 1 < nq) {
            const int xb = xa + LR;
            const double* cb = &m1[oy][win_start(xb, W, LR) - sx0];
            double mb = cb[0];
#pragma unroll
            for (int i = 1; i < LR; ++i) mb = dmax(mb, cb[i]);
            d2a16 v;
            v.x = ma;
            v.y = mb;
            gstore((d2a16*)dst, v);
            if (j.out16) {   // the pair's fp16 round-ups (o is even: 4-byte aligned)
                gstore((unsigned*)(j.out16 + o),
                       (unsigned)half_round_up_bits(ma) | ((unsigned)half_round_up_bits(mb) << 16));
                if (ma < 0.0 || mb < 0.0) gstore(j.negflag, j.pgen);
            }
        } else {
            gstore(dst, ma);
            if (j.out16) {
                gstore(j.out16 + o, half_round_up_bits(ma));
                if (ma < 0.0) gstore(j.negflag, j.pgen);
            }
        }
    }
}

// Column-streaming batched precompute: one workgroup walks kSub consecutive
// kPTY-row tiles of one tile column, so a footprint row is loaded once (the
// LR - 1 halo rows carry over in registers) and the next tile's rows are in
// flight while this tile's x pass runs.  Tiles, zero-tile words and outputs
// are those of k_precompute_planes<LR, kPTY> (tile row by = blockIdx.y *
// kSub + s of gyt).
#ifndef LGS_PTY_SUB
#define LGS_PTY_SUB 2   // measured (64 config-2 maps, one stream): 1: 0.145 ms, 2: 0.116, 3: 0.124, 4: 0.120, 8: 0.122
#endif
template <int LR, int kPTY, int kSub>
__global__ __launch_bounds__(256) void k_precompute_planes_s(const PrecompJob* __restrict__ jobs, int gyt, DevTs dts)
{
    const DtsScope dts_scope(dts);
    const int gx = gridDim.x, gy = gridDim.y, nwg = gx * gy * gridDim.z;
    const int b = blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z);
    const int xcd = b & 7, q = nwg >> 3, r = nwg & 7;
    const int l = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (b >> 3);
    const int bx = __builtin_amdgcn_readfirstlane(l % gx), bys = __builtin_amdgcn_readfirstlane((l / gx) % gy),
              bz = __builtin_amdgcn_readfirstlane(l / (gx * gy));
    const PrecompJob& j = jobs[bz];
    const int W = j.W, H = j.H;
    constexpr int kPQX = pqx<LR>();
    constexpr int FW = kPQX * LR + LR - 1;
    static_assert(FW <= 256, "one footprint column per thread");
    constexpr int FH = kPTY + LR - 1;
    const int x0 = bx * kPQX * LR;
    if (x0 >= W) return;   // past this job's map (uniform)
    const int x1 = min(x0 + kPQX * LR, W);
    const int sx0 = win_start(x0, W, LR);
    const int fw = win_start(x1 - 1, W, LR) + LR - sx0;
    __shared__ double m1[kPTY][FW];
    const double* __restrict__ in = j.in;
    const int tid = threadIdx.x;
    const int xx = sx0 + tid;
    const bool col = tid < fw, cin = col && xx < W;   // reads past the end are 0
    const int nq = (x1 - x0) / LR, np = (nq + 1) >> 1;
    const PlaneGeom& pg = j.pg;
    double* __restrict__ out = j.out;
    double v[FH];
    const int by0 = bys * kSub;
    // prologue: the first tile's footprint rows
    int sy0 = win_start(by0 * kPTY, H, LR);
    if (by0 >= gyt || by0 * kPTY >= H) return;
#pragma unroll
    for (int k = 0; k < FH; ++k) {
        const int yy = sy0 + k;
        v[k] = (cin && yy < H) ? gload(in + ((size_t)yy * W + xx)) : 0.0;
    }
    for (int s = 0; s < kSub; ++s) {
        const int by = by0 + s, y0 = by * kPTY;
        if (by >= gyt || y0 >= H) break;   // uniform
        const int y1 = min(y0 + kPTY, H), oh = y1 - y0;
        int nz = 0;
#pragma unroll
        for (int k = 0; k < FH; ++k) nz |= __double_as_longlong(v[k]) != 0;
        double wm[kPTY];
#pragma unroll
        for (int k = 0; k < kPTY; ++k) {
            double m = v[k];
#pragma unroll
            for (int i = 1; i < LR; ++i) m = dmax(m, v[k + i]);
            wm[k] = m;
        }
        if (s > 0) __syncthreads();   // the previous tile's x pass is done with m1
        const int d = y0 - sy0, st = max(0, H - LR - sy0);
        if (col) {
            if (d == 0 && st >= kPTY - 1) {
#pragma unroll
                for (int oy = 0; oy < kPTY; ++oy)
                    if (oy < oh) m1[oy][tid] = wm[oy];
            } else {
#pragma unroll
                for (int oy = 0; oy < kPTY; ++oy) {
                    const int sr = min(oy + d, st);
                    double m = wm[0];
#pragma unroll
                    for (int k = 1; k < kPTY; ++k) m = (k == sr) ? wm[k] : m;
                    if (oy < oh) m1[oy][tid] = m;
                }
            }
        }
        // the next tile's rows go in flight now (its halo rows carry over when
        // its footprint continues this one's), under this tile's x pass
        const int nby = by + 1;
        if (s + 1 < kSub && nby < gyt && nby * kPTY < H) {
            const int nsy0 = win_start(nby * kPTY, H, LR);
            if (nsy0 == sy0 + kPTY) {
#pragma unroll
                for (int k = 0; k < LR - 1; ++k) v[k] = v[k + kPTY];
#pragma unroll
                for (int k = LR - 1; k < FH; ++k) {
                    const int yy = nsy0 + k;
                    v[k] = (cin && yy < H) ? gload(in + ((size_t)yy * W + xx)) : 0.0;
                }
            } else {
#pragma unroll
                for (int k = 0; k < FH; ++k) {
                    const int yy = nsy0 + k;
                    v[k] = (cin && yy < H) ? gload(in + ((size_t)yy * W + xx)) : 0.0;
                }
            }
            sy0 = nsy0;
        }
        unsigned* zw = j.zt ? j.zt + (by * gx + bx) : nullptr;   // uniform per workgroup
        if (zw) {
            const unsigned zprev = *zw;
            const int anynz = __syncthreads_or(nz);
            if (tid == 0 && zprev != (anynz ? 0u : 1u)) *zw = anynz ? 0u : 1u;
            if (!anynz && zprev == 1u) continue;
        } else {
            __syncthreads();
        }
        for (int k = tid; k < oh * LR * (kPQX / 2); k += 256) {   // as k_precompute_planes
            const int oy = k / (LR * (kPQX / 2)), rem = k % (LR * (kPQX / 2));
            const int rx = rem / (kPQX / 2), p = rem % (kPQX / 2);
            if (p >= np) continue;
            const int qxl = 2 * p;
            const int xa = x0 + qxl * LR + rx;
            const double* ca = &m1[oy][win_start(xa, W, LR) - sx0];
            double ma = ca[0];
#pragma unroll
            for (int i = 1; i < LR; ++i) ma = dmax(ma, ca[i]);
            const int y = y0 + oy, qy = y / LR, ry = y - qy * LR;
            const long long o = (ry * LR + rx) * pg.pstride + (long long)(qy + pg.M) * pg.Wqp + (x0 / LR + qxl) + pg.M;
            double* dst = out + o;
            if (qxl + 1 < nq) {
                const int xb = xa + LR;
                const double* cb = &m1[oy][win_start(xb, W, LR) - sx0];
                double mb = cb[0];
#pragma unroll
                for (int i = 1; i < LR; ++i) mb = dmax(mb, cb[i]);
                d2a16 vv;
                vv.x = ma;
                vv.y = mb;
                gstore((d2a16*)dst, vv);
                if (j.out16) {
                    gstore((unsigned*)(j.out16 + o),
                           (unsigned)half_round_up_bits(ma) | ((unsigned)half_round_up_bits(mb) << 16));
                    if (ma < 0.0 || mb < 0.0) gstore(j.negflag, j.pgen);
                }
            } else {
                gstore(dst, ma);
                if (j.out16) {
                    gstore(j.out16 + o, half_round_up_bits(ma));
                    if (ma < 0.0) gstore(j.negflag, j.pgen);
                }
            }
        }
    }
}

// Batched: job blockIdx.z (maps of a batch may differ in size; the grid
// covers the largest, tiles past a job's map exit).
// XCD-aware order (speed only): one map's tiles on one XCD (see k_rtcsm.hip xcd_block)
__global__ __launch_bounds__(256) void k_precompute_jobs(const PrecompJob* __restrict__ jobs, int w)
{
    const int gx = gridDim.x, gy = gridDim.y, nwg = gx * gy * gridDim.z;
    const int b = blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z);
    const int xcd = b & 7, q = nwg >> 3, r = nwg & 7;
    const int l = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (b >> 3);
#ifdef LGS_NO_XCD
    const int bx = blockIdx.x, by = blockIdx.y, bz = blockIdx.z;
    (void)l;
#else
    const int bx = __builtin_amdgcn_readfirstlane(l % gx), by = __builtin_amdgcn_readfirstlane((l / gx) % gy),
              bz = __builtin_amdgcn_readfirstlane(l / (gx * gy));
#endif
    const PrecompJob& j = jobs[bz];
    if (bx * kTileX >= j.W || by * kTileY >= j.H) return;
    precompute_tile(j.in, j.out, j.W, j.H, w, j.pg, bx, by);
}

// Large windows (> 32, e.g. the branch-and-bound pyramid's 64): the two
// separable passes as their own launches through a scratch map, each output
// the max of its w window (SlidingWindowMaxRow, then SlidingWindowMaxCol;
// win_start gives the tail rule, reads past the end are 0).
__global__ void k_precompute_sep_y(const double* __restrict__ in, double* __restrict__ out, int W, int H, int w)
{
    const int x = blockIdx.x * blockDim.x + threadIdx.x;
    const int y = blockIdx.y;
    if (x >= W) return;
    const int s = win_start(y, H, w);
    double m = 0.0;
    for (int j = 0; j < w; ++j) {
        const double v = (s + j < H) ? in[(size_t)(s + j) * W + x] : 0.0;
        m = (j == 0) ? v : dmax(m, v);
    }
    out[(size_t)y * W + x] = m;
}

__global__ void k_precompute_sep_x(const double* __restrict__ in, double* __restrict__ out, int W, int H, int w)
{
    const int x = blockIdx.x * blockDim.x + threadIdx.x;
    const int y = blockIdx.y;
    if (x >= W) return;
    const int s = win_start(x, W, w);
    const double* row = in + (size_t)y * W;
    double m = 0.0;
    for (int j = 0; j < w; ++j) {
        const double v = (s + j < W) ? row[s + j] : 0.0;
        m = (j == 0) ? v : dmax(m, v);
    }
    out[(size_t)y * W + x] = m;
}

}  // namespace

namespace lgs {
bool precompute_planes_ok(const lgs_grid* in, int win)
{
    return win >= 1 && win <= kMaxWinTiled && in->w % win == 0 && in->h % win == 0;
}

void launch_precompute(lgs_ctx* ctx, const lgs_grid* in, int win, double* out, const PlaneGeom* planes)
{
    LGS_REQUIRE(!planes || precompute_planes_ok(in, win), "phase-plane precompute needs W, H multiples of the window");
    const PlaneGeom pg = planes ? *planes : PlaneGeom{ 0, 0, 0 };
    if (in->w == 0 || in->h == 0) return;
    // algorithmic bytes: two separable passes, each reading and
    // writing one fp64 per cell = 32 B/cell
    const int tok = ctx->timing_begin(K_PRECOMPUTE, 32.0 * (double)in->w * (double)in->h);
    if (ctx->skipped(K_PRECOMPUTE)) {
    } else if (win <= kMaxWinTiled) {
        const int fw = kTileX + win - 1, fh = kTileY + win - 1;
        const size_t lds = (size_t)(fh * fw + kTileY * fw) * sizeof(double);
        dim3 grid((in->w + kTileX - 1) / kTileX, (in->h + kTileY - 1) / kTileY);
        hipLaunchKernelGGL(k_precompute_tiled, grid, dim3(256), lds, ctx->stream, in->d, out,
                           in->w, in->h, win, pg);
    } else {
        LGS_REQUIRE(!planes, "phase-plane precompute: window must be <= 32");
        double* tmp = (double*)ctx->ensure(S_PRECOMP_TMP, sizeof(double) * (size_t)in->w * in->h);
        dim3 grid((in->w + 255) / 256, in->h);
        hipLaunchKernelGGL(k_precompute_sep_y, grid, dim3(256), 0, ctx->stream, in->d, tmp, in->w, in->h, win);
        hipLaunchKernelGGL(k_precompute_sep_x, grid, dim3(256), 0, ctx->stream, tmp, out, in->w, in->h, win);
    }
    ctx->timing_end(tok);
    LGS_HIP_CHECK(hipGetLastError());
}
// the tile grid of a plane precompute launch (win <= 8; one job: the lone
// LGS_PTY_LONE-row tiles, else 16-row tiles): k_rtcsm.hip's zero-tile words
// are indexed by it
void precompute_tile_grid(int maxW, int maxH, int win, int njobs, int* gx, int* gy, int* rows)
{
    const int q = pqx_of(win) * win;
    *rows = njobs == 1 ? LGS_PTY_LONE : LGS_PTY_BATCH;
    *gx = (maxW + q - 1) / q;
    *gy = (maxH + *rows - 1) / *rows;
}
void launch_precompute_jobs(lgs_ctx* ctx, const PrecompJob* d_jobs, int njobs, int maxW, int maxH, int win)
{
    LGS_REQUIRE(win >= 1 && win <= kMaxWinTiled, "batched precompute: window must be in [1, 32]");
    if (njobs == 0 || maxW == 0 || maxH == 0) return;
    const int tok = ctx->timing_begin(K_PRECOMPUTE, 32.0 * (double)maxW * (double)maxH * njobs);
    if (ctx->skipped(K_PRECOMPUTE)) {
    } else if (win <= 8) {
        // plane-ordered tiles (every job of this path writes planes)
        switch (win) {
#define LGS_PP_CASE(L) case L: \
            if (njobs == 1) \
                hipLaunchKernelGGL(HIP_KERNEL_NAME(k_precompute_planes<L, LGS_PTY_LONE>), \
                    dim3((maxW + pqx<L>() * L - 1) / (pqx<L>() * L), (maxH + LGS_PTY_LONE - 1) / LGS_PTY_LONE, njobs), \
                    dim3(256), 0, ctx->stream, d_jobs, ctx->dts(tok)); \
            else if (LGS_PTY_SUB > 1) { \
                const int gyt = (maxH + LGS_PTY_BATCH - 1) / LGS_PTY_BATCH; \
                hipLaunchKernelGGL(HIP_KERNEL_NAME(k_precompute_planes_s<L, LGS_PTY_BATCH, LGS_PTY_SUB>), \
                    dim3((maxW + pqx<L>() * L - 1) / (pqx<L>() * L), (gyt + LGS_PTY_SUB - 1) / LGS_PTY_SUB, njobs), \
                    dim3(256), 0, ctx->stream, d_jobs, gyt, ctx->dts(tok)); \
            } else \
                hipLaunchKernelGGL(HIP_KERNEL_NAME(k_precompute_planes<L, LGS_PTY_BATCH>), \
                    dim3((maxW + pqx<L>() * L - 1) / (pqx<L>() * L), (maxH + LGS_PTY_BATCH - 1) / LGS_PTY_BATCH, njobs), dim3(256), 0, ctx->stream, \
                    d_jobs, ctx->dts(tok)); \
            break;
        LGS_PP_CASE(1) LGS_PP_CASE(2) LGS_PP_CASE(3) LGS_PP_CASE(4) LGS_PP_CASE(5) LGS_PP_CASE(6)
        LGS_PP_CASE(7) LGS_PP_CASE(8)
#undef LGS_PP_CASE
        }
    } else {
        const int fw = kTileX + win - 1, fh = kTileY + win - 1;
        const size_t lds = (size_t)(fh * fw + kTileY * fw) * sizeof(double);
        dim3 grid((maxW + kTileX - 1) / kTileX, (maxH + kTileY - 1) / kTileY, njobs);
        hipLaunchKernelGGL(k_precompute_jobs, grid, dim3(256), lds, ctx->stream, d_jobs, win);
    }
    ctx->timing_end(tok);
    LGS_HIP_CHECK(hipGetLastError());
}
}  // namespace lgs

extern "C" int lgs_grid_precompute_max(lgs_ctx* ctx, const lgs_grid* in, int win, lgs_grid* out)
{
    if (!ctx || !in || !out) return LGS_ERR_INVALID_ARG;
    return guarded(ctx, [&] {
        LGS_REQUIRE(win >= 1, "window must be >= 1");
        LGS_REQUIRE(out->w == in->w && out->h == in->h, "precompute output geometry mismatch");
        LGS_REQUIRE(out->d != in->d, "precompute cannot run in place");
        grid_acquire(ctx, in);
        out->min_x = in->min_x;
        out->min_y = in->min_y;
        out->res = in->res;
        launch_precompute(ctx, in, win, out->d, nullptr);
    });
}

// ---------------------------------------------------------------------------
// scans
// ---------------------------------------------------------------------------
namespace {
// A scan's device copy (ranges then angles, one allocation) comes from a small
// per-device pool: a frontend creates and drops two scans per step, and a
// hipMalloc/hipFree pair costs ~26 us each (hipFree also waits for the whole
// device).  A buffer goes back to the pool when its scan is destroyed; every
// library call that reads a scan's device copy finishes with it before it
// returns (the asynchronous latest-map step reads the host copy), so the
// buffer can be handed out again at once.  Buffers are binned by power-of-two
// size; the pool keeps at most kScanPoolBytes per device.
constexpr size_t kScanPoolBytes = size_t(64) << 20;
struct ScanPool {
    std::mutex mu;
    std::vector<std::vector<void*>> bins;   // bins[log2 bytes]
    size_t held = 0;
};
ScanPool& scan_pool(int device)
{
    static std::mutex mu;
    static std::vector<std::unique_ptr<ScanPool>> pools;
    std::lock_guard<std::mutex> g(mu);
    if ((int)pools.size() <= device) pools.resize((size_t)device + 1);
    if (!pools[device]) pools[device].reset(new ScanPool());
    return *pools[device];
}
int scan_bin(size_t bytes)
{
    int b = 8;
    while ((size_t(1) << b) < bytes) ++b;
    return b;
}
void* scan_buffer_get(int device, size_t bytes)
{
    const int b = scan_bin(bytes);
    ScanPool& P = scan_pool(device);
    {
        std::lock_guard<std::mutex> g(P.mu);
        if ((int)P.bins.size() > b && !P.bins[b].empty()) {
            void* p = P.bins[b].back();
            P.bins[b].pop_back();
            P.held -= size_t(1) << b;
            return p;
        }
    }
    void* p = nullptr;
    if (hipMalloc(&p, size_t(1) << b) != hipSuccess) throw Error(LGS_ERR_OOM, "hipMalloc failed for scan");
    return p;
}
void scan_buffer_put(int device, void* p, size_t bytes)
{
    const int b = scan_bin(bytes);
    ScanPool& P = scan_pool(device);
    {
        std::lock_guard<std::mutex> g(P.mu);
        if (P.held + (size_t(1) << b) <= kScanPoolBytes) {
            if ((int)P.bins.size() <= b) P.bins.resize((size_t)b + 1);
            P.bins[b].push_back(p);
            P.held += size_t(1) << b;
            return;
        }
    }
    hipSetDevice(device);
    hipFree(p);
}
}  // namespace

extern "C" int lgs_scan_create(lgs_ctx* ctx, const lgs_scan_host* hs, lgs_scan** out)
{
    if (!ctx || !hs || !out) return LGS_ERR_INVALID_ARG;
    *out = nullptr;
    return guarded(ctx, [&] {
        LGS_REQUIRE(hs->n >= 1 && hs->ranges && hs->angles, "scan must have >= 1 beam");
        LGS_HIP_CHECK(hipSetDevice(ctx->device));
        lgs_scan* s = new lgs_scan();
        std::unique_ptr<lgs_scan> own(s);
        static std::atomic<unsigned long long> uids{ 0 };
        s->uid = uids.fetch_add(1, std::memory_order_relaxed) + 1;
        s->ctx = ctx;
        s->device = ctx->device;
        s->n = hs->n;
        s->rel = hs->rel_sensor_pose;
        s->min_range = hs->min_range;
        s->max_range = hs->max_range;
        s->h_ranges.assign(hs->ranges, hs->ranges + hs->n);
        s->h_angles.assign(hs->angles, hs->angles + hs->n);
        double m = hs->ranges[0];  // std::max_element: first maximum
        for (int i = 1; i < hs->n; ++i)
            if (m < hs->ranges[i]) m = hs->ranges[i];
        s->max_elem = m;
        *out = own.release();   // the device copy is made at first use (lgs::scans_to_device)
    });
}

extern "C" int lgs_scan_get(const lgs_scan* s, int* n, double* ranges, double* angles)
{
    if (!s || !n) return LGS_ERR_INVALID_ARG;
    *n = s->n;
    if (ranges) std::memcpy(ranges, s->h_ranges.data(), sizeof(double) * (size_t)s->n);
    if (angles) std::memcpy(angles, s->h_angles.data(), sizeof(double) * (size_t)s->n);
    return LGS_OK;
}

// ScanInterpolator::Interpolate (C/mapping/scan_interpolator.cpp:9-98).  The
// walk along the polyline carries (previous point, accumulated distance) from
// point to point and revisits a point after each inserted one, so it is a
// sequential recurrence; it stays on the host with glibc's sincos (the
// reference's ToCartesianCoordinate sin/cos pair, H/util.hpp:148-152, fused by
// GCC), sqrt and atan2 (ToPolarCoordinate :156-161) for bit-exact points.
extern "C" int lgs_scan_interpolate(lgs_ctx* ctx, const lgs_scan* in, double dist_scans,
                                    double dist_threshold_empty, lgs_scan** out)
{
    if (!ctx || !in || !out) return LGS_ERR_INVALID_ARG;
    *out = nullptr;
    std::vector<double> rr, aa;
    int rc = guarded(ctx, [&] {
        LGS_REQUIRE(in->n >= 1, "scan must have >= 1 beam");
        // the walk below advances only if every distance is a number and a
        // point is inserted at most dist_scans along a segment: reject what
        // would make the reference's loop run forever (NaN/inf points,
        // dist_scans <= 0)
        LGS_REQUIRE(std::isfinite(dist_scans) && std::isfinite(dist_threshold_empty) && dist_scans > 0.0 &&
                        dist_scans <= dist_threshold_empty,
                    "need 0 < dist_scans <= dist_threshold_empty, both finite");
        const int n = in->n;
        std::vector<double> px(n), py(n);
        sincos_batch(in->h_angles.data(), n, py.data(), px.data());   // glibc's sincos, four at a time
        for (int i = 0; i < n; ++i) {
            px[i] = in->h_ranges[i] * px[i];
            py[i] = in->h_ranges[i] * py[i];
            LGS_REQUIRE(std::isfinite(px[i]) && std::isfinite(py[i]), "non-finite range or angle");
        }
        rr.reserve(2 * (size_t)n);
        aa.reserve(2 * (size_t)n);
        auto polar = [&](double x, double y) {
            rr.push_back(std::sqrt(x * x + y * y));
            aa.push_back(std::atan2(y, x));
        };
        polar(px[0], py[0]);
        double qx = px[0], qy = py[0], acc = 0.0;  // previous point, distance walked since it
        int i = 1;
        while (i < n) {
            const double dx = qx - px[i], dy = qy - py[i];
            const double d = std::sqrt(dx * dx + dy * dy);  // Distance (H/point.hpp:113-117)
            if (acc + d < dist_scans) {           // too close: walk on
                acc += d;
                qx = px[i], qy = py[i];
                ++i;
            } else if (acc + d >= dist_threshold_empty) {  // gap: keep the point as is
                polar(px[i], py[i]);
                qx = px[i], qy = py[i];
                acc = 0.0;
                ++i;
            } else {                              // insert a point dist_scans along the segment
                const double t = (dist_scans - acc) / d;
                const double nx = (px[i] - qx) * t + qx, ny = (py[i] - qy) * t + qy;
                polar(nx, ny);
                qx = nx, qy = ny;
                acc = 0.0;                        // and look at point i again
            }
        }
    });
    if (rc != LGS_OK) return rc;
    const lgs_scan_host hs{ rr.data(), aa.data(), (int)rr.size(), in->rel, in->min_range, in->max_range };
    return lgs_scan_create(ctx, &hs, out);
}

extern "C" void lgs_scan_destroy(lgs_scan* s)
{
    if (!s) return;
    if (s->d_ranges) scan_buffer_put(s->device, s->d_ranges, 2 * sizeof(double) * (size_t)s->n);
    delete s;
}

namespace lgs {
void wait_foreign_scans(ForeignScans& f)
{
    for (auto& e : f)
        if (e.second && e.second->wait() == 2)
            throw Error(LGS_ERR_INTERNAL, "a scan's device copy was abandoned by the context that made it");
    // enqueued on another context's stream, maybe still pending
    LGS_HIP_CHECK(hipDeviceSynchronize());
    for (auto& e : f) {
        std::lock_guard<std::mutex> g(e.first->dev_mu);
        if (e.first->dev_fence == e.second) e.first->dev_done.store(true, std::memory_order_release);
    }
    f.clear();
}

void abandon_scan_copies(lgs_ctx* ctx, const std::shared_ptr<CopyFence>& fence, const std::vector<lgs_scan*>& scans)
{
    for (lgs_scan* s : scans) {
        std::lock_guard<std::mutex> g(s->dev_mu);
        if (s->dev_fence != fence || !s->d_ranges) continue;
        scan_buffer_put(ctx->device, s->d_ranges, 2 * sizeof(double) * (size_t)s->n);
        s->d_ranges = s->d_angles = nullptr;
        s->dev_ctx = nullptr;
        s->dev_fence.reset();
    }
    fence->set(2);
}

void scans_to_device(lgs_ctx* ctx, const lgs_scan* const* scans, int n, Upload* up)
{
    // scans without a copy yet (each once), and copies made by other contexts
    std::vector<lgs_scan*> todo;
    ForeignScans foreign;
    for (int j = 0; j < n; ++j) {
        lgs_scan* s = const_cast<lgs_scan*>(scans[j]);
        if (!s || s->dev_done.load(std::memory_order_acquire)) continue;
        std::lock_guard<std::mutex> g(s->dev_mu);
        if (!s->d_ranges) {
            if (std::find(todo.begin(), todo.end(), s) == todo.end()) todo.push_back(s);
        } else if (s->dev_ctx != ctx) {
            foreign.emplace_back(s, s->dev_fence);
        }
    }
    size_t total = 0;
    for (lgs_scan* s : todo) total += 2 * sizeof(double) * (size_t)s->n;
    std::vector<FetchSeg> segs;
    std::vector<lgs_scan*> mine;
    auto fence = std::make_shared<CopyFence>();
    const int b = ctx->bank;
    if (!todo.empty()) {
        if (ctx->scan_ev_live[b]) {   // the staging's previous copies are done
            LGS_HIP_CHECK(hipEventSynchronize(ctx->scan_ev[b]));
            ctx->scan_ev_live[b] = false;
        }
        char* pin = (char*)grow_pinned(ctx->stream, ctx->pinned_scan[b], ctx->pinned_scan_bytes[b], total, true);
        size_t off = 0;
        for (lgs_scan* s : todo) {
            std::lock_guard<std::mutex> g(s->dev_mu);
            if (s->d_ranges) {   // another thread got there first
                if (s->dev_ctx != ctx) foreign.emplace_back(s, s->dev_fence);
                continue;
            }
            const size_t bytes = sizeof(double) * (size_t)s->n;
            double* d = (double*)scan_buffer_get(ctx->device, 2 * bytes);
            std::memcpy(pin + off, s->h_ranges.data(), bytes);
            std::memcpy(pin + off + bytes, s->h_angles.data(), bytes);
            try {
                segs.push_back(fetch_seg(d, pin + off, 2 * bytes));
            } catch (...) {
                scan_buffer_put(ctx->device, d, 2 * bytes);
                throw;
            }
            off += 2 * bytes;
            s->d_angles = d + s->n;
            s->dev_ctx = ctx;
            s->dev_fence = fence;   // published now; other contexts wait for the fence
            s->d_ranges = d;
            mine.push_back(s);
        }
    }
    if (up) {
        // copied with the call's upload (one launch); the upload is flushed
        // before any kernel of the call reads the scans, and sets the fence
        up->extra.insert(up->extra.end(), segs.begin(), segs.end());
        if (!mine.empty()) {
            up->fence = fence;
            up->fence_scans = mine;
        }
        up->foreign.insert(up->foreign.end(), foreign.begin(), foreign.end());
        return;
    }
    if (!mine.empty()) {
        try {
            fetch_list(ctx, segs);
        } catch (...) {
            abandon_scan_copies(ctx, fence, mine);
            throw;
        }
        if (!ctx->scan_ev[b]) LGS_HIP_CHECK(hipEventCreateWithFlags(&ctx->scan_ev[b], hipEventDisableTiming));
        LGS_HIP_CHECK(hipEventRecord(ctx->scan_ev[b], ctx->stream));
        ctx->scan_ev_live[b] = true;
        fence->set(1);
    }
    if (!foreign.empty()) wait_foreign_scans(foreign);
}

// Beams with range < ScanRangeMax in beam order (ComputeScanIndices filter,
// C/mapping/scan_matcher_real_time_correlative.cpp:189-193).  Cached per
// ScanRangeMax; the upload happens once per (scan, matcher).
const int* scan_valid_indices(lgs_ctx* ctx, lgs_scan* s, double rmax, int* nv)
{
    std::lock_guard<std::mutex> g(s->cache_mu);   // two contexts may match this scan at once
    uint64_t key;
    std::memcpy(&key, &rmax, sizeof(key));
    if (std::isnan(rmax)) key = 0x7ff8000000000000ull;
    auto it = s->vidx_by_rmax.find(key);
    if (it == s->vidx_by_rmax.end()) {
        std::vector<int> v;
        for (int i = 0; i < s->n; ++i)
            if (!(s->h_ranges[i] >= rmax)) v.push_back(i);
        it = s->vidx_by_rmax.emplace(key, std::move(v)).first;
    }
    (void)ctx;
    *nv = (int)it->second.size();   // the device compacts the same beams itself (k_project)
    return it->second.data();
}

namespace {
// Host worker pool behind host_parallel_for: workers sleep on a condition
// variable between regions (a region costs a wake-up, not thread creation).
class HostPool {
public:
    static HostPool* get()
    {
        static std::once_flag once;
        std::call_once(once, [] { pthread_atfork(nullptr, nullptr, [] { pool = nullptr; }); });
        std::lock_guard<std::mutex> lk(create_mu);
        if (!pool) pool = new HostPool();  // never destroyed: workers live for the process
        return pool;
    }
    int size() const { return nworkers + 1; }
    // false (nothing run) if another region holds the pool: the caller runs inline
    bool run(int n, int nt, const std::function<void(int)>& f)
    {
        std::unique_lock<std::mutex> call(call_mu, std::try_to_lock);
        if (!call.owns_lock()) return false;
        const int helpers = std::min(nt - 1, nworkers);
        {
            std::lock_guard<std::mutex> lk(mu);
            fn = &f;
            count = n;
            next.store(0);
            slots = helpers;
            busy = helpers;
            ++gen;
        }
        if (helpers > 0) cv.notify_all();
        work();
        std::unique_lock<std::mutex> lk(mu);
        done.wait(lk, [&] { return busy == 0; });
        return true;
    }
    static inline thread_local bool inside = false;  // running a region's f (nested calls go inline)

private:
    HostPool()
    {
        const int hw = std::max(1, (int)std::thread::hardware_concurrency());
        nworkers = std::min(15, hw - 1);
        for (int i = 0; i < nworkers; ++i) std::thread([this] { loop(); }).detach();
    }
    void work()
    {
        inside = true;
        for (int i; (i = next.fetch_add(1)) < count;) (*fn)(i);
        inside = false;
    }
    void loop()
    {
        unsigned long long seen = 0;
        std::unique_lock<std::mutex> lk(mu);
        for (;;) {
            cv.wait(lk, [&] { return gen != seen; });
            seen = gen;
            if (slots == 0) continue;
            --slots;
            lk.unlock();
            work();
            lk.lock();
            if (--busy == 0) done.notify_all();
        }
    }
    static inline HostPool* pool = nullptr;
    static inline std::mutex create_mu;
    std::mutex call_mu, mu;
    std::condition_variable cv, done;
    const std::function<void(int)>* fn = nullptr;
    int count = 0, nworkers = 0, slots = 0, busy = 0;
    std::atomic<int> next{0};
    unsigned long long gen = 0;
};
}  // namespace

void host_parallel_for(int n, int grain, const std::function<void(int)>& f)
{
    HostPool* p = (n > 1) ? HostPool::get() : nullptr;
    const int nt = p ? std::min(p->size(), (n + std::max(1, grain) - 1) / std::max(1, grain)) : 1;
    if (nt <= 1 || HostPool::inside || !p->run(n, nt, f))
        for (int i = 0; i < n; ++i) f(i);
}
}  // namespace lgs
