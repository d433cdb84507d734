// lgs_internal.hpp -- internal types of the MI355X hot-path library (not part of the ABI).
//
// Device layout (DESIGN.md §Data layout):
//   grid      dense fp64, row-major, cell (x,y) at y*w + x, 0.0 = unknown/unallocated
//   scan      ranges[n], angles[n] fp64 (SoA, as ScanData<double>)
//   indices   int2 idx[T][Nv] projected hit cells per search angle (ComputeScanIndices)
//   scores    coarse fp64 cscore[T*ncx*ncy] in reference block order (t, xc, yc)
#pragma once

#include <hip/hip_runtime.h>

#include <climits>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <functional>
#include <stdexcept>
#include <string>
#include <memory>
#include <map>
#include <mutex>
#include <atomic>
#include <condition_variable>
#include <utility>
#include <vector>

#include "lgs_hip.h"

namespace lgs {

struct Error : std::runtime_error {
    int code;
    Error(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

#define LGS_HIP_CHECK(expr)                                                              \
    do {                                                                                 \
        hipError_t e_ = (expr);                                                          \
        if (e_ != hipSuccess)                                                            \
            throw ::lgs::Error(LGS_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

#define LGS_REQUIRE(cond, msg)                                                           \
    do {                                                                                 \
        if (!(cond))                                                                     \
            throw ::lgs::Error(LGS_ERR_INVALID_ARG, msg);                                \
    } while (0)

// Scratch slots of the per-context device arena.
enum Slot {
    S_IDX = 0,      // int2 [T*Nv]
    S_CSCORE,       // double [K]
    S_CFLAG,        // uint8 [K]
    S_SEL,          // uint8 [K]
    S_LIST,         // int [K]
    S_FVAL,         // double [K]
    S_FPOS,         // int [K]
    S_PART_C,       // double [parts]
    S_PART_K,       // int64 [parts]
    S_CUB_TEMP,     // hipcub temp
    S_COUNT,        // int [4]
    S_RECORDS,      // RtcsmRecord [batch]
    S_POSES7,       // double [7*3]
    S_COST_IDX,     // int4 [7*N]
    S_COST_TERM,    // double [7*N]
    S_PATCH,        // int4 [patches]
    S_INGEST,       // lgs_grid_upload_patches: slot table + staged raw patch cells
    S_DENSE_FINE,   // double (dense diagnostics)
    S_COARSE_GRID,  // double (coarse map for OptimizePose(query))
    S_DECIM,        // double (phase-plane coarse map)
    S_CINFO,        // int4 [T*Nv] phase-plane addressing per (angle, beam)
    S_TEDGE,        // int [items][T]: generation-stamped 'angle touches the low map edge' flags; holds
                    // nothing else, so stamps never need clearing (zeroed once when allocated)
    S_RAY0, S_RAY1, S_RAY2, S_RAY3, S_RAY4, S_RAY5, S_RAY6, S_RAY7,
    S_RAY8,         // device hit points / ray cells of a map rebuild (k_raycast.hip construct_maps_device)
    S_LS0, S_LS1,
    S_LIN0, S_LIN1,   // K4 staging
    S_LIN2,           // K4 split refine: flags, timeout word, double-buffered per-beam terms
    S_LIN3,           // K4 split refine: phase stamps (LGS_LS_TRACE diagnostics)
    S_SUPER,        // double: superblock planes (forward kSB x kSB max of S_DECIM)
    S_SBOUND,       // double [T * nsb2] superblock bounds
    S_UPLOAD,       // per-batch descriptors (MatchItem, PlaneJob, PrecompJob), one H2D copy
    S_BATCH_WS,     // per-item match workspaces of a batch (k_rtcsm.hip ItemLayout)
    S_NEGFLAG,      // int per coarse-map set: negative-cell stamp of its planes
    S_BB0, S_BB1, S_BB2, S_BB3, S_BB4, S_BB5,   // branch-and-bound (k_bb.hip)
    S_PRECOMP_TMP,  // double [W*H]: pass-1 result of the large-window precompute
    S_KEEP,         // int: kept-superblock work list of a batch (k_keep / k_coarse_list)
    S_COLL,         // lgs_loop_records_allgather: send block + gathered rows (lgs_coll.hip)
    S_ZTILE,        // unsigned: zero-tile words of the per-map passes (k_rtcsm.hip ZeroTiles), per set
    // bank 1 of the per-batch buffers: a batched call keeps two 64-query
    // chunks in flight (the next chunk's launches go out before the host
    // finishes the previous one), each in its own bank (lgs_ctx::banked)
    S_BATCH_WS_B, S_RECORDS_B, S_UPLOAD_B, S_DECIM_B, S_SUPER_B, S_NEGFLAG_B, S_TEDGE_B, S_ZTILE_B,
    S_NUM_SLOTS
};

constexpr int kGuardInline = 64;
constexpr int kTedgeCtrs = 64;   // k_match_small's per-item wrap-around counters (one per batch item)

struct GuardRec { int t, v, ix, iy; };        // projection near a cell boundary
struct CostGuardRec { int pose_which, beam, ix, iy; };

// Device-written per-scan result record (copied to host once per batch).
// The guard counters are generation-tagged (gen << 32 | count), so the record
// needs no memset before a match: a word carrying another generation counts
// as zero (tagged_slot / tagged_count).
struct RtcsmRecord {
    int status;           // bit0: dangerous unsafe block -> dense rerun
    int found;
    unsigned long long guard_word;
    unsigned long long cost_guard_word;
    long long n_eval;     // coarse blocks refined on the fine map
    int best[3];
    int pad0;
    double score_max;
    double L;             // lower bound used for pruning
    double costs[7];
    unsigned long long coarse_evals;   // blocks k_coarse evaluated (superblock pruning)
    GuardRec guard[kGuardInline];
    CostGuardRec cost_guard[kGuardInline];
};

enum RecordStatus { REC_DANGEROUS = 1 };

// Host-side search plan: everything the reference computes on the host before
// the loops, evaluated with glibc (bit-exact), then shipped to kernels by value.
struct RtcsmPlan {
    double sx, sy, st;          // sensor pose (Compound(initialPose, relPose))
    double step_x, step_y, step_t;
    double min_x, min_y, res;   // grid geometry
    double thr;                 // normalizedScoreThreshold * NumOfScans()
    int W, H;
    int win_x, win_y, win_t;
    int T, ncx, ncy, P;         // angles, coarse grid per angle, P = ncx*ncy
    int low_res;
    int Nv;                     // beams with range < ScanRangeMax
    int N;                      // all beams
    double rmax;                // ScanRangeMax (the compaction filter, :192-193)
    // padded phase-plane coarse layout: lr*lr planes of
    // (Hq + 2M) x (Wq + 2M) doubles, interior = D[ry][rx][qy][qx], margins
    // (M = max(ncx, ncy)) all zero
    int Wq, Hq, M, Wqp, Hqp;
    long long pstride;
    long long K;                // T * P coarse blocks
    // superblocks (kSB x kSB coarse blocks of one angle)
    int nsbx, nsby;
    double sb_mult;             // 1 + 4 (Nv + 1) 2^-53: rounding slack of the bound
    // superblock planes, compact: every phase plane split into 4 x 4
    // sub-phases (padded x mod 4, y mod 4) of Wq4 x Hq4 values, so the
    // superblocks of one beam are consecutive doubles
    int Wq4, Hq4;
    long long sub4, pstride4;
    long long sb_off;           // superblock base offsets start at cbase + sb_off
    // octet layout (windows of at most 5 x 5 superblocks):
    // each sub-phase array is stored as 16-byte units (q, X) holding its rows
    // 4q .. 4q + 7 at column X (every row twice), so a beam's 5 window rows at
    // one column are one aligned 16-byte load; superblock bases are then
    // (unit << 2) | (first row & 3).  Windows of 6-9 superblock rows use
    // 24-byte units (rows 4q .. 4q + 11, every row three times): a beam's 9
    // rows at one column are then one contiguous 24-byte read (unit8 = 3,
    // else 2: the unit's size in 8-byte words)
    int oct, Qo, unit8;
    long long subO, pstrideO;   // units per sub-phase array / per plane
};

// Padded phase-plane geometry handed to the precompute kernel.
struct PlaneGeom {
    int M, Wqp;
    long long pstride;
};

// One coarse-map precompute of a batched launch (k_precompute_jobs).
struct PrecompJob {
    const double* in;
    double* out;
    int W, H;
    PlaneGeom pg;   // pg.Wqp > 0: write the padded phase planes
    // k_precompute_planes also writes every plane value rounded up to fp16
    // (same layout, 2 B per cell; null: not) and stamps *negflag with pgen
    // when a value is negative: what k_super_planes reads
    unsigned short* out16;
    int* negflag;
    int pgen;
    // zero-tile words of this set (k_precompute_planes<L, 16> only; null: none):
    // word (by * gridDim.x + bx) is 1 when the tile's last build read an all-zero
    // footprint, i.e. its plane and fp16 outputs hold +0 -- a tile whose
    // footprint is still all zero then leaves them as they are (k_rtcsm.hip
    // ZeroTiles keeps the words valid per bank, set and layout)
    unsigned* zt;
};

// fp16 (bit pattern) of m rounded toward +inf; zeros as +0 (so nonnegative
// values order like their bit patterns) and NaN as +0 (a max skips it)
__device__ __forceinline__ unsigned short half_round_up_bits_cvt(double m)
{
    // nearest float, then nearest half: one of the two fp16 neighbours of m
    // (double rounding never skips past one), so a one-ulp step away from the
    // lower neighbour gives the round-up
    const _Float16 h = (_Float16)(float)m;
    unsigned short b = __builtin_bit_cast(unsigned short, h);
    if ((double)(float)h < m) b = (m > 0.0) ? (unsigned short)(b + 1) : (unsigned short)(b - 1);
    if (m == 0.0 || m != m) b = 0;
    return b;
}
// The same from the fp64 bit fields (32-bit integer operations only) for the
// fp16 normal range and above; zeros, fp16 subnormals, negatives and NaN take
// the conversion path
__device__ __forceinline__ unsigned short half_round_up_bits(double m)
{
    const unsigned long long b = __builtin_bit_cast(unsigned long long, m);
    const unsigned hi = (unsigned)(b >> 32), lo = (unsigned)b;
    const unsigned e = (hi >> 20) & 0x7FFu;   // biased exponent (sign 0 below)
    if ((hi >> 31) == 0u && e >= 1009u && e < 2047u) {
        if (e > 1038u) return 0x7C00u;         // above the fp16 range: +inf
        unsigned h = ((e - 1008u) << 10) | ((hi >> 10) & 0x3FFu);
        h += ((hi & 0x3FFu) | lo) != 0u;       // dropped bits: round up (a carry steps the exponent)
        return (unsigned short)h;
    }
    return half_round_up_bits_cvt(m);
}

struct CostPlan {
    double min_range, max_range;   // filter (open interval)
    double hit_and_missed_dist, occupancy_threshold;
    double variance, scaling_factor;
    double min_x, min_y, res;
    int W, H, kernel_size, N;
};

}  // namespace lgs

// Phase probes (diagnostics build only, make probe): block 0 / thread 0
// stamps the 100 MHz wall clock at phase boundaries and prints the deltas.
#ifdef LGS_PROBE
#define LGS_PROBE_DECL unsigned long long lgs_probe_t[16]; int lgs_probe_n = 0
#define LGS_PROBE_MARK() do { if (threadIdx.x == 0) lgs_probe_t[lgs_probe_n < 16 ? lgs_probe_n++ : 15] = wall_clock64(); } while (0)
#define LGS_PROBE_PRINT(name) do { if (threadIdx.x == 0 && blockIdx.x == 0 && blockIdx.y == 0) { \
    printf("probe %s:", name); for (int i_ = 1; i_ < lgs_probe_n; ++i_) printf(" %.2f", 0.01 * (double)(lgs_probe_t[i_] - lgs_probe_t[i_ - 1])); \
    printf(" us\n"); } } while (0)
#else
#define LGS_PROBE_DECL do { } while (0)
#define LGS_PROBE_MARK() do { } while (0)
#define LGS_PROBE_PRINT(name) do { } while (0)
#endif

namespace lgs {
enum KernelId { K_PROJECT = 0, K_COARSE, K_SEED, K_SELECT, K_FINE, K_REPLAY, K_COST, K_PRECOMPUTE,
                K_LINSOLVE, K_RAY_EMIT, K_RAY_APPLY, K_SUPER, K_SUPER_PLANES, K_BB_SCORE, K_BB_EXPAND,
                K_COARSE_AUX,   // k_keep + k_unsafe_list: the work-list passes around k_coarse_list
                K_MATCH_SMALL,  // k_match_small: a small window's whole search (one coarse block per angle)
                K_NUM_KERNELS };
extern const char* const kKernelNames[K_NUM_KERNELS];
struct PendingTiming {
    int kernel;
    hipEvent_t a, b;
    double algo_bytes;
    // pruned k_coarse: algo_bytes is set from the batch's records (blocks
    // actually scored x 8 B x Nv) once their host copy is known
    bool coarse_evals = false;
    long long batch = 0;   // lgs_ctx::timing_batch when launched
    // device-timed launch (LGS_OPT_DEVICE_TIMING): the slot's host copy and tag
    const unsigned long long* hw = nullptr;
    unsigned long long tag = 0;
};

// Device timing of a launch (LGS_OPT_DEVICE_TIMING): kDtsSub sub-slots of two
// words (start, end), each word gen << 40 | 40-bit value, raised by relaxed
// agent-scope atomic maxima (vector atomics).  The start word holds
// kDtsMask - t, so its maximum is the earliest start of this generation;
// older generations' values are smaller, so the words need no reset between
// launches (only zero at allocation).  Atomics on one address serialise at
// the memory side (~50 ns each: one pair per workgroup took a 27k-workgroup
// launch from 10 to 358 us), so only a sample of workgroups stamps: the
// first kDtsSub dispatched (workgroups are dispatched in linear-id order, so
// one of them starts first) stamp the start; the last kDtsSub dispatched and
// every kDtsEvery-th stamp the end (the last workgroup to finish is one of
// the last dispatched when workgroups carry even work).
constexpr int kDtsSub = 8;
constexpr int kDtsEvery = 31;   // odd: a multiple of 8 would sample only blockIdx % 8 == 0 (XCD 0)
constexpr int kDtsSlots = 32;   // device-timed launches per chunk
constexpr unsigned long long kDtsMask = (1ull << 40) - 1ull;
struct DevTs {
    unsigned long long* w;   // this launch's 2 x kDtsSub words (null: not device-timed)
    unsigned long long tag;  // gen << 40
};
__device__ __forceinline__ void dts_begin(const DevTs& d)
{
    if (d.w && threadIdx.x == 0 && threadIdx.y == 0) {
        const unsigned b = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
        if (b < (unsigned)kDtsSub) {
            const unsigned long long t = __builtin_amdgcn_s_memrealtime() & kDtsMask;
            __hip_atomic_fetch_max(d.w + 2 * b, d.tag | (kDtsMask - t), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}
__device__ __forceinline__ void dts_end(const DevTs& d)
{
    if (d.w && threadIdx.x == 0 && threadIdx.y == 0) {
        const unsigned b = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
        const unsigned nwg = gridDim.x * gridDim.y * gridDim.z;
        if (b + (unsigned)kDtsSub >= nwg || b % (unsigned)kDtsEvery == 0u) {
            const unsigned long long t = __builtin_amdgcn_s_memrealtime() & kDtsMask;
            const unsigned sub = (b + b / (unsigned)kDtsEvery) & (unsigned)(kDtsSub - 1);
            __hip_atomic_fetch_max(d.w + 2 * sub + 1, d.tag | t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}
// start stamp at construction (the kernel's first statement), end stamp at
// every exit of thread 0
struct DtsScope {
    const DevTs d;
    __device__ explicit DtsScope(const DevTs& x) : d(x) { dts_begin(d); }
    __device__ ~DtsScope() { dts_end(d); }
};
}  // namespace lgs

struct lgs_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    std::string last_error;
    // options
    double guard_eps = 1e-9;
    bool force_dense = false;
    bool inject_index = false;
    int guard_cap = lgs::kGuardInline;
    bool super_prune = true;     // superblock pruning of k_coarse (LGS_OPT_SUPER_PRUNE)
    bool linsolve_split = true;  // lone refine over one workgroup per 64 beams (LGS_OPT_LINSOLVE_SPLIT)
    long long handoff_spin_us = 200000;   // split refine spin bound (LGS_OPT_HANDOFF_SPIN_US; 0 = force the fallback)
#ifndef LGS_FINE_STAGED_DEFAULT
#define LGS_FINE_STAGED_DEFAULT 1
#endif
    bool fine_staged = LGS_FINE_STAGED_DEFAULT;   // batched LowRes-5 fine evaluator: LDS-staged windows (LGS_OPT_FINE_STAGED)
    long long coop_tiles = -1;   // one-launch sort: tile limit for this ctx (LGS_OPT_COOP_TILES; -1 = device capacity)
    long long sort_barrier_us = 50000;   // one-launch sort: barrier wait bound (LGS_OPT_SORT_BARRIER_US)
    long long handoff_fallbacks = 0;      // split refines rerun on one workgroup after a time-out
    bool peer_staged = false;    // cross-context copies through host memory (LGS_OPT_PEER_COPY)
    int prune_min_super = 1;     // LGS_OPT_PRUNE_MIN_SUPER
    bool small_window = true;    // one-launch search of one-block windows (LGS_OPT_SMALL_WINDOW)
    bool fused_planes = true;    // superblock units by k_super_hv (LGS_OPT_FUSED_PLANES)
    int seed_wide = 12;
    bool lean_project = true;    // LGS_OPT_LEAN_PROJECT (k_rtcsm.hip lean_rows)
    bool zero_tiles = true;   // LGS_OPT_ZERO_TILES          // batches: candidate superblocks whose best members seed the bound (LGS_OPT_SEED_WIDE; <= 4: one launch)
    bool device_hits = true;     // map rebuilds of many scans: hit points / ray cells on the device (LGS_OPT_DEVICE_HITS)
    bool split_chunks = false;   // calls of 32..64 matches as two chunks (LGS_OPT_SPLIT_CHUNKS; measured r05, 8-rank loop block: 1.007 vs 0.869 ms as one)
    bool hv_full = false;        // k_super_hv stores 16-byte units whole (LGS_OPT_HV_FULL, A/B; measured r05: 0.24 vs 0.17 ms per 64 sets)
    // a batch's stages after the coarse-map builds run on `hi`, a stream of
    // the device's highest priority, behind an event on `stream`: the
    // latency-bound tail of one context's chunk is not queued behind other
    // contexts' plane builds (LGS_OPT_PRIORITY_TAIL)
    bool prio_tail = false;   // measured r05: no gain (60.1k vs 59.6k scans/s), lone p50 +10 us, batch call +0.4 ms
    hipStream_t hi = nullptr;
    hipEvent_t split_ev[2] = {};
    bool post_records = true;    // records written to pinned memory by k_post + a flag (LGS_OPT_POST_RECORDS)
    long long copies_direct = 0, copies_staged = 0;   // lgs_debug_copy_counters
    int lanes_min_batch = 2;     // pruned coarse stage: the work list (k_coarse_list) from this batch size on (LGS_OPT_LANES_MIN_BATCH)
    long long ray_chunk_keys = 1LL << 28;  // ray-cast keys per emit/sort/apply pass (LGS_OPT_RAY_CHUNK_KEYS)
    // Stamps come from one process-wide counter: a context's scratch may be
    // memory a destroyed context used, and its stale tags must never match.
    int next_stamp();
    // LGS_OPT_SKIP_MASK (diagnostics only): launches of these kernels are
    // skipped, leaving stale scratch -- results are meaningless; used to
    // measure each stage's share of device throughput
    unsigned skip_mask = 0;
    bool skipped(int kernel) const { return (skip_mask >> kernel) & 1u; }
    // LGS_OPT_POISON_WS (diagnostics): 0xFF-fill match workspaces before a batch
    bool poison_ws = false;
    // intermediates of every item of the last correlative batch (lgs_debug_item_buffer)
    struct DbgItem {
        const void* buf[10];
        size_t bytes[10];
        int gen;
    };
    std::vector<DbgItem> dbg;
    int generation = 0;          // per-enqueue stamp (edge flags need no memset), from next_stamp()
    // arena
    void* buf[lgs::S_NUM_SLOTS] = {};
    size_t buf_bytes[lgs::S_NUM_SLOTS] = {};
    void* pinned = nullptr;
    size_t pinned_bytes = 0;
    void* pinned_up = nullptr;   // staging of the per-batch descriptor upload
    size_t pinned_up_bytes = 0;
    // bank 1 (two chunks in flight): descriptor staging and record copies
    void* pinned_up_b = nullptr;
    size_t pinned_up_b_bytes = 0;
    // a copy out of bank b's descriptor staging may still be reading it
    // (set by Upload::copy, cleared by sync() and when the bank's chunk is
    // known complete); the next Upload::copy into that staging waits first
    bool up_busy[2] = { false, false };
    void* pinned_rec[2] = {};
    size_t pinned_rec_bytes[2] = {};
    int bank = 0;                // which bank the per-batch buffers come from
    size_t tedge_zeroed[2] = {}; // bytes of the S_TEDGE allocation already zeroed, per bank
                                 // (a reallocation always grows the slot)
    int* tedge_buffer(size_t n); // n flags, zeroed at allocation only
    // the kTedgeCtrs counters in front of the same allocation (sized for n flags)
    int* small_counters(size_t n);
    int banked(int slot) const
    {
        if (!bank) return slot;
        switch (slot) {
        case lgs::S_BATCH_WS: return lgs::S_BATCH_WS_B;
        case lgs::S_RECORDS: return lgs::S_RECORDS_B;
        case lgs::S_UPLOAD: return lgs::S_UPLOAD_B;
        case lgs::S_DECIM: return lgs::S_DECIM_B;
        case lgs::S_SUPER: return lgs::S_SUPER_B;
        case lgs::S_NEGFLAG: return lgs::S_NEGFLAG_B;
        case lgs::S_TEDGE: return lgs::S_TEDGE_B;
        case lgs::S_ZTILE: return lgs::S_ZTILE_B;
        default: return slot;
        }
    }
    void* ensure_pinned_rec(size_t bytes);   // per bank: a batch's record copies
    // staging of scans' first device copies (lgs::scans_to_device), per bank;
    // scan_ev[bank] marks the end of the copies out of it
    void* pinned_scan[2] = {};
    size_t pinned_scan_bytes[2] = {};
    hipEvent_t scan_ev[2] = {};
    bool scan_ev_live[2] = {};
    void* pinned_in = nullptr;   // staging of lgs_grid_upload_patches
    size_t pinned_in_bytes = 0;
    // padded phase-plane buffer (per bank): margins zeroed once per (buffer, layout, set count)
    void* planes_ptr[2] = {};
    int planes_sets[2] = {};
    void* super_ptr[2] = {};   // superblock planes zeroed with them
    int super_sets[2] = {};
    long long planes_key[2][4] = { { -1, -1, -1, -1 }, { -1, -1, -1, -1 } };
    // zero-tile words of the per-map passes (k_rtcsm.hip ZeroTiles), per bank:
    // the layout they were kept for and which sets' words are current
    long long zt_key[2][12] = {};
    std::vector<unsigned char> zt_pre[2], zt_hv[2];
    std::vector<long long> zt_dims[2];   // per set: W << 32 | H of the map its precompute words describe
    double* zero = nullptr;      // 32 zero doubles: target of out-of-map gathers
    // profiling (LGS_OPT_PROFILE)
    bool profile = false;
    unsigned profile_mask = ~0u;  // kernels (KernelId bits) timed while profile is on
    std::vector<lgs::PendingTiming> pending;
    std::vector<hipEvent_t> event_pool;
    int64_t stat_launches[lgs::K_NUM_KERNELS] = {};
    double stat_ms[lgs::K_NUM_KERNELS] = {};
    double stat_bytes[lgs::K_NUM_KERNELS] = {};
    double stat_disp_ms[lgs::K_NUM_KERNELS] = {};   // device timing: from the previous launch's end (lgs_kernel_stat)
    // correlative matches since the last lgs_ctx_reset_stats (lgs_ctx_match_counters)
    int64_t count_matches = 0, count_coarse_blocks = 0, count_coarse_blocks_dense = 0, count_pruned = 0;

    // profiling helpers: begin() before a launch, end() after it, harvest()
    // after a stream synchronisation.
    int timing_begin(int kernel, double algo_bytes);
    void timing_end(int token);
    // LGS_OPT_DEVICE_TIMING: per-bank device words of a chunk's launches (zeroed
    // at allocation), the chunk's region while its chain is enqueued (null
    // otherwise: event timing), its host copy (written by k_post) and slots used
    bool dev_timing = false;
    unsigned long long* dts_buf[2] = {};
    unsigned long long* dts_dev = nullptr;
    const unsigned long long* dts_host = nullptr;
    int dts_used = 0;
    unsigned dts_gen = 0;   // 24-bit generations, per context (monotonic per bank region)
    // the launch's device-timing words for a timing token (DevTs{} = none)
    lgs::DevTs dts(int token) const
    {
        if (token < 0 || !pending[(size_t)token].hw) return lgs::DevTs{ nullptr, 0ull };
        const size_t slot = (size_t)(pending[(size_t)token].hw - dts_host) / (2 * lgs::kDtsSub);
        return lgs::DevTs{ dts_dev + slot * 2 * lgs::kDtsSub, pending[(size_t)token].tag };
    }
    void harvest();
    // timings of the launches tagged with batch <= b only (the next chunk's
    // may still be running)
    void harvest_upto(long long b);
    long long timing_batch = 0;
    hipEvent_t bank_ev[2] = {};   // end of each bank's chunk (its record copy)
    void wait_event(hipEvent_t ev);   // spin or block, as sync()

    // wait for the stream: spin on hipStreamQuery (default; the host thread
    // wakes within ~1 us instead of the blocking wait's interrupt latency) or
    // hipStreamSynchronize (LGS_OPT_SPIN_SYNC 0)
    bool spin_sync = true;
    void sync();

    void* ensure(int slot, size_t bytes);
    // grow-only auxiliary device buffers indexed by number (per-level
    // branch-and-bound lists; freed in release())
    std::vector<void*> aux;
    std::vector<size_t> aux_bytes;
    void* ensure_aux(int i, size_t bytes);
    void* ensure_pinned(size_t bytes);
    void* ensure_pinned_up(size_t bytes);
    void* ensure_pinned_in(size_t bytes);
    void release();
};

namespace lgs {
// Device work still writing a map's cells when its call returned (the latest
// map's asynchronous incremental rebuild, k_raycast.hip): a one-thread kernel
// after the work stores the writer's generation into a coherent pinned word
// (r05: an event recorded on the stream instead cost the next kernel a ~5 us
// gap on the config-4 step's chain).  The host waits by spinning on the word;
// a reader on another stream gets an event recorded on the writer's stream
// only when it needs one (grid_acquire: everything queued there so far, so
// the writer's work included).
struct WriterEvent {
    hipEvent_t ev = nullptr;      // created and recorded lazily, under mu
    // (st, gen) are set together under mu by the owner's record_writer;
    // readers in other contexts (grid_acquire, clone_grid) load them without
    // the lock, so both are atomics: a reader sees either pair member of a
    // newer writer, which only makes it wait for more work, never less
    std::atomic<hipStream_t> st{ nullptr };
    unsigned* flag = nullptr;     // coherent pinned word (k_raycast.hip record_writer)
    std::atomic<unsigned> gen{ 0 };   // the pending writer's generation
    std::mutex mu;
    WriterEvent() = default;
    WriterEvent(const WriterEvent&) = delete;
    WriterEvent& operator=(const WriterEvent&) = delete;
    ~WriterEvent()
    {
        if (ev) hipEventDestroy(ev);
        if (flag) hipHostFree(flag);
    }
    bool done() const { return __atomic_load_n(flag, __ATOMIC_ACQUIRE) == gen.load(std::memory_order_acquire); }
    // the host waits for the writer's work; a stream that went idle without
    // the word (a fault, a lost store) is an error
    void wait()
    {
        for (unsigned spins = 1; !done(); ++spins) {
            if (spins % 4096) continue;
            const hipError_t e = hipStreamQuery(st.load(std::memory_order_acquire));
            if (e == hipSuccess && !done()) throw Error(LGS_ERR_INTERNAL, "map writer: completion word lost");
            if (e != hipSuccess && e != hipErrorNotReady) LGS_HIP_CHECK(e);
        }
    }
    // reader's stream after the writer's work (a device-side wait)
    void order_after(hipStream_t reader)
    {
        std::lock_guard<std::mutex> lk(mu);
        if (done()) return;
        if (!ev) LGS_HIP_CHECK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        LGS_HIP_CHECK(hipEventRecord(ev, st.load(std::memory_order_acquire)));
        LGS_HIP_CHECK(hipStreamWaitEvent(reader, ev, 0));
    }
};
}  // namespace lgs

struct lgs_grid {
    lgs_ctx* ctx = nullptr;   // creating context (not used after its destruction)
    int device = 0;
    double* d = nullptr;
    int w = 0, h = 0;
    double min_x = 0, min_y = 0, res = 0;
    bool owned = false;       // device cells freed by lgs_grid_destroy
    bool map_view = false;    // handle embedded in an lgs_map: destroy is a no-op
    std::shared_ptr<lgs::WriterEvent> writer;   // pending writer of the cells (null: none)
};

namespace lgs {
// A scan's first device copy, as other contexts see it: 0 published but not
// yet enqueued (the copy rides on its call's upload, flushed later in that
// call), 1 enqueued on the copying context's stream, 2 abandoned (the flush
// failed; the scan was unpublished).  A context that finds a scan copied by
// another waits for 1 -- after enqueueing its own copies, so two calls that
// first touch each other's scans cannot wait for each other -- and then for
// the device.
struct CopyFence {
    std::mutex mu;
    std::condition_variable cv;
    int state = 0;
    void set(int s)
    {
        {
            std::lock_guard<std::mutex> g(mu);
            state = s;
        }
        cv.notify_all();
    }
    int wait()
    {
        std::unique_lock<std::mutex> g(mu);
        cv.wait(g, [&] { return state != 0; });
        return state;
    }
};
}  // namespace lgs

// Loads from global memory through a generic pointer (a descriptor field)
// compile to flat_load, which also counts against lgkmcnt: every LDS wait of
// the kernel then waits for the gathers in flight too.  gload issues them as
// global_load (address space 1); every target passed to it is device memory.
#ifndef LGS_GLOBAL_GATHER
#define LGS_GLOBAL_GATHER 1
#endif
#ifdef __HIP_DEVICE_COMPILE__
template <class T>
__device__ __forceinline__ T gload(const T* p)
{
#if LGS_GLOBAL_GATHER
    return *(const __attribute__((address_space(1))) T*)p;
#else
    return *p;
#endif
}
template <class T>
__device__ __forceinline__ void gstore(T* p, T v)
{
#if LGS_GLOBAL_GATHER
    *(__attribute__((address_space(1))) T*)p = v;
#else
    *p = v;
#endif
}
#else
template <class T>
__device__ __forceinline__ T gload(const T* p)
{
    return *p;
}
template <class T>
__device__ __forceinline__ void gstore(T* p, T v)
{
    *p = v;
}
#endif

struct lgs_scan {
    lgs_ctx* ctx = nullptr;   // creating context (not used after its destruction)
    int device = 0;
    unsigned long long uid = 0;   // process-unique id (the latest map's window identity, §4.4b)
    // device copy (ranges then angles, one pooled buffer): made by the first
    // call that reads it, on that call's stream (lgs::scans_to_device); null
    // until then -- a frontend's raw scans, only ever interpolated on the
    // host, never get one
    double* d_ranges = nullptr;
    double* d_angles = nullptr;
    std::mutex dev_mu;
    const lgs_ctx* dev_ctx = nullptr;   // whose stream the copy went on
    std::shared_ptr<lgs::CopyFence> dev_fence;   // when the copy is enqueued
    std::atomic<bool> dev_done{ false };  // the copy is known to be complete
    int n = 0;
    lgs_pose2d rel{0, 0, 0};
    double min_range = 0, max_range = 0;
    double max_elem = 0;                 // *std::max_element(ranges)
    std::vector<double> h_ranges, h_angles;
    // compaction cache: beams with range < scan_range_max, in beam order, one
    // list per distinct ScanRangeMax (the frontend's and the loop detector's
    // matchers may alternate on one scan), built once under cache_mu and never
    // modified after: a reader's pointer stays valid for the scan's lifetime
    // and the set of lists is bounded by the matchers' distinct values (host
    // copy for the guard re-projection; the device compacts itself).
    // cache_mu also guards hits_cache.
    mutable std::mutex cache_mu;
    std::map<uint64_t, std::vector<int>> vidx_by_rmax;   // keyed by the bits of ScanRangeMax (any NaN: one key)
    // hit points of the last (robot pose, usable range) they were computed for
    // (k_raycast.hip scan_hits): the frontend inserts a scan at its estimated
    // pose and then rebuilds the latest map from it at that same pose 10 times
    mutable std::shared_ptr<const void> hits_cache;
    mutable double hits_key[5] = { NAN, NAN, NAN, NAN, NAN };
};

extern "C" void sincos(double x, double* s, double* c);  // glibc

namespace lgs {

// The reference is built with GCC, which fuses sin(x) and cos(x) of the same
// argument into one glibc sincos() call; glibc's sincos differs from separate
// sin/cos in ~0.1% of inputs.  Every host recomputation that must be
// bit-exact therefore calls sincos() explicitly wherever the reference
// evaluates both (HitPoint, Compound, MoveBackward, ...).
inline void ref_sincos(double x, double& s, double& c) { ::sincos(x, &s, &c); }

// Host pose algebra restated from H/pose.hpp (glibc sincos, no contraction).
inline lgs_pose2d compound(lgs_pose2d s, lgs_pose2d d)
{
    double sinT, cosT;
    ref_sincos(s.theta, sinT, cosT);
    return { cosT * d.x - sinT * d.y + s.x, sinT * d.x + cosT * d.y + s.y, s.theta + d.theta };
}
inline lgs_pose2d move_backward(lgs_pose2d e, lgs_pose2d d)
{
    const double theta = e.theta - d.theta;
    double sinT, cosT;
    ref_sincos(theta, sinT, cosT);
    return { e.x - cosT * d.x + sinT * d.y, e.y - sinT * d.x - cosT * d.y, theta };
}
inline lgs_pose2d inverse_compound(lgs_pose2d s, lgs_pose2d e)
{
    double sinT, cosT;
    ref_sincos(s.theta, sinT, cosT);
    const double dx = e.x - s.x, dy = e.y - s.y;
    return { cosT * dx + sinT * dy, -sinT * dx + cosT * dy, e.theta - s.theta };
}

const int* scan_valid_indices(lgs_ctx* ctx, lgs_scan* scan, double scan_range_max, int* nv);
// Device copies of the scans' ranges/angles, ordered before the ctx stream's
// next work: the first use of a scan stages its host copy (pinned, per bank)
// and enqueues the copy on ctx->stream.  Every caller synchronises its
// stream before returning, after which the copy is complete; a scan whose
// copy was enqueued by another context is waited for (device-wide) once.
// With an Upload, the copies join that upload's (one launch when it flushes;
// the staging is reused only after the call's synchronisation).
struct Upload;
void scans_to_device(lgs_ctx* ctx, const lgs_scan* const* scans, int n, Upload* up = nullptr);
// scans whose first copy another context made: wait until it is enqueued
// there, then for the device (lgs_core.hip)
using ForeignScans = std::vector<std::pair<lgs_scan*, std::shared_ptr<CopyFence>>>;
void wait_foreign_scans(ForeignScans& f);
// a first copy that was never enqueued: the scans lose their device copy
void abandon_scan_copies(lgs_ctx* ctx, const std::shared_ptr<CopyFence>& fence, const std::vector<lgs_scan*>& scans);
// Host-to-device copy of pinned staging (the ctx's coherent hipHostMalloc
// buffers) by a kernel on ctx->stream (k_fetch): a small hipMemcpyAsync waits
// ~11 us in the copy engine's queue and takes ~6 us more (r03 trace of the
// config-4 frontend), a kernel reads the staging over the host link in one
// round trip.  dst and src 16-byte aligned.
void fetch_async(lgs_ctx* ctx, void* dst, const void* src, size_t bytes);
// several copies in one launch (k_fetch: one segment per grid row, kFetchSegs
// per launch)
struct FetchSeg {
    const unsigned char* src;   // device-visible address of the pinned staging
    unsigned char* dst;
    unsigned long long bytes;
};
constexpr int kFetchSegs = 8;
struct FetchList {
    FetchSeg s[kFetchSegs];
};
FetchSeg fetch_seg(void* dst, const void* src, size_t bytes);
void fetch_list(lgs_ctx* ctx, const std::vector<FetchSeg>& segs);
// above this, staging goes through hipMemcpyAsync (a kernel reading host
// memory over the link is slower than the copy engine for bulk data)
constexpr size_t kFetchMaxBytes = size_t(1) << 20;
// glibc sincos of x[j], j < n, bit for bit (host_simd.cpp: AVX2 restatement)
void sincos_batch(const double* x, long long n, double* s, double* c);
// floor((xy[j] - (j odd ? my : mx)) / res) for j < n2 (host_simd.cpp)
void cells_of_points(const double* xy, long long n2, double mx, double my, double res, int* out);
inline void scan_to_device(lgs_ctx* ctx, const lgs_scan* s) { scans_to_device(ctx, &s, 1); }

// Order a read of g's cells on ctx's stream after a pending asynchronous write
// from another stream (a device-side wait, no host synchronisation).
inline void grid_acquire(lgs_ctx* ctx, const lgs_grid* g)
{
    if (g && g->writer && g->writer->st.load(std::memory_order_acquire) != ctx->stream)
        g->writer->order_after(ctx->stream);
}

// Host staging of one batch's descriptors: appended to a pinned buffer, then
// one host-to-device copy into the S_UPLOAD slot (flush).  Offsets are
// returned at append time; device addresses are base + offset after flush.
struct Upload {
    lgs_ctx* ctx;
    std::vector<char> host;
    char* dev = nullptr;
    std::vector<FetchSeg> extra;   // other staged copies launched with this one (scans' first copies)
    std::shared_ptr<CopyFence> fence;   // those scans' copy fence (set once enqueued)
    std::vector<lgs_scan*> fence_scans;
    ForeignScans foreign;               // scans another context copied (waited for after our copies)
    explicit Upload(lgs_ctx* c) : ctx(c) {}
    Upload(const Upload&) = delete;
    Upload& operator=(const Upload&) = delete;
    ~Upload()
    {
        // copies joined to an upload that was never flushed (an error path)
        // still run: their scans already point at the destination
        if (!extra.empty()) {
            try {
                fetch_list(ctx, extra);
            } catch (...) {
                if (fence) abandon_scan_copies(ctx, fence, fence_scans);
                fence.reset();
            }
        }
        if (fence) fence->set(1);
    }
    template <class T>
    size_t append(const T* p, size_t n)
    {
        const size_t off = (host.size() + 255) & ~(size_t)255;
        host.resize(off + sizeof(T) * n);
        std::memcpy(host.data() + off, p, sizeof(T) * n);
        return off;
    }
    // prepare(): the device address of the staged bytes (so that staged
    // descriptors can be patched to point into the upload itself), copy():
    // the host-to-device copy; flush() = both.
    char* prepare()
    {
        dev = (char*)ctx->ensure(ctx->banked(S_UPLOAD), std::max<size_t>(host.size(), 16));
        return dev;
    }
    void copy()
    {
        const size_t b = std::max<size_t>(host.size(), 16);
        // the staging is shared by every upload of this bank: an earlier
        // upload's copy still queued on the stream must have read it first
        if (ctx->up_busy[ctx->bank]) ctx->sync();
        char* pin = (char*)ctx->ensure_pinned_up(b);
        std::memcpy(pin, host.data(), host.size());
        std::vector<FetchSeg> segs;
        try {
            if (host.size() <= kFetchMaxBytes)
                segs.push_back(fetch_seg(dev, pin, host.size()));
            else   // bulk (branch-and-bound node lists): the copy engine
                LGS_HIP_CHECK(hipMemcpyAsync(dev, pin, host.size(), hipMemcpyHostToDevice, ctx->stream));
            segs.insert(segs.end(), extra.begin(), extra.end());
            extra.clear();
            fetch_list(ctx, segs);
        } catch (...) {
            // the scans' copies were never (all) enqueued: unpublish them so
            // no other call reads their uninitialised device copies
            extra.clear();
            if (fence) abandon_scan_copies(ctx, fence, fence_scans);
            fence.reset();
            fence_scans.clear();
            ctx->up_busy[ctx->bank] = true;   // a part may have been queued
            throw;
        }
        ctx->up_busy[ctx->bank] = true;
        if (fence) fence->set(1);
        fence.reset();
        fence_scans.clear();
        if (!foreign.empty()) wait_foreign_scans(foreign);
    }
    void flush()
    {
        prepare();
        copy();
    }
    template <class T>
    T* host_at(size_t off) { return (T*)(host.data() + off); }
    template <class T>
    const T* at(size_t off) const { return (const T*)(dev + off); }
};

// C-ABI guard: run f, map exceptions to status codes + ctx->last_error.
template <class F>
int guarded(lgs_ctx* ctx, F&& f)
{
    try {
        f();
        return LGS_OK;
    } catch (const Error& e) {
        if (ctx) ctx->last_error = e.what();
        return e.code;
    } catch (const std::bad_alloc&) {
        if (ctx) ctx->last_error = "out of host memory";
        return LGS_ERR_OOM;
    } catch (const std::exception& e) {
        if (ctx) ctx->last_error = e.what();
        return LGS_ERR_INTERNAL;
    }
}

// f(i) for i in [0, n) on a persistent pool of host threads (at most 16
// including the caller; at most ceil(n / grain) of them).  f must not throw.
// One parallel region runs at a time; nested calls run inline.
void host_parallel_for(int n, int grain, const std::function<void(int)>& f);

// K3 sort (k_sort.hip): stable LSD radix sort of n 32-bit keys on bits
// [lo, lo + bits) into `out`; `tmp` (n keys) is used when the sort takes two
// or more 8-bit passes.  in, tmp and out are distinct device buffers.
// err: device-visible error word, set to 2 if the one-launch sort's grid
// barrier timed out (null: not reported)
void keysort(lgs_ctx* ctx, const unsigned* in, unsigned* out, unsigned* tmp, long long n, int lo, int bits, int* err);

}  // namespace lgs
