/*
 * lgs_hip.h -- C-ABI of the MI355X-native scan-matching + grid-update hot path.
 *
 * This is the drop-in boundary.  Every entry point is plain C:
 * opaque handles, plain pointers and sizes, an int status (LGS_OK == 0), no
 * exceptions and no torch/HIP types in the signatures.  A C++ adapter above this
 * ABI mirrors the reference's plugin interface (my-lidar-graph-slam_amd/host/);
 * INTEGRATION.md shows the reference-side registration.
 *
 * Reference interfaces each entry point replaces (paths relative to the
 * reference root; H/ = include/my_lidar_graph_slam/, C/ = src/my_lidar_graph_slam/):
 *
 *   lgs_grid_precompute_max      PrecomputeGridMap(gridMap, winSize)
 *                                C/mapping/grid_map_builder.cpp:518-536 (via
 *                                ScanMatcherRealTimeCorrelative::ComputeCoarserMap
 *                                C/mapping/scan_matcher_real_time_correlative.cpp:148-153)
 *   lgs_rtcsm_optimize_pose      ScanMatcherRealTimeCorrelative::OptimizePose(
 *                                gridMap, precompMap, scanData, initialPose, thr) const
 *                                C/mapping/scan_matcher_real_time_correlative.cpp:50-145
 *   lgs_rtcsm_optimize_pose_query  ScanMatcherRealTimeCorrelative::OptimizePose(query)
 *                                C/mapping/scan_matcher_real_time_correlative.cpp:31-47
 *                                (the ScanMatcher plugin entry, H/mapping/scan_matcher.hpp:198-199)
 *   lgs_rtcsm_optimize_pose_query_batch  n independent OptimizePose(query) calls
 *                                (C/mapping/scan_matcher_real_time_correlative.cpp:31-47 each)
 *                                as one batched device pipeline
 *   lgs_rtcsm_optimize_pose_batch  LoopDetectorRealTimeCorrelative::Detect's per-node
 *                                loop C/mapping/loop_detector_real_time_correlative.cpp:66-92
 *   lgs_loop_detect_rtcsm        LoopDetectorRealTimeCorrelative::Detect + FindCorrespondingPose
 *                                C/mapping/loop_detector_real_time_correlative.cpp:26-125
 *   lgs_cost_greedy_endpoint     CostGreedyEndpoint::Cost
 *                                C/mapping/cost_function_greedy_endpoint.cpp:32-111
 *   lgs_map_update_scan          GridMapBuilder::UpdateGridMap's insert of one scan
 *                                (bounding box, Expand, per-beam Bresenham + Bayes update)
 *                                C/mapping/grid_map_builder.cpp:149-186
 *   lgs_map_construct_from_scans GridMapBuilder::ConstructMapFromScans
 *                                C/mapping/grid_map_builder.cpp:227-332 (UpdateLatestMap :196-207)
 *   lgs_map_render_gray          MapSaver::DrawMap C/io/map_saver.cpp:276-313
 *   lgs_map_render_gray_region   MapSaver::SaveMapCore's DrawMap of the actual map size
 *                                C/io/map_saver.cpp:413-437
 *   lgs_map_actual_size          GridMap::ComputeActualMapSize H/grid_map/grid_map.hpp:969-1015
 *   lgs_map_download_patches     Patch::IsAllocated H/grid_map/grid_map_patch.hpp:40
 *   lgs_scan_interpolate         ScanInterpolator::Interpolate
 *                                C/mapping/scan_interpolator.cpp:9-98
 *   lgs_maps_construct_from_scans GridMapBuilder::AfterLoopClosure's rebuild of every
 *                                local map C/mapping/grid_map_builder.cpp:62-80
 *   lgs_map_construct_global     GridMapBuilder::ConstructGlobalMap
 *                                C/mapping/grid_map_builder.cpp:83-95
 *   lgs_linsolve_optimize_pose   ScanMatcherLinearSolver::OptimizePose(query)
 *                                C/mapping/scan_matcher_linear_solver.cpp:38-148
 *   lgs_cost_square_error        CostSquareError::Cost / ComputeCovariance
 *                                C/mapping/cost_function_square_error.cpp:21-58, :112-135
 *   lgs_grid_precompute_pyramid  PrecomputeGridMaps C/mapping/grid_map_builder.cpp:471-495
 *   lgs_bb_optimize_pose_batch   ScanMatcherBranchBound::OptimizePose(map, pyramid, scan, pose, thr)
 *                                C/mapping/scan_matcher_branch_bound.cpp:47-154
 *   lgs_bb_optimize_pose_query   ScanMatcherBranchBound::OptimizePose(query) :29-44
 *   lgs_loop_detect_bb           LoopDetectorBranchBound::Detect + FindCorrespondingPose
 *                                C/mapping/loop_detector_branch_bound.cpp:26-117
 *
 * Threading: one lgs_ctx per matcher instance (the reference's frontend and
 * loop detector own distinct matchers, C/slam_launcher.cpp:774-775, :835).  A
 * context owns one HIP stream and its scratch; calls on one context must not
 * overlap, calls on different contexts may.
 *
 * Numerics: fp64 throughout.  Cell indices, hit/miss counts, map cells, the
 * correlative argmax/score and the Gauss-Newton refine (glibc's
 * sincos/pow restated on the device, sums in beam order) are bit-exact with the
 * reference CPU path; greedy-endpoint costs/covariances agree to within 1e-5
 * (device exp differs from glibc in the last ulp).
 */
#ifndef LGS_HIP_H
#define LGS_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 2: lgs_carmen_load gained ids_bytes (include/lgs_io.h), options 6/12/14/16
 * retired, options 22/23 and lgs_loop_records_allgather added */
#define LGS_ABI_VERSION 2

/* status codes */
#define LGS_OK               0
#define LGS_ERR_INVALID_ARG  1
#define LGS_ERR_HIP          2
#define LGS_ERR_NO_DEVICE    3
#define LGS_ERR_OOM          4
#define LGS_ERR_INTERNAL     5

typedef struct lgs_ctx  lgs_ctx;   /* device, stream, scratch arena */
typedef struct lgs_grid lgs_grid;  /* device-resident dense fp64 grid */
typedef struct lgs_scan lgs_scan;  /* device-resident scan (ScanData<double>) */

/* RobotPose2D<double> (H/pose.hpp:14-42) */
typedef struct { double x, y, theta; } lgs_pose2d;

/* Host view of a ScanData<double> (H/sensor/sensor_data.hpp:65-158) */
typedef struct {
    const double* ranges;        /* n */
    const double* angles;        /* n */
    int n;
    lgs_pose2d rel_sensor_pose;  /* RelativeSensorPose() */
    double min_range, max_range; /* MinRange(), MaxRange() */
} lgs_scan_host;

/* ScanMatcherRealTimeCorrelative ctor arguments
 * (H/mapping/scan_matcher_real_time_correlative.hpp:19-25) */
typedef struct {
    int low_resolution;
    double range_x, range_y, range_theta;
    double scan_range_max;
} lgs_rtcsm_params;

/* CostGreedyEndpoint *member* values (C/mapping/cost_function_greedy_endpoint.cpp:10-28).
 * The reference launcher passes (stddev, scale) into the (scale, stddev) slots
 * (C/slam_launcher.cpp:70-72); callers fill these with the members as constructed. */
typedef struct {
    double usable_range_min, usable_range_max;
    double hit_and_missed_dist, occupancy_threshold;
    int kernel_size;
    double scaling_factor;
    double standard_deviation;
} lgs_cost_ge_params;

/* ScanMatchingSummary (H/mapping/scan_matcher.hpp:147-174) + diagnostics */
typedef struct {
    int pose_found;
    double normalized_cost;
    lgs_pose2d initial_pose;
    lgs_pose2d estimated_pose;
    double covariance[9];         /* row-major 3x3 */
    /* diagnostics */
    double score_max;             /* best (fine) score, sequential fp64 beam-order sum */
    double score_threshold;       /* normalizedScoreThreshold * NumOfScans() */
    int best_win[3];              /* x, y, theta window indices of the argmax */
    int win[3];                   /* winX, winY, winTheta */
    double steps[3];              /* stepX, stepY, stepTheta */
    lgs_pose2d best_sensor_pose;
    int64_t coarse_blocks;        /* coarse blocks scored: all of them, or those superblock pruning kept */
    int64_t fine_blocks;          /* coarse blocks refined on the fine map */
    int guard_hits;               /* projections near a cell boundary re-checked on host */
    int fixups;                   /* 1 if any device index differed from glibc and was patched */
    int slow_path;                /* 1 if the exact dense fallback was taken */
} lgs_rtcsm_summary;

/* ---- context ---- */
int  lgs_ctx_create(int device, lgs_ctx** out);
void lgs_ctx_destroy(lgs_ctx* ctx);
const char* lgs_ctx_last_error(const lgs_ctx* ctx);
int  lgs_ctx_synchronize(lgs_ctx* ctx);
void* lgs_ctx_stream(lgs_ctx* ctx);       /* hipStream_t, for interop (torch) */
int  lgs_abi_version(void);

/* Test/diagnostic knobs (never needed in production):
 *  LGS_OPT_GUARD_EPS     boundary guard in cells (default 1e-9)
 *  LGS_OPT_FORCE_DENSE   1 = refine every coarse block above threshold
 *  LGS_OPT_INJECT_INDEX  1 = corrupt every guarded device index (exercises the fix-up path)
 *  LGS_OPT_GUARD_CAP     max guard records inspected before full host re-projection */
#define LGS_OPT_GUARD_EPS     1
#define LGS_OPT_FORCE_DENSE   2
#define LGS_OPT_INJECT_INDEX  3
#define LGS_OPT_GUARD_CAP     4
#define LGS_OPT_PROFILE       5   /* 1 = time every kernel launch with HIP events on the ctx stream */
#define LGS_OPT_PROFILE_MASK  7   /* time only the kernels whose lgs_kernel_stat index bit is set (0 = off) */
#define LGS_OPT_SPIN_SYNC     8   /* 1 (default) = spin on the stream when waiting for results, 0 = blocking wait */
#define LGS_OPT_SKIP_MASK     10  /* diagnostics only: bitmask of kernels (lgs_ctx_kernel_stats order) not launched -- results are invalid */
#define LGS_OPT_SUPER_PRUNE   9   /* 1 (default) = skip coarse blocks whose 4x4-superblock bound is below the seed score, 0 = evaluate every coarse block */
#define LGS_OPT_RAY_CHUNK_KEYS 13  /* ray-cast keys per emit/sort/apply pass (default 2^28, max 2^30); more keys are cast in scan order over several passes */
#define LGS_OPT_LANES_MIN_BATCH 11 /* pruned coarse stage: the kept-superblock work list (lane-per-block sums) for batches of at least this many matches (default 2; 1 = always), else the row kernel */
#define LGS_OPT_LINSOLVE_SPLIT 17 /* 1 (default) = a lone ScanMatcherLinearSolver refine of <= 1280 beams runs one workgroup per 64 beams (in-launch hand-off per pass) when they fit the device at once, 0 = one workgroup */
#define LGS_OPT_HANDOFF_SPIN_US 18 /* split refine: bound of a workgroup's wait for the others (default 200000 us); on time-out the refine is rerun on one workgroup.  0 = force that fallback (tests) */
#define LGS_OPT_PEER_COPY     19  /* lgs_loop_detect_rtcsm_multi, on the shard's ctx: 0 (default) = maps copied device to device (peer access enabled when the devices differ and allow it, else staged through pinned host memory), 1 = always staged through host memory */
#define LGS_OPT_PRUNE_MIN_SUPER 21 /* superblock pruning only for windows of at least this many superblocks per angle (default 1); smaller windows score every coarse block */
#define LGS_OPT_COOP_TILES    22  /* K3 one-launch sort (k_sort_wide): at most this many tiles for this ctx's launches (default -1 = the device's co-residency capacity, shared by every ctx of the process; 0 = always the multi-pass sort) */
#define LGS_OPT_SORT_BARRIER_US 23 /* bound of a one-launch sort tile's wait at its grid barrier (default 50000 us); on time-out the call reports LGS_ERR_INTERNAL.  0 = time out at once (tests) */
#define LGS_OPT_FINE_STAGED   24  /* 1 (default) = batched fine evaluation of LowRes-5 blocks stages each beam's window in LDS (k_fine_regs), 0 = per-beam gathers (k_fine_lanes) */
#define LGS_OPT_SMALL_WINDOW  25  /* 1 (default) = windows with one coarse block per angle (2 winX < LowRes, 2 winY < LowRes, LowRes 2..7, map width >= LowRes, <= 2048 valid beams) search in one launch (k_match_small: no coarse map), 0 = the general path */
#define LGS_OPT_POST_RECORDS  26  /* 1 (default) = a match call's result records reach the host through a kernel that writes them (and a completion flag) into pinned memory, the host spinning on the flag; 0 = a device-to-host copy and a stream event */
#define LGS_OPT_FUSED_PLANES  27  /* 1 (default) = the per-query coarse-map precompute writes the phase planes AND the octet superblock units in one pass from the fine map (k_planes_super, LowRes 5), 0 = the precompute + k_super_planes passes */
#define LGS_OPT_PRIORITY_TAIL 28  /* 0 (default) = one stream; 1 = a correlative batch's stages after the coarse-map builds run on a second stream of the device's highest priority (behind an event), so that other contexts' plane builds cannot queue ahead of its latency-bound tail */
#define LGS_OPT_HV_FULL       29  /* A/B: 1 = the superblock pass (k_super_hv) stores each 16-byte unit whole from two quads' maxima; 0 (default) = each quad's halves */
#define LGS_OPT_SPLIT_CHUNKS  30  /* A/B: 1 = a correlative call of 32..64 matches runs as two chunks of half the size (the two buffer banks overlap); 0 (default) = one chunk per 64 */
#define LGS_OPT_DEVICE_HITS   31  /* 1 (default) = lgs_maps_construct_from_scans / lgs_map_construct_global form the hit points (glibc sincos restated), boxes, ray cells and key offsets on the device; 0 = on the host */
#define LGS_OPT_SEED_WIDE     32  /* batches: the pruning bound seeded from the best members of this many candidate superblocks (5..16, default 12; the 4 best members fine-scored); 0..4 = 4 candidates in one launch */
#define LGS_OPT_ZERO_TILES    33  /* 1 (default) = the per-map passes of a correlative batch skip the stores of a tile whose inputs are all +0 when that set's buffer already holds the tile's +0 outputs (per-tile words kept per bank, set and layout); 0 = every tile stored */
#define LGS_OPT_DEVICE_TIMING 34  /* 1 = while LGS_OPT_PROFILE(_MASK) times a kernel of a correlative batch chunk, time it on the device instead of with stream events: its workgroups stamp s_memrealtime (100 MHz) at start and end into per-chunk words (two relaxed atomic maxima per workgroup), copied back with the chunk's records; a launch's time is its first workgroup's start to its last workgroup's end (the execution span rocprofv3 reports, not the wait of a stream event for the CUs).  Launches outside a chunk's main chain keep event timing.  0 (default) = events */
#define LGS_OPT_LEAN_PROJECT  35  /* 1 (default) = batched pruned correlative chunks (work list, wide seed, staged fine evaluation) write only the superblock base of every (angle, beam) plus per-beam / per-angle trig tables, and the kernels that stage a coarse-base or cell row form it themselves with the projection's own arithmetic (bit-identical); 0 = every row materialised (the guard fix-up reruns and lone matches always materialise) */
#define LGS_OPT_POISON_WS     15  /* diagnostics: 1 = fill every match workspace and record with 0xFF bytes before the batch runs (any read-before-write shows up) */
int  lgs_ctx_set_option(lgs_ctx* ctx, int option, double value);

/* Diagnostics: copy one intermediate buffer of item `item` of the context's
 * last correlative batch to `out` (at most cap bytes; *bytes = its full size).
 * which: 0 sbound [T*nsb2 f64], 1 part_c [nparts f64], 2 part_k [nparts i64],
 * 3 Lp at byte 0, Lc[4] f64 at byte 64, 4 tedge [T i32] (1 = flagged by
 * the last enqueue of item 0, else 0), 5 cbase [2*(T*Nv+pad) i32],
 * 6 idx [T*Nv int2], 7 cscore [K f64], 8 coarse phase planes [lr*lr planes
 * of Hqp x Wqp f64, DESIGN.md §2], 9 superblock planes [fp16]. */
int  lgs_debug_item_buffer(lgs_ctx* ctx, int item, int which, void* out, size_t cap, size_t* bytes);

/* Diagnostics: the device's restatements of glibc's sincos() (op 0: out[2i] =
 * sin x[i], out[2i+1] = cos x[i]) and pow(x, 3.0) (op 1: out[i]) evaluated on
 * the GPU for n host inputs (csrc/glibc_math.hpp; tests compare them with the
 * host libm bit for bit). */
int  lgs_debug_libm(lgs_ctx* ctx, int op, const double* x, int n, double* out);

/* Diagnostics: the K3 sort (csrc/k_sort.hip, the stable radix sort behind
 * every ray-cast pass) of n host keys on bits [lo, lo + bits), through the
 * device; out receives the sorted keys. */
int  lgs_debug_keysort(lgs_ctx* ctx, const unsigned* keys, unsigned* out, long long n, int lo, int bits);

/* Diagnostics: cross-context copies made by lgs_loop_detect_rtcsm_multi onto
 * this context since it was created: device to device (same device or peer
 * access over xGMI) and staged through pinned host memory. */
int  lgs_debug_copy_counters(const lgs_ctx* ctx, long long* direct, long long* staged);

/* Diagnostics, checked build only (liblgs_hip_checked.so, compiled with
 * LGS_CHECK_OFFSETS): the correlative consumers test every
 * coarse / superblock plane offset they form or read against its padded
 * plane.  out[0] = offsets checked, out[1] = violations, out[2] = the first
 * violation (kind << 60 | angle << 32 | beam; kind 1 coarse, 2 superblock),
 * out[3] = its offset; since the last reset (reset != 0 zeroes them after
 * the read).  The product build returns LGS_ERR_INVALID_ARG (no checks). */
int  lgs_debug_offset_checks(lgs_ctx* ctx, int reset, unsigned long long* out);

/* Per-kernel statistics gathered while LGS_OPT_PROFILE is on.  algo_bytes is
 * the algorithmic byte count of DESIGN.md §Roofline (e.g. 8 B per coarse-score
 * lookup), summed over launches; total_ms sums hipEventElapsedTime, or with
 * LGS_OPT_DEVICE_TIMING each launch's execution span (first workgroup start to
 * last workgroup end); dispatch_ms (device timing only, else = total_ms) sums
 * the span from the end of the chunk's previous device-timed launch on the
 * same stream to the launch's end -- what a stream event or a rocprofv3
 * dispatch duration counts: the execution plus the wait for CUs held by other
 * streams' kernels (r06). */
typedef struct {
    char name[32];
    int64_t launches;
    double total_ms;
    double algo_bytes;
    double dispatch_ms;
} lgs_kernel_stat;
int  lgs_ctx_kernel_stats(lgs_ctx* ctx, lgs_kernel_stat* out, int cap);  /* returns count (>=0) or -status */
int  lgs_ctx_reset_stats(lgs_ctx* ctx);
/* Correlative-match counters since the last lgs_ctx_reset_stats, over every
 * OptimizePose / loop-detect match on the context (always collected):
 * out4 = {matches, coarse blocks scored, coarse blocks a dense search scores
 * (sum of the plans' K), matches that used superblock pruning}. */
int  lgs_ctx_match_counters(lgs_ctx* ctx, int64_t* out4);

/* ---- grids: dense row-major fp64, cell (x,y) at y*w+x, 0.0 = unknown ---- */
int  lgs_grid_create(lgs_ctx* ctx, int w, int h, double min_x, double min_y,
                     double resolution, lgs_grid** out);
/* non-owning view over existing device memory (e.g. a torch tensor) */
int  lgs_grid_wrap(lgs_ctx* ctx, double* device_cells, int w, int h, double min_x,
                   double min_y, double resolution, lgs_grid** out);
void lgs_grid_destroy(lgs_grid* grid);
int  lgs_grid_upload(lgs_ctx* ctx, lgs_grid* grid, const double* host_cells);
/* Patch-native upload of a reference GridMapType (GridMap<BinaryBayesGridCell
 * <double>>, H/grid_map/grid_map.hpp:295-317 mPatches, H/grid_map/
 * grid_map_patch.hpp:15-193): patches[py * npx + px] = PatchAt(px, py).Data()
 * (its patch_size^2 cells, cell (x, y) of the patch at y * patch_size + x) or
 * NULL for an unallocated patch (reads Unknown = 0.0, as GridMap::Value
 * does).  Each cell is cell_bytes bytes with its fp64 value at value_offset
 * (BinaryBayesGridCell<double>: 16 and 8 -- vptr, mValue).  The grid must be
 * npx*patch_size x npy*patch_size.  Only allocated patches cross PCIe, as
 * their raw cells (host copies into pinned staging overlap the DMA); a kernel
 * extracts the values into the dense grid and zero-fills unallocated patches.
 * Replaces INTEGRATION.md §2's Flatten (one virtual Value() per cell) +
 * lgs_grid_upload of the whole dense map. */
int  lgs_grid_upload_patches(lgs_ctx* ctx, lgs_grid* grid, const void* const* patches, int npx, int npy,
                             int patch_size, int cell_bytes, int value_offset);
int  lgs_grid_download(lgs_ctx* ctx, const lgs_grid* grid, double* host_cells);
int  lgs_grid_fill(lgs_ctx* ctx, lgs_grid* grid, double value);
int  lgs_grid_info(const lgs_grid* grid, int* w, int* h, double* min_x, double* min_y,
                   double* resolution);
double* lgs_grid_device_ptr(lgs_grid* grid);

/* PrecomputeGridMap(grid, win) into `out` (same geometry). */
int  lgs_grid_precompute_max(lgs_ctx* ctx, const lgs_grid* in, int win, lgs_grid* out);

/* ---- scans: a host copy, and a device copy resident in HBM once made ----
 * lgs_scan_create copies the ranges/angles (host memory only: no device
 * work, no synchronisation).  The first call that reads the scan on the
 * device copies it there, on that call's context (pooled device buffers), and
 * it stays resident until lgs_scan_destroy.  A scan belongs to the context
 * that created it; other contexts use clones (lgs_loop_detect_rtcsm_multi
 * re-creates them from the host copy).  Copies are waited for where a scan is
 * read on a context other than the one that made them. */
int  lgs_scan_create(lgs_ctx* ctx, const lgs_scan_host* host, lgs_scan** out);
void lgs_scan_destroy(lgs_scan* scan);
/* Number of beams, and (if the pointers are non-null) a copy of the ranges and
 * angles of `scan` into caller arrays of at least that many doubles. */
int  lgs_scan_get(const lgs_scan* scan, int* n, double* ranges, double* angles);
/* ScanInterpolator::Interpolate (C/mapping/scan_interpolator.cpp:9-98): a new
 * device-resident scan whose points are spaced dist_scans apart along the
 * polyline of `in`'s points, except across gaps of >= dist_threshold_empty
 * (launcher JSON "ScanInterpolator": DistScans 0.05, DistThresholdEmpty 0.25).
 * The relative sensor pose and min/max range are copied.  The recurrence is
 * sequential and uses glibc sincos/atan2/sqrt, so it runs on the host; the
 * result is a scan like lgs_scan_create's.  LGS_ERR_INVALID_ARG unless
 * 0 < dist_scans <= dist_threshold_empty (both finite) and every point of
 * `in` is finite: the reference's loop would never end otherwise. */
int  lgs_scan_interpolate(lgs_ctx* ctx, const lgs_scan* in, double dist_scans, double dist_threshold_empty,
                          lgs_scan** out);

/* ---- correlative scan matcher ---- */
int  lgs_rtcsm_optimize_pose(lgs_ctx* ctx, const lgs_grid* grid, const lgs_grid* coarse,
                             const lgs_rtcsm_params* params,
                             const lgs_cost_ge_params* cost,
                             const lgs_scan* scan, lgs_pose2d initial_pose,
                             double normalized_score_threshold,
                             lgs_rtcsm_summary* out);
/* OptimizePose(query): coarse map computed on device, threshold DBL_MIN */
int  lgs_rtcsm_optimize_pose_query(lgs_ctx* ctx, const lgs_grid* grid,
                                   const lgs_rtcsm_params* params,
                                   const lgs_cost_ge_params* cost,
                                   const lgs_scan* scan, lgs_pose2d initial_pose,
                                   lgs_rtcsm_summary* out);
/* n independent OptimizePose(query) calls (each query: its map, scan and
 * initial pose; every query computes its own coarse map, as the reference's
 * OptimizePose(query) does, even when two queries pass the same map).  One
 * batched device pipeline: every stage is a single launch over all n queries.
 * The maps of one call must share size and resolution.  out[j] is
 * bit-identical to lgs_rtcsm_optimize_pose_query on query j. */
int  lgs_rtcsm_optimize_pose_query_batch(lgs_ctx* ctx, const lgs_grid* const* grids,
                                         const lgs_rtcsm_params* params,
                                         const lgs_cost_ge_params* cost,
                                         const lgs_scan* const* scans,
                                         const lgs_pose2d* initial_poses, int n,
                                         lgs_rtcsm_summary* out);
/* n independent matches against one grid and its coarse map, as one batched
 * device pipeline (loop-closure candidates, C/.../loop_detector_real_time_correlative.cpp:66) */
int  lgs_rtcsm_optimize_pose_batch(lgs_ctx* ctx, const lgs_grid* grid, const lgs_grid* coarse,
                                   const lgs_rtcsm_params* params,
                                   const lgs_cost_ge_params* cost,
                                   const lgs_scan* const* scans, const lgs_pose2d* initial_poses,
                                   int n, double normalized_score_threshold,
                                   lgs_rtcsm_summary* out);
/* Every coarse and fine score of the search window (kernel-level parity).
 * dims[7] = {winX, winY, winTheta, ncx, ncy, nfx, nfy}; pass NULL score
 * buffers to query dims.  coarse_scores[T][ncx][ncy], fine_scores[T][nfx][nfy]. */
int  lgs_rtcsm_dense_scores(lgs_ctx* ctx, const lgs_grid* grid, const lgs_grid* coarse,
                            const lgs_rtcsm_params* params, const lgs_scan* scan,
                            lgs_pose2d initial_pose, double* coarse_scores,
                            double* fine_scores, int* dims);

/* ---- occupancy-grid maps: GridMap<BinaryBayesGridCell<double>> ----
 * Geometry follows the reference exactly (H/grid_map/grid_map.hpp): square
 * patches of patch_size cells, minPos anchoring, Resize/Expand with the
 * negative patch-index quirk (:905-915).  Cells live on the device (dense,
 * row-major over the whole patch grid, 0.0 = unknown); the per-beam
 * Bresenham ray-cast and binary Bayes update run on the device in the
 * reference's update order (beam order; misses along a ray before its hit),
 * so every cell value is bit-exact. */
typedef struct lgs_map lgs_map;

/* GridMapBuilder ctor arguments used by the ray-cast (C/mapping/grid_map_builder.cpp:20-45) */
typedef struct {
    double usable_range_min, usable_range_max;
    double prob_hit, prob_miss;
} lgs_builder_params;

typedef struct {
    double resolution;
    int patch_size;
    int num_patches_x, num_patches_y;
    int num_cells_x, num_cells_y;
    double min_x, min_y;
} lgs_map_geometry;

/* GridMap(res, patchSize, numCellsX, numCellsY, centerPos) (H/grid_map/grid_map.hpp:337-391) */
int  lgs_map_create(lgs_ctx* ctx, double resolution, int patch_size, int num_cells_x,
                    int num_cells_y, double center_x, double center_y, lgs_map** out);
void lgs_map_destroy(lgs_map* map);
int  lgs_map_get_geometry(const lgs_map* map, lgs_map_geometry* out);
/* Non-owning grid view of the map's cells (valid until the next geometry change
 * or lgs_map_destroy); lgs_grid_destroy on a view is a no-op. */
int  lgs_map_grid(lgs_map* map, lgs_grid** out);
/* One scan into the map as GridMapBuilder::UpdateGridMap does after choosing
 * the local map (C/mapping/grid_map_builder.cpp:149-186): bounding box,
 * Expand(.., 5.0), then the ray-cast update. */
int  lgs_map_update_scan(lgs_ctx* ctx, lgs_map* map, const lgs_scan* scan, lgs_pose2d robot_pose,
                         const lgs_builder_params* params);
/* GridMapBuilder::ConstructMapFromScans (C/mapping/grid_map_builder.cpp:227-332):
 * Resize to the bounding box of all scans (topRight starts at DBL_MIN), Reset,
 * then ray-cast every scan in order.  Called again on the same map with the
 * window of UpdateLatestMap (:196-207: the previous scans, less at most the
 * oldest, plus one new scan; same poses, parameters and geometry), only the
 * cells the new or the dropped scan touch are recomputed (DESIGN.md §4.4b;
 * same cells, counts and patch flags as a full rebuild).  Such an incremental
 * call returns before its device work has finished: reads of the map through
 * this library wait for it (on any context); lgs_grid_device_ptr users
 * synchronise the context first.  An internal error of that work is reported
 * by the map's next rebuild (LGS_ERR_INTERNAL, e.g. "grid barrier timed out"
 * when the one-launch sort's tiles could not be co-resident): the update
 * kernels of that step have then run over unsorted keys, so the cells of this
 * map AND of the local map an lgs_map_append_scan step inserted into are
 * undefined.  The library drops the latest map's incremental state (its next
 * call rebuilds it in full); the caller must rebuild the local map
 * (lgs_map_construct_from_scans) before reading it again. */
int  lgs_map_construct_from_scans(lgs_ctx* ctx, lgs_map* map, const lgs_scan* const* scans,
                                  const lgs_pose2d* robot_poses, int n,
                                  const lgs_builder_params* params);
/* GridMapBuilder::AppendScan (C/mapping/grid_map_builder.cpp:48-59): the
 * newest scan scans[n-1] at robot_poses[n-1] inserted into `local` exactly as
 * lgs_map_update_scan does (UpdateGridMap :98-193), and `latest` rebuilt from
 * all n scans exactly as lgs_map_construct_from_scans does (UpdateLatestMap
 * :196-207; n = min(node count, NumOfScansForLatestMap)).  Same results as the
 * two calls; both ray-casts share one device pass (one cast of the new scan
 * when the two maps' cells of it differ by a whole-cell shift).  Incremental
 * and asynchronous as lgs_map_construct_from_scans.  local != latest. */
int  lgs_map_append_scan(lgs_ctx* ctx, lgs_map* local, lgs_map* latest, const lgs_scan* const* scans,
                         const lgs_pose2d* robot_poses, int n, const lgs_builder_params* params);

/* Diagnostics: how a map's ConstructMapFromScans / AppendScan rebuilds ran
 * (DESIGN.md §4.4b): incremental steps (the window gained one scan and lost
 * at most its oldest, same geometry: only the touched cells recomputed) and
 * full rebuilds.  Both zero for a map never rebuilt. */
int  lgs_debug_map_rebuilds(const lgs_map* m, long long* incremental, long long* full);

/* GridMapBuilder::AfterLoopClosure's map loop (C/mapping/grid_map_builder.cpp:62-80):
 * ConstructMapFromScans(maps[i], poseGraph, idx_min[i], idx_max[i]) for every
 * i, where node k of the pose graph is (scans[k], robot_poses[k]) and
 * idx_min[i] <= idx_max[i] < n_nodes (inclusive ranges; they may overlap).
 * The maps must be distinct.  Each map is resized and reset as
 * lgs_map_construct_from_scans does; all maps then share one ray-cast pass,
 * which gives the same cells as constructing them one after another. */
int  lgs_maps_construct_from_scans(lgs_ctx* ctx, lgs_map* const* maps, const int* idx_min,
                                   const int* idx_max, int n_maps, const lgs_scan* const* scans,
                                   const lgs_pose2d* robot_poses, int n_nodes,
                                   const lgs_builder_params* params);
/* GridMapBuilder::ConstructGlobalMap (C/mapping/grid_map_builder.cpp:83-95): a
 * new map of (resolution, patch_size) with 0 x 0 cells centred at (0, 0),
 * then ConstructMapFromScans over all n nodes.  Any number of scans: the
 * ray-cast runs in passes of at most LGS_OPT_RAY_CHUNK_KEYS keys. */
int  lgs_map_construct_global(lgs_ctx* ctx, double resolution, int patch_size,
                              const lgs_scan* const* scans, const lgs_pose2d* robot_poses, int n,
                              const lgs_builder_params* params, lgs_map** out);
/* MapSaver::DrawMap (C/io/map_saver.cpp:276-313) over the whole map: one gray
 * byte per cell, (uint8)((1 - p) * 255) for 0 < p <= 1 and 192 otherwise, rows
 * flipped up-down as the reference writes its PNG (:455-456); image holds
 * num_cells_x * num_cells_y bytes.  The reference crops the image to the
 * allocated patches (GridMap::ComputeActualMapSize); the caller crops with
 * the hit/miss counts if it needs that extent. */
int  lgs_map_render_gray(lgs_ctx* ctx, const lgs_map* map, uint8_t* image);
/* MapSaver::DrawMap for the w x h cells starting at cell (x0, y0) -- the
 * region SaveMapCore draws (C/io/map_saver.cpp:413-437): gray bytes as
 * lgs_map_render_gray, rows flipped up-down if flip_rows.  The region must lie
 * inside the map. */
int  lgs_map_render_gray_region(lgs_ctx* ctx, const lgs_map* map, int x0, int y0, int w, int h,
                                int flip_rows, uint8_t* image);
/* Patch::IsAllocated per patch (H/grid_map/grid_map_patch.hpp:40), row-major
 * num_patches_x * num_patches_y bytes: a patch is allocated by the first
 * update of one of its cells (GridMap::GridCellAt, H/grid_map/grid_map.hpp:807-823),
 * moves with Resize (:652-711) and stays allocated across Reset. */
int  lgs_map_download_patches(lgs_ctx* ctx, const lgs_map* map, uint8_t* flags);
/* GridMap::ComputeActualMapSize (H/grid_map/grid_map.hpp:969-1015): the
 * bounding box of the allocated patches.  out[12] = patchIdxMin x, y;
 * patchIdxMax x, y (exclusive, after the reference's +1); gridCellIdxMin x, y;
 * gridCellIdxMax x, y; mapSizeInPatches x, y; mapSizeInGridCells x, y.
 * *num_allocated = allocated patches; with none the reference's bounds are
 * INT_MAX/INT_MIN (undefined sizes) and out is all zero here. */
int  lgs_map_actual_size(lgs_ctx* ctx, const lgs_map* map, int* num_allocated, int* out);
/* Copy cells and per-cell hit/miss update counts (since create/construct) to
 * the host; any pointer may be NULL.  Sizes: num_cells_x * num_cells_y. */
int  lgs_map_download(lgs_ctx* ctx, const lgs_map* map, double* cells, uint32_t* hit_count,
                      uint32_t* miss_count);

/* CostGreedyEndpoint::Cost at one sensor pose */
int  lgs_cost_greedy_endpoint(lgs_ctx* ctx, const lgs_grid* grid,
                              const lgs_cost_ge_params* cost, const lgs_scan* scan,
                              lgs_pose2d sensor_pose, double* out_cost);

/* ---- loop-closure batch (LoopDetectorRealTimeCorrelative::Detect) ----
 * C/mapping/loop_detector_real_time_correlative.cpp:26-125.  A query is one
 * local map (LoopDetectionQuery::mLocalMapInfo / mLocalMapNode) and the
 * contiguous range of candidates (its mPoseGraphNodes) matched against it. */
typedef struct {
    const lgs_grid* map;            /* local grid map */
    const lgs_grid* coarse;         /* its cached coarse map, or NULL = compute (:52-60) */
    lgs_pose2d local_map_node_pose; /* mLocalMapNode.Pose() */
    int local_map_node_index;       /* mLocalMapNode.Index() */
    int first_candidate, num_candidates;
} lgs_loop_query;

typedef struct {
    const lgs_scan* scan;           /* poseGraphNode.ScanData() */
    lgs_pose2d node_pose;           /* poseGraphNode.Pose() (initial pose) */
    int node_index;                 /* poseGraphNode.Index() */
    int pad;
} lgs_loop_candidate;

/* LoopDetectionResult (H/mapping/loop_detector.hpp:60-87) + diagnostics; a
 * fixed 176-byte record (22 x 8 B) so shards can be all-gathered as a flat array. */
typedef struct {
    int found;                      /* 0: the reference appends no result */
    int start_node_index, end_node_index;
    int pad;
    lgs_pose2d relative_pose;       /* InverseCompound(localMapNode.Pose(), estimated) */
    lgs_pose2d start_node_pose;
    lgs_pose2d estimated_pose;      /* matcher's estimate (world frame) */
    double covariance[9];
    double score;                   /* correlative score of the best pose */
    double normalized_cost;
} lgs_loop_result;

/* One result per candidate, in candidate order. */
int  lgs_loop_detect_rtcsm(lgs_ctx* ctx, const lgs_rtcsm_params* params, const lgs_cost_ge_params* cost,
                           double score_threshold, const lgs_loop_query* queries, int num_queries,
                           const lgs_loop_candidate* candidates, int num_candidates,
                           lgs_loop_result* results);

/* Multi-GPU Detect for a caller that owns several GPUs in one
 * process (the reference's backend calls Detect once,
 * C/mapping/lidar_graph_slam_backend.cpp:39-40): the same contract and the
 * same results, byte for byte, as lgs_loop_detect_rtcsm on ctxs[0].  The
 * candidates are split into num_ctx contiguous shards, shard k =
 * [k*n/N, (k+1)*n/N) runs on ctxs[k] on its own host thread; maps, coarse maps
 * and scans owned by another context are copied to ctxs[k] first (peer copy
 * over xGMI; scans re-uploaded from their host copy).  Errors of any shard are
 * reported on ctxs[0]. */
int  lgs_loop_detect_rtcsm_multi(lgs_ctx* const* ctxs, int num_ctx, const lgs_rtcsm_params* params,
                                 const lgs_cost_ge_params* cost, double score_threshold,
                                 const lgs_loop_query* queries, int num_queries,
                                 const lgs_loop_candidate* candidates, int num_candidates,
                                 lgs_loop_result* results);

/* ---- the loop batch over several processes (one per GPU) ----
 * Candidates are independent (C/mapping/loop_detector_real_time_correlative.cpp:38, :66):
 * rank r of `world` matches the contiguous block [lo_r, hi_r) of the n
 * candidates (lgs_loop_shard_bounds: block sizes differ by at most one, the
 * larger blocks first) with lgs_loop_detect_rtcsm, then
 * lgs_loop_records_allgather gathers every rank's records into `all` (host,
 * n records, candidate order -- the order the reference's
 * LoopDetectionResultVector keeps) with ONE ncclAllGather of fixed-size rows
 * on ctx's stream (RCCL over xGMI), and synchronises the stream.  `comm` is an
 * ncclComm_t of `world` ranks whose rank `rank` lives on ctx's device (made
 * by the caller, or with lgs_rccl_comm_init).  RCCL is resolved at run time
 * (librccl.so.1, an already loaded copy first). */
int  lgs_loop_shard_bounds(int n, int world, int rank, int* lo, int* hi);
int  lgs_loop_records_allgather(lgs_ctx* ctx, void* comm, int rank, int world, int n,
                                const lgs_loop_result* local, lgs_loop_result* all);
/* RCCL communicator helpers: a 128-byte ncclUniqueId made on one rank and
 * sent to the others by the caller, then one lgs_rccl_comm_init per rank. */
int  lgs_rccl_unique_id(unsigned char* id128);
int  lgs_rccl_comm_init(lgs_ctx* ctx, const unsigned char* id128, int world, int rank, void** comm);
int  lgs_rccl_comm_destroy(void* comm);

/* ---- branch-and-bound matcher ----
 * ScanMatcherBranchBound (C/mapping/scan_matcher_branch_bound.cpp:8-200,
 * H/mapping/scan_matcher_branch_bound.hpp) with ScorePixelAccurate
 * (C/mapping/score_function_pixel_accurate.cpp:19-77) and the grid-map
 * pyramid PrecomputeGridMaps (C/mapping/grid_map_builder.cpp:471-495).
 * The device scores every node the reference's depth-first search can visit
 * (level by level, a superset bounded by the threshold argument of
 * DESIGN.md §4.6); the host then replays the reference's LIFO search over
 * those scores, so the result is the reference's own (best node, score,
 * nodes visited).  Field order follows the constructor (nodeHeightMax,
 * rangeX, rangeY, rangeTheta, scanRangeMax) then ScorePixelAccurate
 * (usableRangeMin, usableRangeMax). */
typedef struct {
    int    node_height_max;
    double range_x, range_y, range_theta;
    double scan_range_max;
    double score_usable_range_min, score_usable_range_max;
} lgs_bb_params;

/* PrecomputeGridMaps: pyramid[h] = window-max map with window 2^h,
 * h = 0..node_height_max (node_height_max + 1 grids of the input's geometry,
 * created by the caller). */
int  lgs_grid_precompute_pyramid(lgs_ctx* ctx, const lgs_grid* in, int node_height_max,
                                 lgs_grid* const* pyramid);
/* OptimizePose(gridMap, precompMaps, scan, pose, thr) (:47-154) for n scans
 * against one pyramid (loop-closure candidates); summaries as the RTCSM
 * ones, with best_win = the best node's (x, y, theta), coarse_blocks = nodes
 * scored on the device, fine_blocks = nodes the reference's search visits. */
int  lgs_bb_optimize_pose_batch(lgs_ctx* ctx, const lgs_grid* grid, const lgs_grid* const* pyramid,
                                const lgs_bb_params* params, const lgs_cost_ge_params* cost,
                                const lgs_scan* const* scans, const lgs_pose2d* initial_poses, int n,
                                double normalized_score_threshold, lgs_rtcsm_summary* out);
/* OptimizePose(query) (:29-44): pyramid of the query's map, threshold DBL_MIN */
int  lgs_bb_optimize_pose_query(lgs_ctx* ctx, const lgs_grid* grid, const lgs_bb_params* params,
                                const lgs_cost_ge_params* cost, const lgs_scan* scan,
                                lgs_pose2d initial_pose, lgs_rtcsm_summary* out);
/* LoopDetectorBranchBound::Detect + FindCorrespondingPose
 * (C/mapping/loop_detector_branch_bound.cpp:26-117): per query the pyramid of
 * its local map (computed here; lgs_loop_query.coarse is ignored), then every
 * candidate matched with the score threshold.  One result per candidate. */
int  lgs_loop_detect_bb(lgs_ctx* ctx, const lgs_bb_params* params, const lgs_cost_ge_params* cost,
                        double score_threshold, const lgs_loop_query* queries, int num_queries,
                        const lgs_loop_candidate* candidates, int num_candidates,
                        lgs_loop_result* results);

/* ---- K4: Gauss-Newton refine (ScanMatcherLinearSolver + CostSquareError) ----
 * Replaces ScanMatcherLinearSolver::OptimizePose (C/mapping/scan_matcher_linear_solver.cpp:38-85,
 * H/mapping/scan_matcher_linear_solver.hpp:15-56) with its CostSquareError
 * (C/mapping/cost_function_square_error.cpp).  Field order follows the
 * constructor (numOfIterationsMax, convergenceThreshold, usableRangeMin/Max,
 * translation/rotation regularizer) then CostSquareError(usableRangeMin/Max). */
typedef struct {
    int    num_iterations_max;
    double convergence_threshold;
    double usable_range_min, usable_range_max;
    double translation_regularizer, rotation_regularizer;
    double cost_usable_range_min, cost_usable_range_max;
} lgs_linsolve_params;

/* ScanMatchingSummary (H/mapping/scan_matcher.hpp:26-77) plus diagnostics */
typedef struct {
    int pose_found;               /* always 1, as the reference */
    int iterations;               /* OptimizeStep calls made */
    double normalized_cost;       /* cost / NumOfScans() */
    lgs_pose2d initial_pose;
    lgs_pose2d estimated_pose;    /* MoveBackward(bestSensorPose, relPose) */
    double covariance[9];         /* CostSquareError::ComputeCovariance, row-major */
    lgs_pose2d sensor_pose;       /* Compound(initialPose, relPose) */
    lgs_pose2d best_sensor_pose;
    double cost;                  /* un-normalized final cost */
} lgs_linsolve_summary;

/* One refine; trajectory (may be NULL; room for 4 * max(1, num_iterations_max)
 * doubles) receives, after every OptimizeStep, the sensor pose (x, y, theta)
 * and the cost the convergence test sees at it. */
int  lgs_linsolve_optimize_pose(lgs_ctx* ctx, const lgs_grid* grid, const lgs_linsolve_params* params,
                                const lgs_scan* scan, lgs_pose2d initial_pose,
                                lgs_linsolve_summary* out, double* trajectory);
/* n independent refines against one grid (one workgroup each), one sync */
int  lgs_linsolve_optimize_pose_batch(lgs_ctx* ctx, const lgs_grid* grid,
                                      const lgs_linsolve_params* params,
                                      const lgs_scan* const* scans, const lgs_pose2d* initial_poses,
                                      int n, lgs_linsolve_summary* out);
/* CostSquareError::Cost (C/mapping/cost_function_square_error.cpp:21-58) and,
 * if out_covariance is not NULL, ComputeCovariance (:112-135) at one sensor pose */
int  lgs_cost_square_error(lgs_ctx* ctx, const lgs_grid* grid, double usable_range_min,
                           double usable_range_max, const lgs_scan* scan, lgs_pose2d sensor_pose,
                           double* out_cost, double* out_covariance);

#ifdef __cplusplus
}
#endif

#endif /* LGS_HIP_H */
