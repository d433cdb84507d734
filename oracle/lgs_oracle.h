/*
 * lgs_oracle.h -- CPU restatement of the reference hot path (TEST INFRASTRUCTURE ONLY).
 *
 * This is the parity oracle for the MI355X scan-matching + grid-update hot path.
 * It restates, in plain C, the algorithms of Forrest-Z/my-lidar-graph-slam that
 * sit on the path named by BASELINE.json `north_star`.
 * Every function cites the reference file:line it follows (paths relative to
 * /root/reference; H/ = include/my_lidar_graph_slam/, C/ = src/my_lidar_graph_slam/).
 *
 * Parity status: "parity unpinned".  The reference ships no tests, fixtures or
 * golden vectors, and its hot-path translation units cannot be
 * built in this image without a stand-in for Eigen3 (absent; every TU includes
 * <Eigen/Core> through H/util.hpp:21), which this task forbids.  The oracle is
 * therefore pinned only by hand-traced known-answer tests (tests/golden/) that
 * were derived by executing the reference source text by hand, plus property
 * tests.  See DESIGN.md §Oracle.
 *
 * Who may use this: only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg.  The product path (my-lidar-graph-slam_amd/) never links,
 * loads or calls anything in oracle/.
 *
 * Numerics: compiled with -O2 -ffp-contract=off (no FMA contraction), glibc
 * libm for sin/cos/acos/exp/pow, exactly like the reference's -O3 x86-64 build
 * without -march (R/CMakeLists.txt:33-36).
 */
#ifndef LGS_ORACLE_H
#define LGS_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct { double x, y, theta; } orc_pose;

/* ScanData<double> (H/sensor/sensor_data.hpp:65-158). */
typedef struct {
    const double* ranges;
    const double* angles;
    int n;
    orc_pose rel_sensor_pose;
    double min_range, max_range;
} orc_scan;

/* CostGreedyEndpoint members (C/mapping/cost_function_greedy_endpoint.cpp:10-28).
 * Fields hold the *member* values (mScalingFactor, mStandardDeviation), i.e. after
 * whatever argument order the caller used (SURVEY.md §0 finding 6). */
typedef struct {
    double usable_range_min, usable_range_max;
    double hit_and_missed_dist, occupancy_threshold;
    int kernel_size;
    double scaling_factor;
    double standard_deviation;
} orc_cost_ge;

/* ScanMatcherRealTimeCorrelative ctor args (C/mapping/scan_matcher_real_time_correlative.cpp:14-28). */
typedef struct {
    int low_resolution;
    double range_x, range_y, range_theta;
    double scan_range_max;
} orc_rtcsm_params;

/* Dense view of a GridMapBase<double>: row-major y*w+x, out-of-bounds and
 * unallocated cells read as 0.0 (H/grid_map/grid_map.hpp:858-873). */
typedef struct {
    const double* cells;
    int w, h;
    double min_x, min_y, res;
} orc_grid;

/* ScanMatchingSummary (H/mapping/scan_matcher.hpp:147-174) plus diagnostics. */
typedef struct {
    int pose_found;
    double normalized_cost;
    orc_pose initial_pose;
    orc_pose estimated_pose;
    double covariance[9];          /* row-major 3x3 */
    /* diagnostics */
    double score_max;
    double score_threshold;
    int best_win[3];               /* x, y, theta (window indices) */
    int win[3];
    double steps[3];
    orc_pose sensor_pose;
    orc_pose best_sensor_pose;
    int64_t coarse_evals;          /* number of coarse ComputeScore calls */
    int64_t fine_blocks;           /* number of EvaluateHighResolutionMap calls */
} orc_summary;

/* ---- pose algebra (H/pose.hpp) ---- */
orc_pose orc_compound(orc_pose start, orc_pose diff);              /* :150-161 */
orc_pose orc_inverse_compound(orc_pose start, orc_pose end);       /* :165-180 */
orc_pose orc_move_backward(orc_pose end, orc_pose diff);           /* :195-206 */

/* ---- util (H/util.hpp) ---- */
/* SlidingWindowMax (:198-253) over in[0..n) with stride; reads past n are 0.0 */
void orc_sliding_window_max(const double* in, int in_stride, double* out,
                            int out_stride, int n, int win);
/* Bresenham (:256-303); writes up to cap points (x,y interleaved); returns count */
int orc_bresenham(int x0, int y0, int x1, int y1, int* xy, int cap);

/* ---- grid ---- */
/* PrecomputeGridMap(gridMap, winSize) (C/mapping/grid_map_builder.cpp:518-536) */
void orc_precompute_grid_map(const double* in, int w, int h, int win, double* out);

/* BinaryBayesGridCell::Update (H/grid_map/binary_bayes_grid_cell.hpp:75-92) */
double orc_bayes_update(double value, double prob);

/* ---- correlative matcher ---- */
/* ComputeSearchStep (C/mapping/scan_matcher_real_time_correlative.cpp:156-175) */
void orc_rtcsm_search_step(double res, const orc_scan* scan, double scan_range_max,
                           double* step_x, double* step_y, double* step_theta);
/* ComputeScanIndices (:178-203) for one sensor pose; returns count */
int orc_rtcsm_scan_indices(const orc_grid* g, orc_pose sensor_pose, const orc_scan* scan,
                           double scan_range_max, int* ixy);
/* OptimizePose(gridMap, precompMap, scan, initialPose, thr) const (:50-145) */
int orc_rtcsm_optimize_pose(const orc_grid* grid, const orc_grid* coarse,
                            const orc_rtcsm_params* p, const orc_cost_ge* cost,
                            const orc_scan* scan, orc_pose initial_pose,
                            double normalized_score_threshold, orc_summary* out);
/* OptimizePose(query) (:31-47): precompute + search with DBL_MIN threshold */
int orc_rtcsm_optimize_pose_query(const orc_grid* grid, const orc_rtcsm_params* p,
                                  const orc_cost_ge* cost, const orc_scan* scan,
                                  orc_pose initial_pose, orc_summary* out);
/* Every coarse and fine score of the window in reference iteration order
 * (for kernel-level parity tests): coarse[t][jx][jy], fine[t][xf][yf] with
 * xf,yf over the full fine range [-win, -win + ncoarse*lowres). */
int orc_rtcsm_dense_scores(const orc_grid* grid, const orc_grid* coarse,
                           const orc_rtcsm_params* p, const orc_scan* scan,
                           orc_pose initial_pose, double* coarse_scores,
                           double* fine_scores, int* dims /* win[3], ncx, ncy, nfx, nfy */);

/* ---- cost function (C/mapping/cost_function_greedy_endpoint.cpp) ---- */
double orc_cost_ge_cost(const orc_grid* g, const orc_cost_ge* c, const orc_scan* scan,
                        orc_pose sensor_pose);                               /* :32-111 */
void orc_cost_ge_covariance(const orc_grid* g, const orc_cost_ge* c,
                            const orc_scan* scan, orc_pose sensor_pose,
                            double cov[9]);                                  /* :114-171 */

/* ---- grid map with the reference's patch geometry (H/grid_map/grid_map.hpp) ---- */
typedef struct {
    double res;
    int patch_size;
    int npx, npy;            /* patches */
    int w, h;                /* cells = npx*ps, npy*ps */
    double min_x, min_y;
    double* cells;           /* dense w*h, 0.0 = unknown */
    uint32_t* hit_count;     /* per-cell number of pHit updates (diagnostic) */
    uint32_t* miss_count;    /* per-cell number of pMiss updates (diagnostic) */
    uint8_t* patch_alloc;    /* npx*npy: Patch::IsAllocated (H/grid_map/grid_map_patch.hpp:40) --
                              * set by the first Update of a cell of the patch (GridCellAt :807-823),
                              * moved by Resize (:676-697), kept by Reset (grid_map_patch.hpp:194-203) */
} orc_map;

/* GridMap(res, ps, numCellsX, numCellsY, center) (:337-391) */
int orc_map_init(orc_map* m, double res, int patch_size, int ncx, int ncy,
                 double center_x, double center_y);
void orc_map_free(orc_map* m);
void orc_map_resize(orc_map* m, double min_x, double min_y, double max_x, double max_y); /* :652-711 */
void orc_map_expand(orc_map* m, double min_x, double min_y, double max_x, double max_y,
                    double enlarge_step);                                            /* :714-736 */
void orc_map_reset(orc_map* m);                                                       /* :739-753 */
/* GridMap::ComputeActualMapSize (:969-1015): out[12] = patchIdxMin x,y; patchIdxMax x,y
 * (after the +1 correction); gridCellIdxMin x,y; gridCellIdxMax x,y; mapSizeInPatches x,y;
 * mapSizeInGridCells x,y.  Returns the number of allocated patches (0: the
 * reference's result is undefined -- INT_MAX/INT_MIN bounds -- and out is zeroed). */
int orc_map_actual_size(const orc_map* m, int out[12]);
/* MapSaver::SaveMapCore's image (C/io/map_saver.cpp:413-463) before PNG
 * encoding: DrawMap (:278-317) on a 192-gray canvas of the actual map size,
 * DrawTrajectory (:320-362) of nodes[node_min..node_max] if draw_trajectory,
 * DrawScan (:365-410) of `scan` at scan_pose if scan != NULL, then flipped
 * up-down (:455-462).  rgb receives w*h*3 bytes (w, h = mapSizeInGridCells);
 * returns 0, or 1 if the map has no allocated patch.  Pixels a reference
 * subimage_view would place outside the image are dropped. */
int orc_map_draw_image(const orc_map* m, const orc_pose* node_poses, int n_nodes, int draw_trajectory,
                       int node_min, int node_max, const orc_scan* scan, orc_pose scan_pose,
                       uint8_t* rgb, int* w, int* h);

typedef struct { orc_pose pose; orc_scan scan; } orc_node;

typedef struct {
    double usable_range_min, usable_range_max;
    double prob_hit, prob_miss;
} orc_builder_params;

/* GridMapBuilder::ConstructMapFromScans (C/mapping/grid_map_builder.cpp:227-332) */
int orc_construct_map_from_scans(orc_map* m, const orc_node* nodes, int n_nodes,
                                 const orc_builder_params* bp);
/* Per-scan integration of UpdateGridMap (:149-186): bounding box, Expand, rays */
int orc_integrate_scan(orc_map* m, orc_pose robot_pose, const orc_scan* scan,
                       const orc_builder_params* bp);

/* ---- branch-and-bound matcher (C/mapping/scan_matcher_branch_bound.cpp,
 *      C/mapping/score_function_pixel_accurate.cpp, pyramid
 *      C/mapping/grid_map_builder.cpp:471-495) ---- */
typedef struct {
    int node_height_max;
    double range_x, range_y, range_theta;
    double scan_range_max;
    double score_usable_range_min, score_usable_range_max;   /* ScorePixelAccurate */
} orc_bb_params;

/* ScorePixelAccurate::Score (:19-77): sum of the map values at the hit cells
 * of the beams with range in (max(umin, scan.min), min(umax, scan.max)) */
double orc_pixel_accurate_score(const orc_grid* g, const orc_bb_params* p, const orc_scan* scan,
                                orc_pose sensor_pose);
/* PrecomputeGridMaps (:471-495): maps[h] = window-max map with window 2^h,
 * h = 0..node_height_max; maps must hold node_height_max+1 buffers of w*h */
void orc_precompute_grid_maps(const double* in, int w, int h, int node_height_max, double** maps);
/* ScanMatcherBranchBound::OptimizePose(gridMap, precompMaps, scan, pose, thr)
 * (:47-154): LIFO depth-first branch and bound.  maps[h] (h = 0..H) share the
 * grid's geometry.  out->coarse_evals = nodes scored, out->fine_blocks =
 * leaves accepted; best_win = the best node's (x, y, t). */
int orc_bb_optimize_pose(const orc_grid* grid, const orc_grid* maps, const orc_bb_params* p,
                         const orc_cost_ge* cost, const orc_scan* scan, orc_pose initial_pose,
                         double normalized_score_threshold, orc_summary* out);
/* OptimizePose(query) (:29-44): pyramid, then DBL_MIN threshold */
int orc_bb_optimize_pose_query(const orc_grid* grid, const orc_bb_params* p, const orc_cost_ge* cost,
                               const orc_scan* scan, orc_pose initial_pose, orc_summary* out);

/* ---- Gauss-Newton refine (C/mapping/scan_matcher_linear_solver.cpp, cost_function_square_error.cpp) ---- */
typedef struct {
    int num_iterations_max;
    double convergence_threshold;
    double usable_range_min, usable_range_max;      /* matcher's own */
    double translation_regularizer, rotation_regularizer;
    double cost_usable_range_min, cost_usable_range_max; /* CostSquareError's */
} orc_linsolve_params;

double orc_sq_smoothed_value(const orc_grid* g, double fx, double fy);     /* :276-346 */
double orc_sq_cost(const orc_grid* g, double umin, double umax, const orc_scan* scan,
                   orc_pose sensor_pose);                                   /* :21-58 */
int orc_linsolve_optimize_pose(const orc_grid* g, const orc_linsolve_params* p,
                               const orc_scan* scan, orc_pose initial_pose,
                               orc_summary* out, orc_pose* trajectory /* may be NULL; max_iter sensor poses */);
/* One OptimizeStep (:88-148) from a sensor pose */
orc_pose orc_linsolve_step(const orc_grid* g, const orc_linsolve_params* p, const orc_scan* scan,
                           orc_pose sensor_pose);
/* ComputeCovariance (:112-135) at a sensor pose */
void orc_sq_covariance(const orc_grid* g, double umin, double umax, const orc_scan* scan,
                       orc_pose sensor_pose, double cov[9]);
/* colPivHouseholderQr().solve() restated for 3x3 (Eigen, not vendored) */
void orc_solve3_colpiv_qr(const double H[9], const double b[3], double x[3]);

/* ---- ScanInterpolator::Interpolate (C/mapping/scan_interpolator.cpp:9-98) ----
 * n >= 1 input beams; writes at most cap output beams (range, angle) and
 * returns the number the reference produces (may exceed cap: call again). */
int orc_scan_interpolate(const double* ranges, const double* angles, int n, double dist_scans,
                         double dist_threshold_empty, double* out_ranges, double* out_angles, int cap);

#ifdef __cplusplus
}
#endif

#endif /* LGS_ORACLE_H */
