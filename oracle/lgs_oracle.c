/*
 * lgs_oracle.c -- CPU restatement of the reference hot path (TEST INFRASTRUCTURE ONLY).
 *
 * Parity unpinned: see lgs_oracle.h and DESIGN.md §Oracle.  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this code.
 *
 * Each function restates the reference loop in the reference's own order of
 * floating-point operations (left-to-right association as written in the C++
 * source), so that with -ffp-contract=off and glibc libm the results are the
 * ones the reference computes.  Citations: H/ = include/my_lidar_graph_slam/,
 * C/ = src/my_lidar_graph_slam/ under /root/reference.
 *
 * sin/cos: the reference is built with GCC -O3, which fuses a sin(x)/cos(x)
 * pair into one glibc sincos() call; sincos differs from separate sin/cos in
 * ~0.1% of inputs (last ulp), so every paired site here calls sincos().
 */
#define _GNU_SOURCE 1
#include "lgs_oracle.h"

#include <float.h>
#include <limits.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------ */
/* small helpers mirroring std::min / std::max / std::clamp exactly    */
/* ------------------------------------------------------------------ */
static inline double std_min(double a, double b) { return (b < a) ? b : a; }
static inline double std_max(double a, double b) { return (a < b) ? b : a; }
static inline int imin(int a, int b) { return (b < a) ? b : a; }
static inline int imax(int a, int b) { return (a < b) ? b : a; }
static inline double std_clamp(double v, double lo, double hi)
{
    return (v < lo) ? lo : (hi < v) ? hi : v;
}
static inline int iclamp(int v, int lo, int hi) { return (v < lo) ? lo : (hi < v) ? hi : v; }

/* GridMap::Value(x, y, default) on a dense view (H/grid_map/grid_map.hpp:858-873,
 * H/grid_map/grid_map_patch.hpp:180-190): outside -> default, else cell. */
static inline double grid_value(const orc_grid* g, int x, int y)
{
    if (!(x >= 0 && x < g->w && y >= 0 && y < g->h))
        return 0.0;
    return g->cells[(size_t)y * (size_t)g->w + (size_t)x];
}

/* WorldCoordinateToGridCellIndex (H/grid_map/grid_map.hpp:779-790) */
static inline void world_to_cell(double min_x, double min_y, double res,
                                 double mx, double my, int* ix, int* iy)
{
    *ix = (int)floor((mx - min_x) / res);
    *iy = (int)floor((my - min_y) / res);
}

/* ------------------------------------------------------------------ */
/* pose algebra (H/pose.hpp)                                           */
/* ------------------------------------------------------------------ */
orc_pose orc_compound(orc_pose s, orc_pose d)
{
    /* H/pose.hpp:150-161 */
    double sinT, cosT;
    sincos(s.theta, &sinT, &cosT);
    orc_pose r;
    r.x = cosT * d.x - sinT * d.y + s.x;
    r.y = sinT * d.x + cosT * d.y + s.y;
    r.theta = s.theta + d.theta;
    return r;
}

orc_pose orc_inverse_compound(orc_pose s, orc_pose e)
{
    /* H/pose.hpp:165-180 */
    double sinT, cosT;
    sincos(s.theta, &sinT, &cosT);
    double dx = e.x - s.x;
    double dy = e.y - s.y;
    double dt = e.theta - s.theta;
    orc_pose r;
    r.x = cosT * dx + sinT * dy;
    r.y = -sinT * dx + cosT * dy;
    r.theta = dt;
    return r;
}

orc_pose orc_move_backward(orc_pose e, orc_pose d)
{
    /* H/pose.hpp:195-206 */
    double theta = e.theta - d.theta;
    double sinT, cosT;
    sincos(theta, &sinT, &cosT);
    orc_pose r;
    r.x = e.x - cosT * d.x + sinT * d.y;
    r.y = e.y - sinT * d.x - cosT * d.y;
    r.theta = theta;
    return r;
}

/* ------------------------------------------------------------------ */
/* SlidingWindowMax (H/util.hpp:198-253), deque restated on an array   */
/* ------------------------------------------------------------------ */
void orc_sliding_window_max(const double* in, int in_stride, double* out,
                            int out_stride, int n, int win)
{
    /* inFunc(i) = GridMap::Value(.., i, unknown) -> 0.0 past the end */
#define IN(i) (((i) < n) ? in[(size_t)(i) * (size_t)in_stride] : 0.0)
    int cap = n + win + 1;
    int* q = (int*)malloc(sizeof(int) * (size_t)cap);
    int head = 0, tail = 0; /* [head, tail) */
    int idxIn = 0, idxOut = 0;

    for (idxIn = 0; idxIn < win; ++idxIn) {
        while (tail > head && IN(idxIn) >= IN(q[tail - 1]))
            --tail;
        q[tail++] = idxIn;
    }
    for (; idxIn < n; ++idxIn) {
        out[(size_t)(idxOut++) * (size_t)out_stride] = IN(q[head]);
        while (tail > head && q[head] <= idxIn - win)
            ++head;
        while (tail > head && IN(idxIn) >= IN(q[tail - 1]))
            --tail;
        q[tail++] = idxIn;
    }
    for (; idxOut < n; ++idxOut)
        out[(size_t)idxOut * (size_t)out_stride] = IN(q[head]);
    free(q);
#undef IN
}

/* PrecomputeGridMap (C/mapping/grid_map_builder.cpp:518-536):
 * SlidingWindowMaxRow (:403-434, slides along y for every column x) then
 * SlidingWindowMaxCol (:437-468, slides along x for every row y).  The
 * "write only if allocated or != unknown" condition (:424-425, :458-459)
 * does not change any value read back, so the dense restatement writes all. */
void orc_precompute_grid_map(const double* in, int w, int h, int win, double* out)
{
    double* tmp = (double*)calloc((size_t)w * (size_t)h + 1, sizeof(double));
    for (int x = 0; x < w; ++x)
        orc_sliding_window_max(in + x, w, tmp + x, w, h, win);
    for (int y = 0; y < h; ++y)
        orc_sliding_window_max(tmp + (size_t)y * w, 1, out + (size_t)y * w, 1, w, win);
    free(tmp);
}

/* ------------------------------------------------------------------ */
/* Bresenham (H/util.hpp:256-303)                                      */
/* ------------------------------------------------------------------ */
int orc_bresenham(int x0, int y0, int x1, int y1, int* xy, int cap)
{
    int n = 0;
    int deltaX = x1 - x0;
    int deltaY = y1 - y0;
    int stepX = (deltaX < 0) ? -1 : 1;
    int stepY = (deltaY < 0) ? -1 : 1;
    int nextX = x0;
    int nextY = y0;
#define EMIT(a, b) do { if (n < cap) { xy[2 * n] = (a); xy[2 * n + 1] = (b); } ++n; } while (0)
    deltaX = abs(deltaX * 2);
    deltaY = abs(deltaY * 2);
    EMIT(nextX, nextY);
    if (deltaX > deltaY) {
        int err = deltaY - deltaX / 2;
        while (nextX != x1) {
            if (err >= 0) {
                nextY += stepY;
                err -= deltaX;
            }
            nextX += stepX;
            err += deltaY;
            EMIT(nextX, nextY);
        }
    } else {
        int err = deltaX - deltaY / 2;
        while (nextY != y1) {
            if (err >= 0) {
                nextX += stepX;
                err -= deltaY;
            }
            nextY += stepY;
            err += deltaX;
            EMIT(nextX, nextY);
        }
    }
#undef EMIT
    return n;
}

/* ------------------------------------------------------------------ */
/* BinaryBayesGridCell (H/grid_map/binary_bayes_grid_cell.hpp)         */
/* ------------------------------------------------------------------ */
#define ORC_PMIN 1e-3
#define ORC_PMAX (1.0 - ORC_PMIN)

static inline double bayes_clamp(double p) { return std_clamp(p, ORC_PMIN, ORC_PMAX); } /* :96-100 */
static inline double bayes_odds(double p)                                               /* :103-112 */
{
    const double c = bayes_clamp(p);
    return c / (1.0 - c);
}
static inline double bayes_value(double o) { return bayes_clamp(o / (1.0 + o)); }     /* :115-119 */

double orc_bayes_update(double v, double p)
{
    /* :75-92 */
    if (v == 0.0)
        return bayes_clamp(p);
    const double oldOdds = bayes_odds(v);
    const double valueOdds = bayes_odds(p);
    const double newValue = bayes_value(oldOdds * valueOdds);
    return bayes_clamp(newValue);
}

/* ------------------------------------------------------------------ */
/* Correlative matcher (C/mapping/scan_matcher_real_time_correlative.cpp) */
/* ------------------------------------------------------------------ */
void orc_rtcsm_search_step(double res, const orc_scan* scan, double scan_range_max,
                           double* step_x, double* step_y, double* step_theta)
{
    /* :156-175; std::max_element returns the first maximum */
    double mr = scan->ranges[0];
    for (int i = 1; i < scan->n; ++i)
        if (mr < scan->ranges[i])
            mr = scan->ranges[i];
    const double maxRange = std_min(mr, scan_range_max);
    const double theta = res / maxRange;
    *step_x = res;
    *step_y = res;
    *step_theta = acos(1.0 - 0.5 * theta * theta);
}

int orc_rtcsm_scan_indices(const orc_grid* g, orc_pose sp, const orc_scan* scan,
                           double scan_range_max, int* ixy)
{
    /* :178-203 with ScanData::HitPoint (H/sensor/sensor_data.hpp:162-173) */
    int n = 0;
    for (int i = 0; i < scan->n; ++i) {
        const double range = scan->ranges[i];
        if (range >= scan_range_max)
            continue;
        double sinT, cosT;
        sincos(sp.theta + scan->angles[i], &sinT, &cosT);
        const double hx = sp.x + range * cosT;
        const double hy = sp.y + range * sinT;
        world_to_cell(g->min_x, g->min_y, g->res, hx, hy, &ixy[2 * n], &ixy[2 * n + 1]);
        ++n;
    }
    return n;
}

/* ComputeScore (:207-224): sequential fp64 sum in beam order */
static double rtcsm_score(const orc_grid* g, const int* ixy, int n, int ox, int oy)
{
    double sum = 0.0;
    for (int i = 0; i < n; ++i)
        sum += grid_value(g, ixy[2 * i] + ox, ixy[2 * i + 1] + oy);
    return sum;
}

int orc_rtcsm_optimize_pose(const orc_grid* grid, const orc_grid* coarse,
                            const orc_rtcsm_params* p, const orc_cost_ge* cost,
                            const orc_scan* scan, orc_pose initial_pose,
                            double normalized_score_threshold, orc_summary* out)
{
    memset(out, 0, sizeof(*out));
    if (scan->n <= 0)
        return 1;
    /* :58-59 */
    const orc_pose sensorPose = orc_compound(initial_pose, scan->rel_sensor_pose);
    /* :62-65 */
    double stepX, stepY, stepTheta;
    orc_rtcsm_search_step(grid->res, scan, p->scan_range_max, &stepX, &stepY, &stepTheta);
    /* :69-74 */
    const int winX = (int)ceil(0.5 * p->range_x / stepX);
    const int winY = (int)ceil(0.5 * p->range_y / stepY);
    const int winTheta = (int)ceil(0.5 * p->range_theta / stepTheta);
    /* :77-82 */
    const double scoreThreshold = normalized_score_threshold * (double)scan->n;
    double scoreMax = scoreThreshold;
    int bestWinX = -winX, bestWinY = -winY, bestWinTheta = -winTheta;

    int* idx = (int*)malloc(sizeof(int) * 2 * (size_t)scan->n);
    int64_t coarseEvals = 0, fineBlocks = 0;
    const int lowRes = p->low_resolution;

    /* :88-116 */
    for (int t = -winTheta; t <= winTheta; ++t) {
        orc_pose cur = sensorPose;
        cur.theta = sensorPose.theta + stepTheta * t;
        const int nIdx = orc_rtcsm_scan_indices(coarse, cur, scan, p->scan_range_max, idx);
        for (int x = -winX; x <= winX; x += lowRes) {
            for (int y = -winY; y <= winY; y += lowRes) {
                const double score = rtcsm_score(coarse, idx, nIdx, x, y);
                ++coarseEvals;
                if (score <= scoreMax)
                    continue;
                /* EvaluateHighResolutionMap (:227-256) */
                ++fineBlocks;
                for (int xf = x; xf < x + lowRes; ++xf) {
                    for (int yf = y; yf < y + lowRes; ++yf) {
                        const double s = rtcsm_score(grid, idx, nIdx, xf, yf);
                        if (scoreMax < s) {
                            scoreMax = s;
                            bestWinX = xf;
                            bestWinY = yf;
                            bestWinTheta = t;
                        }
                    }
                }
            }
        }
    }
    free(idx);

    /* :120-125 */
    const int poseFound = scoreMax > scoreThreshold;
    orc_pose best;
    best.x = sensorPose.x + bestWinX * stepX;
    best.y = sensorPose.y + bestWinY * stepY;
    best.theta = sensorPose.theta + bestWinTheta * stepTheta;

    /* :128-138 */
    const double costVal = orc_cost_ge_cost(grid, cost, scan, best);
    out->normalized_cost = costVal / (double)scan->n;
    out->estimated_pose = orc_move_backward(best, scan->rel_sensor_pose);
    orc_cost_ge_covariance(grid, cost, scan, best, out->covariance);

    out->pose_found = poseFound;
    out->initial_pose = initial_pose;
    out->score_max = scoreMax;
    out->score_threshold = scoreThreshold;
    out->best_win[0] = bestWinX;
    out->best_win[1] = bestWinY;
    out->best_win[2] = bestWinTheta;
    out->win[0] = winX;
    out->win[1] = winY;
    out->win[2] = winTheta;
    out->steps[0] = stepX;
    out->steps[1] = stepY;
    out->steps[2] = stepTheta;
    out->sensor_pose = sensorPose;
    out->best_sensor_pose = best;
    out->coarse_evals = coarseEvals;
    out->fine_blocks = fineBlocks;
    return 0;
}

int orc_rtcsm_optimize_pose_query(const orc_grid* grid, const orc_rtcsm_params* p,
                                  const orc_cost_ge* cost, const orc_scan* scan,
                                  orc_pose initial_pose, orc_summary* out)
{
    /* :31-47: ComputeCoarserMap (:148-153) then search with DBL_MIN */
    double* c = (double*)calloc((size_t)grid->w * (size_t)grid->h + 1, sizeof(double));
    orc_precompute_grid_map(grid->cells, grid->w, grid->h, p->low_resolution, c);
    orc_grid cg = *grid;
    cg.cells = c;
    int rc = orc_rtcsm_optimize_pose(grid, &cg, p, cost, scan, initial_pose, DBL_MIN, out);
    free(c);
    return rc;
}

/* ------------------------------------------------------------------ */
/* branch-and-bound matcher                                             */
/* ------------------------------------------------------------------ */
double orc_pixel_accurate_score(const orc_grid* g, const orc_bb_params* p, const orc_scan* scan,
                                orc_pose sp)
{
    /* C/mapping/score_function_pixel_accurate.cpp:19-77 */
    double sumScore = 0.0;
    const double minRange = std_max(p->score_usable_range_min, scan->min_range);
    const double maxRange = std_min(p->score_usable_range_max, scan->max_range);
    for (int i = 0; i < scan->n; ++i) {
        const double scanRange = scan->ranges[i];
        if (scanRange >= maxRange || scanRange <= minRange)
            continue;
        /* ScanData::HitPoint (H/sensor/sensor_data.hpp:162-173), cos/sin fused */
        double sinT, cosT;
        sincos(sp.theta + scan->angles[i], &sinT, &cosT);
        const double hx = sp.x + scanRange * cosT;
        const double hy = sp.y + scanRange * sinT;
        int ix, iy;
        world_to_cell(g->min_x, g->min_y, g->res, hx, hy, &ix, &iy);
        const double v = grid_value(g, ix, iy);
        if (v == 0.0)     /* unknown: skipped (:55-56) */
            continue;
        sumScore += v;
    }
    return sumScore;
}

void orc_precompute_grid_maps(const double* in, int w, int h, int node_height_max, double** maps)
{
    /* C/mapping/grid_map_builder.cpp:471-495: window 1, 2, 4, ..., 2^H */
    for (int nodeHeight = 0, winSize = 1; nodeHeight <= node_height_max; ++nodeHeight, winSize <<= 1)
        orc_precompute_grid_map(in, w, h, winSize, maps[nodeHeight]);
}

typedef struct { int x, y, t, h; } bb_node;

int orc_bb_optimize_pose(const orc_grid* grid, const orc_grid* maps, const orc_bb_params* p,
                         const orc_cost_ge* cost, const orc_scan* scan, orc_pose initial_pose,
                         double normalized_score_threshold, orc_summary* out)
{
    memset(out, 0, sizeof(*out));
    if (scan->n <= 0)
        return 1;
    /* :54-56 */
    const orc_pose sensorPose = orc_compound(initial_pose, scan->rel_sensor_pose);
    /* :59-62 ComputeSearchStep (:178-198), identical to the RTCSM one */
    double stepX, stepY, stepTheta;
    orc_rtcsm_search_step(grid->res, scan, p->scan_range_max, &stepX, &stepY, &stepTheta);
    /* :65-70 */
    const int winX = (int)ceil(0.5 * p->range_x / stepX);
    const int winY = (int)ceil(0.5 * p->range_y / stepY);
    const int winTheta = (int)ceil(0.5 * p->range_theta / stepTheta);
    /* :73-78 */
    const double scoreThreshold = normalized_score_threshold * (double)scan->n;
    double scoreMax = scoreThreshold;
    orc_pose bestSensorPose = sensorPose;
    int best[3] = { 0, 0, 0 };
    /* :81-88 stack of nodes covering the window (x outer, y, t inner) */
    const int winSizeMax = 1 << p->node_height_max;
    size_t cap = 1024, top = 0;
    bb_node* st = (bb_node*)malloc(sizeof(bb_node) * cap);
    for (int x = -winX; x <= winX; x += winSizeMax)
        for (int y = -winY; y <= winY; y += winSizeMax)
            for (int t = -winTheta; t <= winTheta; ++t) {
                if (top == cap) {
                    cap *= 2;
                    st = (bb_node*)realloc(st, sizeof(bb_node) * cap);
                }
                st[top].x = x;
                st[top].y = y;
                st[top].t = t;
                st[top].h = p->node_height_max;
                ++top;
            }
    int64_t nodes = 0, accepted = 0;
    /* :92-140 */
    while (top > 0) {
        const bb_node cur = st[top - 1];
        orc_pose nodePose;
        nodePose.x = sensorPose.x + cur.x * stepX;
        nodePose.y = sensorPose.y + cur.y * stepY;
        nodePose.theta = sensorPose.theta + cur.t * stepTheta;
        const double score = orc_pixel_accurate_score(&maps[cur.h], p, scan, nodePose);
        ++nodes;
        if (score <= scoreMax) {   /* :105-109 */
            --top;
            continue;
        }
        if (cur.h == 0) {          /* :112-119 leaf */
            --top;
            bestSensorPose = nodePose;
            scoreMax = score;
            best[0] = cur.x;
            best[1] = cur.y;
            best[2] = cur.t;
            ++accepted;
        } else {                   /* :120-137 four children, pushed in this order */
            const int h = cur.h - 1, ws = 1 << h;
            --top;
            if (top + 4 > cap) {
                cap *= 2;
                st = (bb_node*)realloc(st, sizeof(bb_node) * cap);
            }
            const bb_node c[4] = { { cur.x, cur.y, cur.t, h }, { cur.x + ws, cur.y, cur.t, h },
                                   { cur.x, cur.y + ws, cur.t, h }, { cur.x + ws, cur.y + ws, cur.t, h } };
            for (int k = 0; k < 4; ++k)
                st[top++] = c[k];
        }
    }
    free(st);
    /* :142-153 */
    const int poseFound = scoreMax > scoreThreshold;
    const double costVal = orc_cost_ge_cost(grid, cost, scan, bestSensorPose);
    out->normalized_cost = costVal / (double)scan->n;
    out->estimated_pose = orc_move_backward(bestSensorPose, scan->rel_sensor_pose);
    orc_cost_ge_covariance(grid, cost, scan, bestSensorPose, out->covariance);
    out->pose_found = poseFound;
    out->initial_pose = initial_pose;
    out->score_max = scoreMax;
    out->score_threshold = scoreThreshold;
    out->best_win[0] = best[0];
    out->best_win[1] = best[1];
    out->best_win[2] = best[2];
    out->win[0] = winX;
    out->win[1] = winY;
    out->win[2] = winTheta;
    out->steps[0] = stepX;
    out->steps[1] = stepY;
    out->steps[2] = stepTheta;
    out->sensor_pose = sensorPose;
    out->best_sensor_pose = bestSensorPose;
    out->coarse_evals = nodes;
    out->fine_blocks = accepted;
    return 0;
}

int orc_bb_optimize_pose_query(const orc_grid* grid, const orc_bb_params* p, const orc_cost_ge* cost,
                               const orc_scan* scan, orc_pose initial_pose, orc_summary* out)
{
    /* :29-44: ComputeCoarserMaps (:157-165) then DBL_MIN */
    const int H = p->node_height_max;
    double** bufs = (double**)malloc(sizeof(double*) * (size_t)(H + 1));
    orc_grid* maps = (orc_grid*)malloc(sizeof(orc_grid) * (size_t)(H + 1));
    for (int h = 0; h <= H; ++h) {
        bufs[h] = (double*)calloc((size_t)grid->w * (size_t)grid->h + 1, sizeof(double));
        maps[h] = *grid;
        maps[h].cells = bufs[h];
    }
    orc_precompute_grid_maps(grid->cells, grid->w, grid->h, H, bufs);
    const int rc = orc_bb_optimize_pose(grid, maps, p, cost, scan, initial_pose, DBL_MIN, out);
    for (int h = 0; h <= H; ++h)
        free(bufs[h]);
    free(bufs);
    free(maps);
    return rc;
}

int orc_rtcsm_dense_scores(const orc_grid* grid, const orc_grid* coarse,
                           const orc_rtcsm_params* p, const orc_scan* scan,
                           orc_pose initial_pose, double* coarse_scores,
                           double* fine_scores, int* dims)
{
    const orc_pose sensorPose = orc_compound(initial_pose, scan->rel_sensor_pose);
    double stepX, stepY, stepTheta;
    orc_rtcsm_search_step(grid->res, scan, p->scan_range_max, &stepX, &stepY, &stepTheta);
    const int winX = (int)ceil(0.5 * p->range_x / stepX);
    const int winY = (int)ceil(0.5 * p->range_y / stepY);
    const int winTheta = (int)ceil(0.5 * p->range_theta / stepTheta);
    const int lowRes = p->low_resolution;
    const int ncx = (2 * winX) / lowRes + 1;
    const int ncy = (2 * winY) / lowRes + 1;
    const int nfx = ncx * lowRes, nfy = ncy * lowRes;
    if (dims) {
        dims[0] = winX; dims[1] = winY; dims[2] = winTheta;
        dims[3] = ncx; dims[4] = ncy; dims[5] = nfx; dims[6] = nfy;
    }
    if (!coarse_scores && !fine_scores)
        return 0;
    int* idx = (int*)malloc(sizeof(int) * 2 * (size_t)scan->n);
    for (int t = -winTheta; t <= winTheta; ++t) {
        orc_pose cur = sensorPose;
        cur.theta = sensorPose.theta + stepTheta * t;
        const int nIdx = orc_rtcsm_scan_indices(coarse, cur, scan, p->scan_range_max, idx);
        const size_t ti = (size_t)(t + winTheta);
        if (coarse_scores)
            for (int jx = 0; jx < ncx; ++jx)
                for (int jy = 0; jy < ncy; ++jy)
                    coarse_scores[(ti * ncx + jx) * ncy + jy] =
                        rtcsm_score(coarse, idx, nIdx, -winX + jx * lowRes, -winY + jy * lowRes);
        if (fine_scores)
            for (int fx = 0; fx < nfx; ++fx)
                for (int fy = 0; fy < nfy; ++fy)
                    fine_scores[(ti * nfx + fx) * nfy + fy] =
                        rtcsm_score(grid, idx, nIdx, -winX + fx, -winY + fy);
    }
    free(idx);
    return 0;
}

/* ------------------------------------------------------------------ */
/* CostGreedyEndpoint (C/mapping/cost_function_greedy_endpoint.cpp)     */
/* ------------------------------------------------------------------ */
static inline double sq_dist_cells(double res, int x0, int y0, int x1, int y1)
{
    /* GridMap::SquaredDistance (H/grid_map/grid_map.hpp:894-902) */
    const double dX = (x1 - x0) * res;
    const double dY = (y1 - y0) * res;
    return dX * dX + dY * dY;
}

double orc_cost_ge_cost(const orc_grid* g, const orc_cost_ge* c, const orc_scan* scan,
                        orc_pose sp)
{
    /* :32-111 */
    double costValue = 0.0;
    const double minRange = std_max(c->usable_range_min, scan->min_range);
    const double maxRange = std_min(c->usable_range_max, scan->max_range);
    const double variance = c->standard_deviation * c->standard_deviation;
    const int K = c->kernel_size;

    for (int i = 0; i < scan->n; ++i) {
        const double scanRange = scan->ranges[i];
        if (scanRange >= maxRange || scanRange <= minRange)
            continue;
        /* HitAndMissedPoint (H/sensor/sensor_data.hpp:177-198) */
        double sinT, cosT;
        sincos(sp.theta + scan->angles[i], &sinT, &cosT);
        const double hx = sp.x + scanRange * cosT;
        const double hy = sp.y + scanRange * sinT;
        const double mx = sp.x + (scanRange - c->hit_and_missed_dist) * cosT;
        const double my = sp.y + (scanRange - c->hit_and_missed_dist) * sinT;
        int hix, hiy, mix, miy;
        world_to_cell(g->min_x, g->min_y, g->res, hx, hy, &hix, &hiy);
        world_to_cell(g->min_x, g->min_y, g->res, mx, my, &mix, &miy);

        double minSq = sq_dist_cells(g->res, 0, 0, K + 1, K + 1);
        for (int ky = -K; ky <= K; ++ky) {
            for (int kx = -K; kx <= K; ++kx) {
                const double hv = grid_value(g, hix + kx, hiy + ky);
                const double mv = grid_value(g, mix + kx, miy + ky);
                if (hv == 0.0 || mv == 0.0)
                    continue;
                if (hv < c->occupancy_threshold || mv > c->occupancy_threshold)
                    continue;
                const double sq = sq_dist_cells(g->res, hix, hiy, hix + kx, hiy + ky);
                minSq = std_min(sq, minSq);
            }
        }
        costValue -= exp(-0.5 * minSq / variance);
    }
    costValue *= c->scaling_factor;
    return costValue;
}

void orc_cost_ge_covariance(const orc_grid* g, const orc_cost_ge* c, const orc_scan* scan,
                            orc_pose sp, double cov[9])
{
    /* ComputeGradient (:114-144) then ComputeCovariance (:147-171) */
    const double diffLinear = g->res;
    const double diffAngular = 1e-2;
    orc_pose px = sp, mx = sp, py = sp, my = sp, pt = sp, mt = sp;
    px.x = sp.x + diffLinear; px.y = sp.y + 0.0; px.theta = sp.theta + 0.0;
    mx.x = sp.x - diffLinear; mx.y = sp.y - 0.0; mx.theta = sp.theta - 0.0;
    py.x = sp.x + 0.0; py.y = sp.y + diffLinear; py.theta = sp.theta + 0.0;
    my.x = sp.x - 0.0; my.y = sp.y - diffLinear; my.theta = sp.theta - 0.0;
    pt.x = sp.x + 0.0; pt.y = sp.y + 0.0; pt.theta = sp.theta + diffAngular;
    mt.x = sp.x - 0.0; mt.y = sp.y - 0.0; mt.theta = sp.theta - diffAngular;
    const double dX = orc_cost_ge_cost(g, c, scan, px) - orc_cost_ge_cost(g, c, scan, mx);
    const double dY = orc_cost_ge_cost(g, c, scan, py) - orc_cost_ge_cost(g, c, scan, my);
    const double dT = orc_cost_ge_cost(g, c, scan, pt) - orc_cost_ge_cost(g, c, scan, mt);
    const double gv[3] = { 0.5 * dX / diffLinear, 0.5 * dY / diffLinear, 0.5 * dT / diffAngular };
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j)
            cov[3 * i + j] = gv[i] * gv[j];
    cov[0] += 0.01;
    cov[4] += 0.01;
    cov[8] += 0.01;
}

/* ------------------------------------------------------------------ */
/* GridMap geometry (H/grid_map/grid_map.hpp)                          */
/* ------------------------------------------------------------------ */
static inline int cell_to_patch(int idx, int ps)
{
    /* GridCellIndexToPatchIndex (:905-915), including the off-by-one at
     * exact negative multiples */
    return (idx < 0) ? (idx / ps - 1) : (idx / ps);
}

int orc_map_init(orc_map* m, double res, int ps, int ncx, int ncy, double cx, double cy)
{
    /* :337-391 */
    memset(m, 0, sizeof(*m));
    m->res = res;
    m->patch_size = ps;
    ncx = imax(0, ncx);
    ncy = imax(0, ncy);
    m->npx = (int)ceil((double)ncx / (double)ps);
    m->npy = (int)ceil((double)ncy / (double)ps);
    m->w = m->npx * ps;
    m->h = m->npy * ps;
    const double offX = (m->w % 2 == 0) ? (double)(m->w / 2) : ((double)(m->w / 2) + 0.5);
    const double offY = (m->h % 2 == 0) ? (double)(m->h / 2) : ((double)(m->h / 2) + 0.5);
    m->min_x = cx - offX * res;
    m->min_y = cy - offY * res;
    const size_t n = (size_t)m->w * (size_t)m->h;
    m->cells = (double*)calloc(n + 1, sizeof(double));
    m->hit_count = (uint32_t*)calloc(n + 1, sizeof(uint32_t));
    m->miss_count = (uint32_t*)calloc(n + 1, sizeof(uint32_t));
    m->patch_alloc = (uint8_t*)calloc((size_t)m->npx * (size_t)m->npy + 1, 1);
    return (m->cells && m->hit_count && m->miss_count && m->patch_alloc) ? 0 : 1;
}

void orc_map_free(orc_map* m)
{
    free(m->cells);
    free(m->hit_count);
    free(m->miss_count);
    free(m->patch_alloc);
    memset(m, 0, sizeof(*m));
}

void orc_map_resize(orc_map* m, double minX, double minY, double maxX, double maxY)
{
    /* :652-711 */
    int cminx, cminy, cmaxx, cmaxy;
    world_to_cell(m->min_x, m->min_y, m->res, minX, minY, &cminx, &cminy);
    world_to_cell(m->min_x, m->min_y, m->res, maxX, maxY, &cmaxx, &cmaxy);
    const int ps = m->patch_size;
    const int pminx = cell_to_patch(cminx, ps), pminy = cell_to_patch(cminy, ps);
    const int pmaxx = cell_to_patch(cmaxx, ps), pmaxy = cell_to_patch(cmaxy, ps);
    const int npx = imax(0, pmaxx - pminx + 1);
    const int npy = imax(0, pmaxy - pminy + 1);
    const int nw = npx * ps, nh = npy * ps;
    const size_t n = (size_t)nw * (size_t)nh;
    double* cells = (double*)calloc(n + 1, sizeof(double));
    uint32_t* hc = (uint32_t*)calloc(n + 1, sizeof(uint32_t));
    uint32_t* mc = (uint32_t*)calloc(n + 1, sizeof(uint32_t));
    uint8_t* pa = (uint8_t*)calloc((size_t)npx * (size_t)npy + 1, 1);

    const int x0 = imax(0, pminx), y0 = imax(0, pminy);
    const int x1 = imin(m->npx, pmaxx + 1), y1 = imin(m->npy, pmaxy + 1);
    for (int py = y0; py < y1; ++py) {
        for (int px = x0; px < x1; ++px) {
            pa[(size_t)(py - pminy) * npx + (px - pminx)] = m->patch_alloc[(size_t)py * m->npx + px];
            const int nx = (px - pminx) * ps, ny = (py - pminy) * ps;
            const int ox = px * ps, oy = py * ps;
            for (int yy = 0; yy < ps; ++yy) {
                const size_t src = (size_t)(oy + yy) * m->w + ox;
                const size_t dst = (size_t)(ny + yy) * nw + nx;
                memcpy(cells + dst, m->cells + src, sizeof(double) * ps);
                memcpy(hc + dst, m->hit_count + src, sizeof(uint32_t) * ps);
                memcpy(mc + dst, m->miss_count + src, sizeof(uint32_t) * ps);
            }
        }
    }
    free(m->cells);
    free(m->hit_count);
    free(m->miss_count);
    free(m->patch_alloc);
    m->cells = cells;
    m->hit_count = hc;
    m->miss_count = mc;
    m->patch_alloc = pa;
    m->npx = npx;
    m->npy = npy;
    m->w = nw;
    m->h = nh;
    m->min_x += (pminx * ps) * m->res;
    m->min_y += (pminy * ps) * m->res;
}

static inline int map_is_inside_world(const orc_map* m, double x, double y)
{
    int ix, iy;
    world_to_cell(m->min_x, m->min_y, m->res, x, y, &ix, &iy);
    return (ix >= 0 && ix < m->w) && (iy >= 0 && iy < m->h);
}

void orc_map_expand(orc_map* m, double minX, double minY, double maxX, double maxY,
                    double enlargeStep)
{
    /* :714-736 */
    if (map_is_inside_world(m, minX, minY) && map_is_inside_world(m, maxX, maxY))
        return;
    double minPX = m->min_x + m->res * 0, minPY = m->min_y + m->res * 0;
    double maxPX = m->min_x + m->res * m->w, maxPY = m->min_y + m->res * m->h;
    minPX = (minX < minPX) ? minX - enlargeStep : minPX;
    minPY = (minY < minPY) ? minY - enlargeStep : minPY;
    maxPX = (maxX > maxPX) ? maxX + enlargeStep : maxPX;
    maxPY = (maxY > maxPY) ? maxY + enlargeStep : maxPY;
    orc_map_resize(m, minPX, minPY, maxPX, maxPY);
}

void orc_map_reset(orc_map* m)
{
    /* :739-753 (and the per-cell diagnostic counters) */
    const size_t n = (size_t)m->w * (size_t)m->h;
    memset(m->cells, 0, n * sizeof(double));
    memset(m->hit_count, 0, n * sizeof(uint32_t));
    memset(m->miss_count, 0, n * sizeof(uint32_t));
}

int orc_map_actual_size(const orc_map* m, int out[12])
{
    /* GridMap::ComputeActualMapSize (H/grid_map/grid_map.hpp:969-1015) */
    int pminx = INT_MAX, pminy = INT_MAX, pmaxx = INT_MIN, pmaxy = INT_MIN, n = 0;
    for (int y = 0; y < m->npy; ++y)
        for (int x = 0; x < m->npx; ++x) {
            if (!m->patch_alloc[(size_t)y * m->npx + x])
                continue;
            ++n;
            pminx = imin(pminx, x);
            pminy = imin(pminy, y);
            pmaxx = imax(pmaxx, x);
            pmaxy = imax(pmaxy, y);
        }
    memset(out, 0, sizeof(int) * 12);
    if (n == 0)
        return 0;
    const int ps = m->patch_size;
    /* PatchIndexToGridCellIndexRange (:918-929): min corner of the min patch,
     * max corner (exclusive) of the max patch */
    out[4] = pminx * ps;
    out[5] = pminy * ps;
    out[6] = pmaxx * ps + ps;
    out[7] = pmaxy * ps + ps;
    out[0] = pminx;
    out[1] = pminy;
    out[2] = pmaxx + 1;
    out[3] = pmaxy + 1;
    out[8] = out[2] - out[0];
    out[9] = out[3] - out[1];
    out[10] = out[6] - out[4];
    out[11] = out[7] - out[5];
    return n;
}

/* gil::fill_pixels(subimage_view(view, x, y, s, s), px): an s x s block
 * (pixels outside the image are dropped) */
static void fill_block(uint8_t* rgb, int w, int h, int x, int y, int s, uint8_t r, uint8_t g, uint8_t b)
{
    for (int yy = y; yy < y + s; ++yy)
        for (int xx = x; xx < x + s; ++xx) {
            if (xx < 0 || xx >= w || yy < 0 || yy >= h)
                continue;
            uint8_t* p = rgb + 3 * ((size_t)yy * w + xx);
            p[0] = r;
            p[1] = g;
            p[2] = b;
        }
}

int orc_map_draw_image(const orc_map* m, const orc_pose* nodes, int n_nodes, int draw_trajectory,
                       int node_min, int node_max, const orc_scan* scan, orc_pose scan_pose,
                       uint8_t* rgb, int* w_out, int* h_out)
{
    int a[12];
    *w_out = *h_out = 0;
    if (!orc_map_actual_size(m, a))
        return 1;
    const int W = a[10], H = a[11], ps = m->patch_size;
    const int gx0 = a[4], gy0 = a[5], gx1 = a[6], gy1 = a[7];
    uint8_t* img = (uint8_t*)malloc((size_t)W * H * 3 + 1);
    memset(img, 192, (size_t)W * H * 3);          /* :430-433 */
    /* DrawMap (:278-317): allocated patches of the bounding box */
    for (int py = 0; py < a[9]; ++py)
        for (int px = 0; px < a[8]; ++px) {
            const int qx = a[0] + px, qy = a[1] + py;
            if (!m->patch_alloc[(size_t)qy * m->npx + qx])
                continue;
            for (int yy = 0; yy < ps; ++yy)
                for (int xx = 0; xx < ps; ++xx) {
                    const double v = m->cells[(size_t)(qy * ps + yy) * m->w + (size_t)(qx * ps + xx)];
                    if (v <= 0.0 || v > 1.0)
                        continue;
                    const uint8_t g = (uint8_t)((1.0 - v) * 255.0);
                    uint8_t* p = img + 3 * ((size_t)(py * ps + yy) * W + (size_t)(px * ps + xx));
                    p[0] = p[1] = p[2] = g;
                }
        }
    /* DrawTrajectory (:320-362) */
    if (draw_trajectory && n_nodes > 0 && node_min >= 0 && node_min < n_nodes && node_max < n_nodes) {
        int pxc, pyc;
        world_to_cell(m->min_x, m->min_y, m->res, nodes[node_min].x, nodes[node_min].y, &pxc, &pyc);
        int* buf = NULL;
        int cap = 0;
        for (int i = node_min + 1; i <= node_max; ++i) {
            int cx, cy;
            world_to_cell(m->min_x, m->min_y, m->res, nodes[i].x, nodes[i].y, &cx, &cy);
            const int need = imax(abs(cx - pxc), abs(cy - pyc)) + 2;
            if (need > cap) {
                cap = 2 * need;
                buf = (int*)realloc(buf, sizeof(int) * 2 * (size_t)cap);
            }
            const int nl = orc_bresenham(pxc, pyc, cx, cy, buf, cap);
            for (int j = 0; j < nl; ++j) {
                const int ix = buf[2 * j], iy = buf[2 * j + 1];
                if (ix < gx0 || ix >= gx1 - 1 || iy < gy0 || iy >= gy1 - 1)
                    continue;
                fill_block(img, W, H, ix - gx0, iy - gy0, 2, 255, 0, 0);
            }
            pxc = cx;
            pyc = cy;
        }
        free(buf);
    }
    /* DrawScan (:365-410); note the reference tests the pose's y index
     * against gridCellIdxMax.mX (:380) */
    if (scan) {
        int sx, sy;
        world_to_cell(m->min_x, m->min_y, m->res, scan_pose.x, scan_pose.y, &sx, &sy);
        if (sx >= gx0 && sx < gx1 - 2 && sy >= gy0 && sy < gx1 - 2)
            fill_block(img, W, H, sx - gx0, sy - gy0, 3, 0, 255, 0);
        const orc_pose sp = orc_compound(scan_pose, scan->rel_sensor_pose);
        for (int i = 0; i < scan->n; ++i) {
            double sinT, cosT;
            sincos(sp.theta + scan->angles[i], &sinT, &cosT);   /* HitPoint, H/sensor/sensor_data.hpp:162-173 */
            const double hx = sp.x + scan->ranges[i] * cosT;
            const double hy = sp.y + scan->ranges[i] * sinT;
            int ix, iy;
            world_to_cell(m->min_x, m->min_y, m->res, hx, hy, &ix, &iy);
            if (ix < gx0 || ix >= gx1 - 1 || iy < gy0 || iy >= gy1 - 1)
                continue;
            fill_block(img, W, H, ix - gx0, iy - gy0, 2, 0, 0, 255);
        }
    }
    /* flipped_up_down_view (:455-462) */
    for (int y = 0; y < H; ++y)
        memcpy(rgb + (size_t)y * W * 3, img + (size_t)(H - 1 - y) * W * 3, (size_t)W * 3);
    free(img);
    *w_out = W;
    *h_out = H;
    return 0;
}

static inline void map_update(orc_map* m, int x, int y, double p, int is_hit)
{
    /* GridMap::Update (:876-881) -> GridCellAt (:807-823) -> Bayes update */
    const size_t k = (size_t)y * (size_t)m->w + (size_t)x;
    m->cells[k] = orc_bayes_update(m->cells[k], p);
    m->patch_alloc[(size_t)(y / m->patch_size) * m->npx + (size_t)(x / m->patch_size)] = 1;
    if (is_hit)
        m->hit_count[k]++;
    else
        m->miss_count[k]++;
}

/* One ray: misses along Bresenham (minus the last cell) then the hit
 * (C/mapping/grid_map_builder.cpp:170-186, :384-396) */
static void integrate_ray(orc_map* m, int sx, int sy, int hx, int hy,
                          const orc_builder_params* bp, int** buf, int* bufcap)
{
    const int need = (abs(hx - sx) > abs(hy - sy) ? abs(hx - sx) : abs(hy - sy)) + 2;
    if (need > *bufcap) {
        *bufcap = need * 2;
        *buf = (int*)realloc(*buf, sizeof(int) * 2 * (size_t)(*bufcap));
    }
    const int n = orc_bresenham(sx, sy, hx, hy, *buf, *bufcap);
    for (int j = 0; j < n - 1; ++j)
        map_update(m, (*buf)[2 * j], (*buf)[2 * j + 1], bp->prob_miss, 0);
    map_update(m, hx, hy, bp->prob_hit, 1);
}

int orc_integrate_scan(orc_map* m, orc_pose robotPose, const orc_scan* scan,
                       const orc_builder_params* bp)
{
    /* UpdateGridMap (C/mapping/grid_map_builder.cpp:149-186) and
     * ComputeBoundingBoxAndScanPoints (:335-380) */
    const orc_pose sp = orc_compound(robotPose, scan->rel_sensor_pose);
    double blx = sp.x, bly = sp.y, trx = sp.x, try_ = sp.y;
    const double minRange = std_max(bp->usable_range_min, scan->min_range);
    const double maxRange = std_min(bp->usable_range_max, scan->max_range);
    double* hp = (double*)malloc(sizeof(double) * 2 * (size_t)(scan->n + 1));
    int nh = 0;
    for (int i = 0; i < scan->n; ++i) {
        const double r = scan->ranges[i];
        if (r >= maxRange || r <= minRange)
            continue;
        double sinT, cosT;
        sincos(sp.theta + scan->angles[i], &sinT, &cosT);
        const double hx = sp.x + r * cosT;
        const double hy = sp.y + r * sinT;
        hp[2 * nh] = hx;
        hp[2 * nh + 1] = hy;
        ++nh;
        blx = std_min(blx, hx);
        bly = std_min(bly, hy);
        trx = std_max(trx, hx);
        try_ = std_max(try_, hy);
    }
    orc_map_expand(m, blx, bly, trx, try_, 5.0);
    int sx, sy;
    world_to_cell(m->min_x, m->min_y, m->res, sp.x, sp.y, &sx, &sy);
    int* buf = NULL;
    int cap = 0;
    for (int i = 0; i < nh; ++i) {
        int hx, hy;
        world_to_cell(m->min_x, m->min_y, m->res, hp[2 * i], hp[2 * i + 1], &hx, &hy);
        integrate_ray(m, sx, sy, hx, hy, bp, &buf, &cap);
    }
    free(buf);
    free(hp);
    return 0;
}

int orc_construct_map_from_scans(orc_map* m, const orc_node* nodes, int n_nodes,
                                 const orc_builder_params* bp)
{
    /* C/mapping/grid_map_builder.cpp:227-332.  Note topRight starts at
     * numeric_limits<double>::min() (smallest positive normal), :236-237. */
    double blx = DBL_MAX, bly = DBL_MAX, trx = DBL_MIN, try_ = DBL_MIN;
    double** hps = (double**)calloc((size_t)(n_nodes + 1), sizeof(double*));
    int* nhs = (int*)calloc((size_t)(n_nodes + 1), sizeof(int));
    for (int k = 0; k < n_nodes; ++k) {
        const orc_scan* scan = &nodes[k].scan;
        const orc_pose sp = orc_compound(nodes[k].pose, scan->rel_sensor_pose);
        blx = std_min(blx, sp.x);
        bly = std_min(bly, sp.y);
        trx = std_max(trx, sp.x);
        try_ = std_max(try_, sp.y);
        const double minRange = std_max(bp->usable_range_min, scan->min_range);
        const double maxRange = std_min(bp->usable_range_max, scan->max_range);
        hps[k] = (double*)malloc(sizeof(double) * 2 * (size_t)(scan->n + 1));
        for (int i = 0; i < scan->n; ++i) {
            const double r = scan->ranges[i];
            if (r >= maxRange || r <= minRange)
                continue;
            double sinT, cosT;
            sincos(sp.theta + scan->angles[i], &sinT, &cosT);
            const double hx = sp.x + r * cosT;
            const double hy = sp.y + r * sinT;
            hps[k][2 * nhs[k]] = hx;
            hps[k][2 * nhs[k] + 1] = hy;
            nhs[k]++;
            blx = std_min(blx, hx);
            bly = std_min(bly, hy);
            trx = std_max(trx, hx);
            try_ = std_max(try_, hy);
        }
    }
    orc_map_resize(m, blx, bly, trx, try_);
    orc_map_reset(m);
    int* buf = NULL;
    int cap = 0;
    for (int k = 0; k < n_nodes; ++k) {
        const orc_scan* scan = &nodes[k].scan;
        const orc_pose sp = orc_compound(nodes[k].pose, scan->rel_sensor_pose);
        int sx, sy;
        world_to_cell(m->min_x, m->min_y, m->res, sp.x, sp.y, &sx, &sy);
        for (int i = 0; i < nhs[k]; ++i) {
            int hx, hy;
            world_to_cell(m->min_x, m->min_y, m->res, hps[k][2 * i], hps[k][2 * i + 1], &hx, &hy);
            integrate_ray(m, sx, sy, hx, hy, bp, &buf, &cap);
        }
        free(hps[k]);
    }
    free(buf);
    free(hps);
    free(nhs);
    return 0;
}

/* ------------------------------------------------------------------ */
/* CostSquareError (C/mapping/cost_function_square_error.cpp)          */
/* ------------------------------------------------------------------ */
static inline double bicubic_h(double t)
{
    /* :281-295 */
    const double at = fabs(t);
    if (at <= 1.0) {
        const double at3 = pow(at, 3.0);
        const double at2 = pow(at, 2.0);
        return (at3 - 2.0 * at2 + 1.0);
    } else if (at <= 2.0) {
        const double at3 = pow(at, 3.0);
        const double at2 = pow(at, 2.0);
        return (-at3 + 5.0 * at2 - 8.0 * at + 4.0);
    }
    return 0.0;
}

static inline double bicubic_f(const orc_grid* g, double x, double y)
{
    /* :298-310: clamp(static_cast<int>(x), 0, W-1) -- truncation */
    const int xc = iclamp((int)x, 0, g->w - 1);
    const int yc = iclamp((int)y, 0, g->h - 1);
    return grid_value(g, xc, yc);
}

double orc_sq_smoothed_value(const orc_grid* g, double x, double y)
{
    /* :276-346.  The reference evaluates vecX^T * M * vecY with Eigen
     * (not vendored; parity unpinned at that boundary).  Restated as
     * r_j = sum_i hx_i M_ij (i ascending), then sum_j r_j hy_j (j ascending). */
    const double floorX = floor(x);
    const double floorY = floor(y);
    const double x1 = 1.0 + x - floorX;
    const double x2 = x - floorX;
    const double x3 = floorX + 1.0 - x;
    const double x4 = floorX + 2.0 - x;
    const double y1 = 1.0 + y - floorY;
    const double y2 = y - floorY;
    const double y3 = floorY + 1.0 - y;
    const double y4 = floorY + 2.0 - y;
    const double vx[4] = { bicubic_h(x1), bicubic_h(x2), bicubic_h(x3), bicubic_h(x4) };
    const double vy[4] = { bicubic_h(y1), bicubic_h(y2), bicubic_h(y3), bicubic_h(y4) };
    const double xs[4] = { x - x1, x - x2, x + x3, x + x4 };
    const double ys[4] = { y - y1, y - y2, y + y3, y + y4 };
    double r[4];
    for (int j = 0; j < 4; ++j) {
        double acc = vx[0] * bicubic_f(g, xs[0], ys[j]);
        for (int i = 1; i < 4; ++i)
            acc = acc + vx[i] * bicubic_f(g, xs[i], ys[j]);
        r[j] = acc;
    }
    double s = r[0] * vy[0];
    for (int j = 1; j < 4; ++j)
        s = s + r[j] * vy[j];
    return std_clamp(s, 0.0, 1.0);
}

double orc_sq_cost(const orc_grid* g, double umin, double umax, const orc_scan* scan,
                   orc_pose sp)
{
    /* :21-58 */
    double costValue = 0.0;
    const double minRange = std_max(umin, scan->min_range);
    const double maxRange = std_min(umax, scan->max_range);
    for (int i = 0; i < scan->n; ++i) {
        const double r = scan->ranges[i];
        if (r >= maxRange || r <= minRange)
            continue;
        double sinT, cosT;
        sincos(sp.theta + scan->angles[i], &sinT, &cosT);
        const double hx = sp.x + r * cosT;
        const double hy = sp.y + r * sinT;
        const double fx = (hx - g->min_x) / g->res;
        const double fy = (hy - g->min_y) / g->res;
        const double sv = orc_sq_smoothed_value(g, fx, fy);
        costValue += pow(1.0 - sv, 2.0);
    }
    return costValue;
}

/* ComputeMapGradient(gridMap, sensorPose, range, angle) (:203-229) via
 * ComputeMapGradient(gridMap, mapPos) (:172-199) */
static void sq_map_gradient(const orc_grid* g, orc_pose sp, double r, double a, double out[3])
{
    double sinT, cosT;
    sincos(sp.theta + a, &sinT, &cosT);
    const double hx = sp.x + r * cosT;
    const double hy = sp.y + r * sinT;
    const double deltaIdx = 0.1;
    const double deltaDist = g->res * deltaIdx;
    const double d = deltaIdx / 2.0;
    const double fx = (hx - g->min_x) / g->res;
    const double fy = (hy - g->min_y) / g->res;
    const double diffX = orc_sq_smoothed_value(g, fx + d, fy + 0.0) -
                         orc_sq_smoothed_value(g, fx - d, fy - 0.0);
    const double diffY = orc_sq_smoothed_value(g, fx + 0.0, fy + d) -
                         orc_sq_smoothed_value(g, fx - 0.0, fy - d);
    const double gx = diffX / deltaDist;
    const double gy = diffY / deltaDist;
    out[0] = gx;
    out[1] = gy;
    out[2] = -r * sinT * gx + r * cosT * gy;
}

/* CostSquareError::ComputeCovariance (:112-135) via ComputeGradient (:61-109):
 * g = sum 2 e (-grad) over usable beams, cov = g g^T + 0.01 I */
void orc_sq_covariance(const orc_grid* g, double umin, double umax, const orc_scan* scan,
                       orc_pose sp, double cov[9])
{
    double gx = 0.0, gy = 0.0, gt = 0.0;
    const double minRange = std_max(umin, scan->min_range);
    const double maxRange = std_min(umax, scan->max_range);
    for (int i = 0; i < scan->n; ++i) {
        const double r = scan->ranges[i];
        const double a = scan->angles[i];
        if (r >= maxRange || r <= minRange)
            continue;
        double sinT, cosT;
        sincos(sp.theta + a, &sinT, &cosT);
        const double hx = sp.x + r * cosT;
        const double hy = sp.y + r * sinT;
        const double fx = (hx - g->min_x) / g->res;
        const double fy = (hy - g->min_y) / g->res;
        const double e = 1.0 - orc_sq_smoothed_value(g, fx, fy);
        double gv[3];
        sq_map_gradient(g, sp, r, a, gv);
        gx += 2.0 * e * (-gv[0]);
        gy += 2.0 * e * (-gv[1]);
        gt += 2.0 * e * (-gv[2]);
    }
    const double gvv[3] = { gx, gy, gt };
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j)
            cov[3 * i + j] = gvv[i] * gvv[j];
    cov[0] += 0.01;
    cov[4] += 0.01;
    cov[8] += 0.01;
}

/* Eigen::ColPivHouseholderQR<Matrix3d>::compute + solve, restated from the
 * published algorithm (Eigen >= 3.3; not vendored in the reference). */
void orc_solve3_colpiv_qr(const double Hin[9], const double bin[3], double xout[3])
{
    enum { N = 3 };
    double A[N][N];      /* A[row][col] */
    for (int i = 0; i < N; ++i)
        for (int j = 0; j < N; ++j)
            A[i][j] = Hin[3 * i + j];
    double hc[N];
    int transp[N];
    double normU[N], normD[N];
    const double eps = DBL_EPSILON;
    for (int k = 0; k < N; ++k) {
        double s = 0.0;
        for (int i = 0; i < N; ++i)
            s += A[i][k] * A[i][k];
        normD[k] = sqrt(s);
        normU[k] = normD[k];
    }
    double maxn = normU[0];
    for (int k = 1; k < N; ++k)
        if (normU[k] > maxn)
            maxn = normU[k];
    const double thrHelper = (maxn * eps) * (maxn * eps) / (double)N;
    const double downdateThr = sqrt(eps);
    int nonzero = N;
    for (int k = 0; k < N; ++k) {
        int big = k;
        double bigv = normU[k];
        for (int j = k + 1; j < N; ++j)
            if (normU[j] > bigv) {
                bigv = normU[j];
                big = j;
            }
        const double bigSq = bigv * bigv;
        if (nonzero == N && bigSq < thrHelper * (double)(N - k))
            nonzero = k;
        transp[k] = big;
        if (k != big) {
            for (int i = 0; i < N; ++i) {
                double t = A[i][k];
                A[i][k] = A[i][big];
                A[i][big] = t;
            }
            double t = normU[k]; normU[k] = normU[big]; normU[big] = t;
            t = normD[k]; normD[k] = normD[big]; normD[big] = t;
        }
        /* makeHouseholderInPlace on A[k..N-1][k] */
        double tailSq = 0.0;
        for (int i = k + 1; i < N; ++i)
            tailSq += A[i][k] * A[i][k];
        const double c0 = A[k][k];
        double tau, beta;
        if (tailSq <= DBL_MIN) {
            tau = 0.0;
            beta = c0;
            for (int i = k + 1; i < N; ++i)
                A[i][k] = 0.0;
        } else {
            beta = sqrt(c0 * c0 + tailSq);
            if (c0 >= 0.0)
                beta = -beta;
            for (int i = k + 1; i < N; ++i)
                A[i][k] = A[i][k] / (c0 - beta);
            tau = (beta - c0) / beta;
        }
        hc[k] = tau;
        A[k][k] = beta;
        /* applyHouseholderOnTheLeft on the bottom-right corner */
        if (tau != 0.0) {
            for (int j = k + 1; j < N; ++j) {
                double tmp = 0.0;
                for (int i = k + 1; i < N; ++i)
                    tmp += A[i][k] * A[i][j];
                tmp += A[k][j];
                A[k][j] -= tau * tmp;
                for (int i = k + 1; i < N; ++i)
                    A[i][j] -= (tau * A[i][k]) * tmp;
            }
        }
        for (int j = k + 1; j < N; ++j) {
            if (normU[j] != 0.0) {
                double temp = fabs(A[k][j]) / normU[j];
                temp = (1.0 + temp) * (1.0 - temp);
                temp = temp < 0.0 ? 0.0 : temp;
                const double q = normU[j] / normD[j];
                const double temp2 = temp * (q * q);
                if (temp2 <= downdateThr) {
                    double s = 0.0;
                    for (int i = k + 1; i < N; ++i)
                        s += A[i][j] * A[i][j];
                    normD[j] = sqrt(s);
                    normU[j] = normD[j];
                } else {
                    normU[j] *= sqrt(temp);
                }
            }
        }
    }
    int perm[N];
    for (int k = 0; k < N; ++k)
        perm[k] = k;
    for (int k = 0; k < N; ++k) {
        int t = perm[k];
        perm[k] = perm[transp[k]];
        perm[transp[k]] = t;
    }
    if (nonzero == 0) {
        xout[0] = xout[1] = xout[2] = 0.0;
        return;
    }
    double c[N] = { bin[0], bin[1], bin[2] };
    /* c = Q^T b: apply H_0 .. H_{nonzero-1} */
    for (int k = 0; k < nonzero; ++k) {
        if (k == N - 1) {
            c[k] *= 1.0 - hc[k];
            continue;
        }
        if (hc[k] == 0.0)
            continue;
        double tmp = 0.0;
        for (int i = k + 1; i < N; ++i)
            tmp += A[i][k] * c[i];
        tmp += c[k];
        c[k] -= hc[k] * tmp;
        for (int i = k + 1; i < N; ++i)
            c[i] -= (hc[k] * A[i][k]) * tmp;
    }
    /* upper-triangular back substitution, column oriented */
    for (int i = nonzero - 1; i >= 0; --i) {
        if (c[i] != 0.0) {
            c[i] /= A[i][i];
            for (int j = 0; j < i; ++j)
                c[j] -= c[i] * A[j][i];
        }
    }
    for (int i = 0; i < nonzero; ++i)
        xout[perm[i]] = c[i];
    for (int i = nonzero; i < N; ++i)
        xout[perm[i]] = 0.0;
}

/* OptimizeStep (C/mapping/scan_matcher_linear_solver.cpp:88-148) */
static orc_pose linsolve_step(const orc_grid* g, const orc_linsolve_params* p,
                              const orc_scan* scan, orc_pose sp)
{
    double b[3] = { 0.0, 0.0, 0.0 };
    double H[9] = { 0 };
    const double minRange = std_max(p->usable_range_min, scan->min_range);
    const double maxRange = std_min(p->usable_range_max, scan->max_range);
    for (int i = 0; i < scan->n; ++i) {
        const double r = scan->ranges[i];
        const double a = scan->angles[i];
        if (r >= maxRange || r <= minRange)
            continue;
        double sinT, cosT;
        sincos(sp.theta + a, &sinT, &cosT);
        const double hx = sp.x + r * cosT;
        const double hy = sp.y + r * sinT;
        const double fx = (hx - g->min_x) / g->res;
        const double fy = (hy - g->min_y) / g->res;
        const double sv = orc_sq_smoothed_value(g, fx, fy);
        const double res = 1.0 - sv;
        double gv[3];
        sq_map_gradient(g, sp, r, a, gv);
        for (int k = 0; k < 3; ++k)
            b[k] += res * gv[k];
        for (int k = 0; k < 3; ++k)
            for (int l = 0; l < 3; ++l)
                H[3 * k + l] += gv[k] * gv[l];
    }
    H[0] += p->translation_regularizer;
    H[4] += p->translation_regularizer;
    H[8] += p->rotation_regularizer;
    double d[3];
    orc_solve3_colpiv_qr(H, b, d);
    orc_pose out = { sp.x + d[0], sp.y + d[1], sp.theta + d[2] };
    return out;
}

orc_pose orc_linsolve_step(const orc_grid* g, const orc_linsolve_params* p, const orc_scan* scan,
                           orc_pose sensor_pose)
{
    return linsolve_step(g, p, scan, sensor_pose);
}

int orc_linsolve_optimize_pose(const orc_grid* g, const orc_linsolve_params* p,
                               const orc_scan* scan, orc_pose initial_pose,
                               orc_summary* out, orc_pose* traj)
{
    /* :38-85 */
    memset(out, 0, sizeof(*out));
    const orc_pose rel = scan->rel_sensor_pose;
    const orc_pose sensorPose = orc_compound(initial_pose, rel);
    double prevCost = DBL_MAX;
    double cost = DBL_MAX;
    orc_pose best = sensorPose;
    int it = 0;
    for (;;) {
        best = linsolve_step(g, p, scan, best);
        cost = orc_sq_cost(g, p->cost_usable_range_min, p->cost_usable_range_max, scan, best);
        if (traj)
            traj[it] = best;
        if (++it >= p->num_iterations_max || fabs(prevCost - cost) < p->convergence_threshold)
            break;
        prevCost = cost;
    }
    out->pose_found = 1;
    out->normalized_cost = cost / (double)scan->n;
    out->initial_pose = initial_pose;
    out->estimated_pose = orc_move_backward(best, rel);
    out->sensor_pose = sensorPose;
    out->best_sensor_pose = best;
    out->best_win[0] = it;
    /* CostSquareError::ComputeCovariance (:112-135) at the best pose */
    orc_sq_covariance(g, p->cost_usable_range_min, p->cost_usable_range_max, scan, best, out->covariance);
    return 0;
}

/* ScanInterpolator::Interpolate, C/mapping/scan_interpolator.cpp:9-98.
 * ToCartesianCoordinate H/util.hpp:148-152 (GCC fuses the sin/cos pair into
 * sincos), Distance H/point.hpp:113-117, ToPolarCoordinate H/util.hpp:156-161. */
int orc_scan_interpolate(const double* ranges, const double* angles, int n, double dist_scans,
                         double dist_threshold_empty, double* out_ranges, double* out_angles, int cap)
{
    if (n < 1) return 0;
    double* px = (double*)malloc(sizeof(double) * (size_t)n);
    double* py = (double*)malloc(sizeof(double) * (size_t)n);
    for (int i = 0; i < n; ++i) { /* :22-27 */
        double s, c;
        sincos(angles[i], &s, &c);
        px[i] = ranges[i] * c;
        py[i] = ranges[i] * s;
    }
    int m = 0;
#define EMIT(X, Y)                                                     \
    do {                                                               \
        const double ex_ = (X), ey_ = (Y);                             \
        if (m < cap) {                                                 \
            out_ranges[m] = sqrt(ex_ * ex_ + ey_ * ey_);               \
            out_angles[m] = atan2(ey_, ex_);                           \
        }                                                              \
        ++m;                                                           \
    } while (0)
    EMIT(px[0], py[0]); /* :30-31 */
    double prevx = px[0], prevy = py[0], acc = 0.0;
    for (int i = 1; i < n; ++i) { /* :37-68 */
        const double x = px[i], y = py[i];
        const double d = sqrt((prevx - x) * (prevx - x) + (prevy - y) * (prevy - y));
        if (acc + d < dist_scans) {
            acc += d;
            prevx = x, prevy = y;
        } else if (acc + d >= dist_threshold_empty) {
            EMIT(x, y);
            prevx = x, prevy = y;
            acc = 0.0;
        } else {
            const double ratio = (dist_scans - acc) / d;
            const double qx = (x - prevx) * ratio + prevx;
            const double qy = (y - prevy) * ratio + prevy;
            EMIT(qx, qy);
            prevx = qx, prevy = qy;
            acc = 0.0;
            --i; /* process the current point again */
        }
    }
#undef EMIT
    free(px);
    free(py);
    return m;
}
