// frontend_bench.cpp -- measurement drivers over the C++ adapter (bench.py
// loads them with ctypes; the loops themselves make no Python calls).
//
// lgs_frontend_bench: LidarGraphSlamFrontEnd::ProcessScan's per-scan loop
// (C/mapping/lidar_graph_slam_frontend.cpp:78-127) for a synthetic
// trajectory, every step through the reference-shaped classes:
//   sensor scan arrives (host ranges)     -> ScanData (upload)
//   ScanInterpolator::Interpolate          -> ScanInterpolatorHip
//   OptimizePose(query) from the odometry  -> ScanMatcherRealTimeCorrelativeHip
//   GridMapBuilder::AppendScan             -> GridMapHip::AppendScan (fused) or
//     (UpdateGridMap insert + UpdateLatestMap)  UpdateScan + ConstructMapFromScans
// The synthetic sensor (exact segment ray cast) is outside every timer.
//
// lgs_dropin_bench: the cost of the unchanged reference frontend's query path
// (INTEGRATION.md §2): its latest map is a patch-based GridMapType on the host.
// Two ingests per query are timed: the Flatten path (one virtual Value() per
// cell + a dense upload) and the patch-native one (the patch pointer table +
// lgs_grid_upload_patches: only allocated patches' raw cells cross PCIe).  A patch map with the reference's layout (row-major patches,
// unallocated = nullptr, cells with a virtual Value(), GridMap::Value's
// patch-index arithmetic) is built from a dense map once; each query then
// times Flatten, the upload and the match, next to the match on the resident
// map.
#include <chrono>
#include <cmath>
#include <cstring>
#include <memory>
#include <vector>

#include "lgs_slam_hip.hpp"

using namespace MyLidarGraphSlam::Hip;

extern "C" {

struct lgs_fb_in {
    int device;
    int n_scans;          // scans of the trajectory (scan 0 starts the maps)
    int warmup;           // untimed steps after scan 0
    int n_beams;
    int n_segs;
    int interp;           // 1: ScanInterpolator on (launcher default)
    int latest_scans;     // scans of the latest map (launcher JSON: 10)
    int fused;            // 1: GridMapBuilder::AppendScan as one call (lgs_map_append_scan)
    int low_res;
    double range_x, range_y, range_theta, scan_range_max;
    const double* segs;     // [n_segs][4] world segments
    const double* angles;   // [n_beams]
    const double* truths;   // [n_scans][3] sensor trajectory
    const double* odo;      // [n_scans][3] odometry increments (robot frame)
    int n_dump;             // first scans whose raw ranges are returned
    int opt_id;             // A/B: one lgs_ctx option set on the device context (0: none)
    double opt_value;
    int profile_warmup;     // 1: every kernel HIP-event-timed during the (untimed) warmup steps
};

struct lgs_fb_out {
    double* est;            // [n_scans][3] estimated poses
    double* guess;          // [n_scans][3] odometry guesses (scan 0: the truth)
    double* dump_ranges;    // [n_dump][n_beams]
    double total_s;         // timed steps, wall clock
    double phase_s[4];      // upload, interpolate, match, AppendScan (insert + latest map)
    int steps_timed;
    int not_found;          // matches with mPoseFound == false
    lgs_kernel_stat* kstats;   // [kstats_cap]: per-kernel times of the profiled warmup steps
    int kstats_cap;
    int kstats_n;
};

struct lgs_dropin_in {
    int device;
    int w, h, patch_size;
    double min_x, min_y, res;
    const double* cells;    // [h][w] dense map
    int n_beams, n_queries;
    const double* ranges;   // [n_queries][n_beams]
    const double* angles;   // [n_beams]
    const double* inits;    // [n_queries][3]
    int low_res;
    double range_x, range_y, range_theta, scan_range_max;
};

struct lgs_dropin_out {
    double flatten_s, upload_s, match_uploaded_s, match_resident_s;   // sums over the queries
    int same;               // 1 if both matches agree on every query
    double patch_ingest_s, match_patch_s;   // patch-native path: table + lgs_grid_upload_patches, match
    int same_patch;         // 1 if the patch-native match agrees with the resident one on every query
    int allocated_patches;  // of npx * npy
};

int lgs_frontend_bench(const lgs_fb_in* in, lgs_fb_out* out);
int lgs_dropin_bench(const lgs_dropin_in* in, lgs_dropin_out* out);
}

namespace {

using Clock = std::chrono::steady_clock;
double secs(Clock::time_point a, Clock::time_point b) { return std::chrono::duration<double>(b - a).count(); }

// synthetic sensor: exact distance along each beam to the nearest segment
// (lgs_amd/scene.py ray_cast), capped at 30 m
void ray_cast(const double* segs, int ns, const double pose[3], const double* ang, int nb, double* r)
{
    for (int i = 0; i < nb; ++i) {
        const double dx = std::cos(pose[2] + ang[i]), dy = std::sin(pose[2] + ang[i]);
        double best = INFINITY;
        for (int s = 0; s < ns; ++s) {
            const double* g = segs + 4 * s;
            const double qx = g[2] - g[0], qy = g[3] - g[1];
            const double px = g[0] - pose[0], py = g[1] - pose[1];
            const double den = dx * qy - dy * qx;
            if (std::fabs(den) <= 1e-12) continue;
            const double t = (px * qy - py * qx) / den;
            const double u = (px * dy - py * dx) / den;
            if (t > 1e-9 && u >= 0.0 && u <= 1.0 && t < best) best = t;
        }
        r[i] = std::fmin(best, 30.0);
    }
}

CostGreedyEndpointParams launcher_cost()
{
    // members scale 0.05 / stddev 1.0, as the launcher builds them (SURVEY finding 6)
    return CostGreedyEndpointParams::FromLauncherJson(0.01, 20.0, 0.075, 0.1, 1, 0.05, 1.0);
}

// --- a GridMapType look-alike for the drop-in measurement -----------------
struct CellBase {   // GridCell<double, double>: virtual Value()
    virtual ~CellBase() = default;
    virtual double Value() const = 0;
};
struct BayesCell final : CellBase {   // BinaryBayesGridCell<double>
    double mValue = 0.0;
    double Value() const override { return mValue; }
};
struct Patch {   // grid_map_patch.hpp: unique_ptr<T[]>, nullptr = unallocated
    std::unique_ptr<BayesCell[]> mData;
    double Value(int x, int y, int ps, double def) const { return mData ? mData[y * ps + x].Value() : def; }
};
struct GridMapBaseLike {   // GridMapBase<double>
    virtual ~GridMapBaseLike() = default;
    virtual double Value(int x, int y, double def) const = 0;
    virtual int NumOfGridCellsX() const = 0;
    virtual int NumOfGridCellsY() const = 0;
};
struct PatchGridMap final : GridMapBaseLike {   // GridMap<BinaryBayesGridCell<double>>
    int ps, npx, npy;
    std::vector<Patch> patches;
    PatchGridMap(const double* cells, int w, int h, int ps_) : ps(ps_), npx(w / ps_), npy(h / ps_)
    {
        patches.resize((size_t)npx * npy);
        for (int py = 0; py < npy; ++py)
            for (int px = 0; px < npx; ++px) {
                bool any = false;
                for (int y = 0; y < ps && !any; ++y)
                    for (int x = 0; x < ps && !any; ++x) any = cells[(size_t)(py * ps + y) * w + px * ps + x] != 0.0;
                if (!any) continue;
                Patch& p = patches[(size_t)py * npx + px];
                p.mData.reset(new BayesCell[(size_t)ps * ps]);
                for (int y = 0; y < ps; ++y)
                    for (int x = 0; x < ps; ++x) p.mData[y * ps + x].mValue = cells[(size_t)(py * ps + y) * w + px * ps + x];
            }
    }
    // GridMap::Value(x, y, default) (H/grid_map/grid_map.hpp:858-873)
    double Value(int x, int y, double def) const override
    {
        if (!(x >= 0 && x < npx * ps && y >= 0 && y < npy * ps)) return def;
        const int pxi = (x < 0) ? (x / ps - 1) : (x / ps), pyi = (y < 0) ? (y / ps - 1) : (y / ps);
        return patches[(size_t)pyi * npx + pxi].Value(x % ps, y % ps, ps, def);
    }
    int NumOfGridCellsX() const override { return npx * ps; }
    int NumOfGridCellsY() const override { return npy * ps; }
};

// INTEGRATION.md §2 Flatten (kept out of line: the virtual calls stay)
__attribute__((noinline)) std::vector<double> Flatten(const GridMapBaseLike& map)
{
    const int w = map.NumOfGridCellsX(), h = map.NumOfGridCellsY();
    std::vector<double> cells((size_t)w * h, 0.0);
    for (int y = 0; y < h; ++y)
        for (int x = 0; x < w; ++x) cells[(size_t)y * w + x] = map.Value(x, y, 0.0);
    return cells;
}

template <typename F>
int guarded(F&& f)
{
    try {
        f();
        return LGS_OK;
    } catch (const Error& e) {
        return e.status ? e.status : LGS_ERR_INTERNAL;
    } catch (...) {
        return LGS_ERR_INTERNAL;
    }
}

}  // namespace

extern "C" int lgs_frontend_bench(const lgs_fb_in* in, lgs_fb_out* out)
{
    if (!in || !out || in->n_scans < 2 || in->n_beams < 1 || in->warmup < 0 || in->warmup >= in->n_scans - 1 ||
        in->latest_scans < 1 || in->n_dump < 0 || in->n_dump > in->n_scans)
        return LGS_ERR_INVALID_ARG;
    return guarded([&] {
        auto dev = std::make_shared<Device>(in->device);
        if (in->opt_id) dev->Check(lgs_ctx_set_option(dev->Handle(), in->opt_id, in->opt_value), "lgs_ctx_set_option");
        const int n = in->n_scans, nb = in->n_beams;
        const std::vector<double> ang(in->angles, in->angles + nb);
        ScanInterpolatorHip interp(dev, 0.05, 0.25);   // launcher JSON DistScans / DistThresholdEmpty
        ScanMatcherRealTimeCorrelativeHip matcher(dev, launcher_cost(), in->low_res, in->range_x, in->range_y,
                                                  in->range_theta, in->scan_range_max);
        const GridMapBuilderParams bp{ 0.01, 20.0, 0.6, 0.45 };
        const double* t0 = in->truths;
        GridMapHip local(dev, 0.05, 100, 200, 200, RobotPose2D<double>(t0[0], t0[1], 0.0));
        GridMapHip latest(dev, 0.05, 100, 200, 200, RobotPose2D<double>(t0[0], t0[1], 0.0));
        std::vector<ScanDataPtr> scans;
        std::vector<RobotPose2D<double>> est;
        // the sensor: every step's ranges ray-cast before the loop, so nothing
        // untimed runs between the timed steps (an asynchronous AppendScan
        // cannot finish in an untimed gap)
        std::vector<double> rall((size_t)n * nb);
        for (int k = 0; k < n; ++k) {
            ray_cast(in->segs, in->n_segs, in->truths + 3 * k, in->angles, nb, rall.data() + (size_t)k * nb);
            if (k < in->n_dump) std::memcpy(out->dump_ranges + (size_t)k * nb, rall.data() + (size_t)k * nb,
                                            sizeof(double) * nb);
        }
        double ph[4] = { 0, 0, 0, 0 };
        out->not_found = 0;
        out->kstats_n = 0;
        const bool prof = in->profile_warmup && in->warmup > 0 && out->kstats && out->kstats_cap > 0;
        for (int k = 0; k < n; ++k) {
            // from step 2: step 1 makes the first match, whose first launches
            // load the kernels' code objects (tens of ms, not a step's time)
            if (prof && k == (in->warmup >= 3 ? 2 : 1)) {
                dev->Synchronize();
                dev->Check(lgs_ctx_set_option(dev->Handle(), LGS_OPT_PROFILE, 1.0), "lgs_ctx_set_option");
                dev->Check(lgs_ctx_reset_stats(dev->Handle()), "lgs_ctx_reset_stats");
            }
            if (k == in->warmup + 1) {   // timed steps from here
                dev->Synchronize();
                if (prof) {
                    const int m = lgs_ctx_kernel_stats(dev->Handle(), out->kstats, out->kstats_cap);
                    if (m < 0) dev->Check(-m, "lgs_ctx_kernel_stats");
                    out->kstats_n = m;
                    dev->Check(lgs_ctx_set_option(dev->Handle(), LGS_OPT_PROFILE, 0.0), "lgs_ctx_set_option");
                }
                for (double& p : ph) p = 0.0;
                out->not_found = 0;
            }
            const std::vector<double> r(rall.begin() + (ptrdiff_t)k * nb, rall.begin() + (ptrdiff_t)(k + 1) * nb);
            const Clock::time_point a = Clock::now();
            auto raw = std::make_shared<const ScanData>(dev, ang, r);
            const Clock::time_point b = Clock::now();
            ScanDataPtr scan = in->interp ? interp.Interpolate(raw) : raw;
            const Clock::time_point c = Clock::now();
            scans.push_back(scan);
            RobotPose2D<double> pose, guess;
            if (k == 0) {
                pose = guess = RobotPose2D<double>(t0[0], t0[1], t0[2]);
            } else {
                // odometry increment composed onto the last estimate (bench.py run_stream)
                const RobotPose2D<double>& l = est.back();
                const double* o = in->odo + 3 * k;
                const double cs = std::cos(l.mTheta), sn = std::sin(l.mTheta);
                guess = RobotPose2D<double>(l.mX + cs * o[0] - sn * o[1], l.mY + sn * o[0] + cs * o[1],
                                            l.mTheta + o[2]);
                // against the latest map of the previous AppendScan
                const ScanMatchingSummary s = matcher.OptimizePose(ScanMatchingQuery(latest.Grid(), scan, guess));
                out->not_found += s.mPoseFound ? 0 : 1;
                pose = s.mEstimatedPose;
            }
            const Clock::time_point d = Clock::now();
            est.push_back(pose);
            // GridMapBuilder::AppendScan: local-map insert + latest map from the
            // last latest_scans scans, one call (lgs_map_append_scan)
            const int lo = std::max(0, k + 1 - in->latest_scans);
            const std::vector<ScanDataPtr> ls(scans.begin() + lo, scans.begin() + k + 1);
            const std::vector<RobotPose2D<double>> lp(est.begin() + lo, est.begin() + k + 1);
            if (in->fused) {
                GridMapHip::AppendScan(local, latest, ls, lp, bp);
            } else {
                local.UpdateScan(*scan, pose, bp);        // UpdateGridMap's insert
                latest.ConstructMapFromScans(ls, lp, bp);   // UpdateLatestMap
            }
            if (k == n - 1) dev->Synchronize();   // the last step's asynchronous map work is timed too
            const Clock::time_point f = Clock::now();
            out->est[3 * k] = pose.mX, out->est[3 * k + 1] = pose.mY, out->est[3 * k + 2] = pose.mTheta;
            out->guess[3 * k] = guess.mX, out->guess[3 * k + 1] = guess.mY, out->guess[3 * k + 2] = guess.mTheta;
            ph[0] += secs(a, b), ph[1] += secs(b, c), ph[2] += secs(c, d), ph[3] += secs(d, f);
        }
        // the sensor's ray cast ran before the loop: total = the four phases,
        // back to back (the r vector copy per step is the only untimed work)
        out->total_s = ph[0] + ph[1] + ph[2] + ph[3];
        for (int i = 0; i < 4; ++i) out->phase_s[i] = ph[i];
        out->steps_timed = n - 1 - in->warmup;
    });
}

extern "C" int lgs_dropin_bench(const lgs_dropin_in* in, lgs_dropin_out* out)
{
    if (!in || !out || in->w <= 0 || in->h <= 0 || in->patch_size <= 0 || in->w % in->patch_size ||
        in->h % in->patch_size || in->n_queries < 1 || in->n_beams < 1)
        return LGS_ERR_INVALID_ARG;
    return guarded([&] {
        auto dev = std::make_shared<Device>(in->device);
        ScanMatcherRealTimeCorrelativeHip matcher(dev, launcher_cost(), in->low_res, in->range_x, in->range_y,
                                                  in->range_theta, in->scan_range_max);
        const PatchGridMap pm(in->cells, in->w, in->h, in->patch_size);
        const std::vector<double> dense(in->cells, in->cells + (size_t)in->w * in->h);
        auto resident = std::make_shared<const DeviceGrid>(dev, dense, in->w, in->h, in->min_x, in->min_y, in->res);
        const std::vector<double> ang(in->angles, in->angles + in->n_beams);
        std::memset(out, 0, sizeof(*out));
        out->same = 1;
        out->same_patch = 1;
        // the patch-native path's grid lives across queries (same geometry)
        auto pgrid = std::make_shared<DeviceGrid>(dev, in->w, in->h, in->min_x, in->min_y, in->res);
        static_assert(sizeof(BayesCell) == 16, "BinaryBayesGridCell<double> layout: vptr + double");
        std::vector<const void*> table(pm.patches.size());
        for (const Patch& p : pm.patches) out->allocated_patches += p.mData ? 1 : 0;
        for (int q = -1; q < in->n_queries; ++q) {   // q = -1: untimed warm-up
            const int qi = std::max(q, 0);
            const std::vector<double> r(in->ranges + (size_t)qi * in->n_beams,
                                        in->ranges + (size_t)(qi + 1) * in->n_beams);
            auto scan = std::make_shared<const ScanData>(dev, ang, r);
            const double* p = in->inits + 3 * qi;
            const RobotPose2D<double> init(p[0], p[1], p[2]);
            const Clock::time_point a = Clock::now();
            std::vector<double> cells = Flatten(pm);
            const Clock::time_point b = Clock::now();
            auto grid = std::make_shared<const DeviceGrid>(dev, cells, in->w, in->h, in->min_x, in->min_y, in->res);
            dev->Synchronize();
            const Clock::time_point c = Clock::now();
            const ScanMatchingSummary s1 = matcher.OptimizePose(ScanMatchingQuery(grid, scan, init));
            const Clock::time_point d = Clock::now();
            const ScanMatchingSummary s2 = matcher.OptimizePose(ScanMatchingQuery(resident, scan, init));
            const Clock::time_point e = Clock::now();
            // patch-native ingest: PatchAt(px, py).Data() per patch, then one call
            for (std::size_t k = 0; k < table.size(); ++k) table[k] = pm.patches[k].mData.get();
            pgrid->UploadPatches(table.data(), pm.npx, pm.npy, pm.ps, (int)sizeof(BayesCell),
                                 (int)(sizeof(BayesCell) - sizeof(double)));
            const Clock::time_point f = Clock::now();
            const ScanMatchingSummary s3 = matcher.OptimizePose(ScanMatchingQuery(pgrid, scan, init));
            const Clock::time_point g = Clock::now();
            if (q < 0) continue;
            out->patch_ingest_s += secs(e, f);
            out->match_patch_s += secs(f, g);
            out->same_patch &= (s3.mEstimatedPose.mX == s2.mEstimatedPose.mX &&
                                s3.mEstimatedPose.mY == s2.mEstimatedPose.mY &&
                                s3.mEstimatedPose.mTheta == s2.mEstimatedPose.mTheta && s3.mNormalizedCost == s2.mNormalizedCost)
                                   ? 1
                                   : 0;
            out->flatten_s += secs(a, b);
            out->upload_s += secs(b, c);
            out->match_uploaded_s += secs(c, d);
            out->match_resident_s += secs(d, e);
            out->same &= (s1.mEstimatedPose.mX == s2.mEstimatedPose.mX && s1.mEstimatedPose.mY == s2.mEstimatedPose.mY &&
                          s1.mEstimatedPose.mTheta == s2.mEstimatedPose.mTheta)
                             ? 1
                             : 0;
        }
    });
}
