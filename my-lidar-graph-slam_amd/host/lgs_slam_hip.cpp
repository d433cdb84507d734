// lgs_slam_hip.cpp -- the reference-shaped C++ classes over the C-ABI (see the header).
#include "lgs_slam_hip.hpp"

#include <cfloat>
#include <cstring>

namespace MyLidarGraphSlam {
namespace Hip {

namespace {

lgs_pose2d to_c(const RobotPose2D<double>& p) { return { p.mX, p.mY, p.mTheta }; }
RobotPose2D<double> from_c(const lgs_pose2d& p) { return { p.x, p.y, p.theta }; }

Matrix3d cov_of(const double* c)
{
    Matrix3d m;
    for (int i = 0; i < 9; ++i) m.m[i] = c[i];
    return m;
}

ScanMatchingSummary summary_of(const lgs_rtcsm_summary& s)
{
    ScanMatchingSummary o;
    o.mPoseFound = s.pose_found != 0;
    o.mNormalizedCost = s.normalized_cost;
    o.mInitialPose = from_c(s.initial_pose);
    o.mEstimatedPose = from_c(s.estimated_pose);
    o.mEstimatedCovariance = cov_of(s.covariance);
    return o;
}

}  // namespace

// ------------------------------------------------------------------ Device
Device::Device(int device)
{
    const int rc = lgs_ctx_create(device, &mCtx);
    if (rc != LGS_OK) throw Error(rc, "lgs_ctx_create(" + std::to_string(device) + ") failed");
}

Device::~Device()
{
    if (mCtx) lgs_ctx_destroy(mCtx);
}

void Device::Check(int status, const char* what) const
{
    if (status == LGS_OK) return;
    const char* m = lgs_ctx_last_error(mCtx);
    throw Error(status, std::string(what) + ": " + (m ? m : "") + " (status " + std::to_string(status) + ")");
}

void Device::Synchronize() const { Check(lgs_ctx_synchronize(mCtx), "lgs_ctx_synchronize"); }

// -------------------------------------------------------------- DeviceGrid
DeviceGrid::DeviceGrid(DevicePtr dev, int w, int h, double minX, double minY, double res)
    : mDev(std::move(dev)), mW(w), mH(h), mMinX(minX), mMinY(minY), mRes(res)
{
    mDev->Check(lgs_grid_create(mDev->Handle(), w, h, minX, minY, res, &mGrid), "lgs_grid_create");
}

DeviceGrid::DeviceGrid(DevicePtr dev, const std::vector<double>& cells, int w, int h, double minX,
                       double minY, double res)
    : DeviceGrid(std::move(dev), w, h, minX, minY, res)
{
    Upload(cells);
}

DeviceGrid::DeviceGrid(DevicePtr dev, lgs_grid* borrowed, int w, int h, double minX, double minY, double res)
    : mDev(std::move(dev)), mGrid(borrowed), mBorrowed(true), mW(w), mH(h), mMinX(minX), mMinY(minY), mRes(res)
{
}

DeviceGrid::DeviceGrid(DeviceGrid&& o) noexcept
    : mDev(std::move(o.mDev)), mGrid(o.mGrid), mBorrowed(o.mBorrowed), mW(o.mW), mH(o.mH), mMinX(o.mMinX),
      mMinY(o.mMinY), mRes(o.mRes)
{
    o.mGrid = nullptr;
}

DeviceGrid::~DeviceGrid()
{
    if (mGrid && !mBorrowed) lgs_grid_destroy(mGrid);
}

void DeviceGrid::Upload(const std::vector<double>& cells)
{
    if (cells.size() != (std::size_t)mW * mH) throw Error(LGS_ERR_INVALID_ARG, "DeviceGrid::Upload: size mismatch");
    mDev->Check(lgs_grid_upload(mDev->Handle(), mGrid, cells.data()), "lgs_grid_upload");
}

void DeviceGrid::UploadPatches(const void* const* patches, int npx, int npy, int patchSize, int cellBytes,
                               int valueOffset)
{
    mDev->Check(lgs_grid_upload_patches(mDev->Handle(), mGrid, patches, npx, npy, patchSize, cellBytes, valueOffset),
                "lgs_grid_upload_patches");
}

std::vector<double> DeviceGrid::Download() const
{
    std::vector<double> out((std::size_t)mW * mH);
    mDev->Check(lgs_grid_download(mDev->Handle(), mGrid, out.data()), "lgs_grid_download");
    return out;
}

// ---------------------------------------------------------------- ScanData
ScanData::ScanData(DevicePtr dev, const std::vector<double>& angles, const std::vector<double>& ranges,
                   const RobotPose2D<double>& relPose, double minRange, double maxRange)
    : mDev(std::move(dev)), mAngles(angles), mRanges(ranges), mRelPose(relPose)
{
    if (angles.size() != ranges.size()) throw Error(LGS_ERR_INVALID_ARG, "ScanData: angles/ranges size mismatch");
    lgs_scan_host h{ mRanges.data(), mAngles.data(), (int)mRanges.size(), to_c(relPose), minRange, maxRange };
    mDev->Check(lgs_scan_create(mDev->Handle(), &h, &mScan), "lgs_scan_create");
}

ScanData::ScanData(DevicePtr dev, lgs_scan* adopted, const RobotPose2D<double>& relPose)
    : mDev(std::move(dev)), mRelPose(relPose), mScan(adopted)
{
    int n = 0;
    mDev->Check(lgs_scan_get(mScan, &n, nullptr, nullptr), "lgs_scan_get");
    mRanges.resize(n);
    mAngles.resize(n);
    mDev->Check(lgs_scan_get(mScan, &n, mRanges.data(), mAngles.data()), "lgs_scan_get");
}

ScanData::~ScanData()
{
    if (mScan) lgs_scan_destroy(mScan);
}

ScanDataPtr ScanInterpolatorHip::Interpolate(const ScanDataPtr& scanData) const
{
    if (!scanData) throw Error(LGS_ERR_INVALID_ARG, "Interpolate: null scan");
    lgs_scan* out = nullptr;
    mDev->Check(lgs_scan_interpolate(mDev->Handle(), scanData->Handle(), mDistScans, mDistThresholdEmpty, &out),
                "lgs_scan_interpolate");
    return ScanDataPtr(new ScanData(mDev, out, scanData->RelativeSensorPose()));
}

// ------------------------------------------------------ cost parameters
CostGreedyEndpointParams CostGreedyEndpointParams::FromLauncherJson(double usableMin, double usableMax,
                                                                    double hitMissed, double occThr,
                                                                    int kernelSize, double jsonStdDev,
                                                                    double jsonScale)
{
    // CreateCostGreedyEndpoint (C/slam_launcher.cpp:54-76) passes
    // (..., kernelSize, standardDeviation, scalingFactor) into the constructor
    // (..., kernelSize, scalingFactor, standardDeviation)
    CostGreedyEndpointParams p;
    p.mUsableRangeMin = usableMin;
    p.mUsableRangeMax = usableMax;
    p.mHitAndMissedDist = hitMissed;
    p.mOccupancyThreshold = occThr;
    p.mKernelSize = kernelSize;
    p.mScalingFactor = jsonStdDev;
    p.mStandardDeviation = jsonScale;
    return p;
}

// ------------------------------------------ ScanMatcherRealTimeCorrelativeHip
ScanMatcherRealTimeCorrelativeHip::ScanMatcherRealTimeCorrelativeHip(DevicePtr dev,
                                                                     const CostGreedyEndpointParams& c,
                                                                     int lowResolution, double rangeX,
                                                                     double rangeY, double rangeTheta,
                                                                     double scanRangeMax)
    : mDev(std::move(dev))
{
    // the reference's constructor only stores its arguments (:13-27); invalid
    // values surface as LGS_ERR_INVALID_ARG from the first OptimizePose
    mParams = { lowResolution, rangeX, rangeY, rangeTheta, scanRangeMax };
    mCost = { c.mUsableRangeMin, c.mUsableRangeMax, c.mHitAndMissedDist, c.mOccupancyThreshold,
              c.mKernelSize, c.mScalingFactor, c.mStandardDeviation };
}

ScanMatchingSummary ScanMatcherRealTimeCorrelativeHip::OptimizePose(const ScanMatchingQuery& q)
{
    mDev->Check(lgs_rtcsm_optimize_pose_query(mDev->Handle(), q.mGridMap->Handle(), &mParams, &mCost,
                                              q.mScanData->Handle(), to_c(q.mInitialPose), &mLast),
                "lgs_rtcsm_optimize_pose_query");
    return summary_of(mLast);
}

ScanMatchingSummary ScanMatcherRealTimeCorrelativeHip::OptimizePose(const DeviceGrid& gridMap,
                                                                    const DeviceGrid& precompMap,
                                                                    const ScanDataPtr& scanData,
                                                                    const RobotPose2D<double>& initialPose,
                                                                    double thr) const
{
    mDev->Check(lgs_rtcsm_optimize_pose(mDev->Handle(), gridMap.Handle(), precompMap.Handle(), &mParams, &mCost,
                                        scanData->Handle(), to_c(initialPose), thr, &mLast),
                "lgs_rtcsm_optimize_pose");
    return summary_of(mLast);
}

DeviceGrid ScanMatcherRealTimeCorrelativeHip::ComputeCoarserMap(const DeviceGrid& g) const
{
    DeviceGrid out(mDev, g.NumCellsX(), g.NumCellsY(), g.MinX(), g.MinY(), g.Resolution());
    mDev->Check(lgs_grid_precompute_max(mDev->Handle(), g.Handle(), mParams.low_resolution,
                                        const_cast<lgs_grid*>(out.Handle())),
                "lgs_grid_precompute_max");
    return out;
}

// ------------------------------------------------ ScanMatcherBranchBoundHip
ScanMatcherBranchBoundHip::ScanMatcherBranchBoundHip(DevicePtr dev, const ScorePixelAccurateParams& sf,
                                                     const CostGreedyEndpointParams& c, int nodeHeightMax,
                                                     double rangeX, double rangeY, double rangeTheta,
                                                     double scanRangeMax)
    : mDev(std::move(dev))
{
    mParams = { nodeHeightMax, rangeX, rangeY, rangeTheta, scanRangeMax, sf.mUsableRangeMin, sf.mUsableRangeMax };
    mCost = { c.mUsableRangeMin, c.mUsableRangeMax, c.mHitAndMissedDist, c.mOccupancyThreshold,
              c.mKernelSize, c.mScalingFactor, c.mStandardDeviation };
}

ScanMatchingSummary ScanMatcherBranchBoundHip::OptimizePose(const ScanMatchingQuery& q)
{
    mDev->Check(lgs_bb_optimize_pose_query(mDev->Handle(), q.mGridMap->Handle(), &mParams, &mCost,
                                           q.mScanData->Handle(), to_c(q.mInitialPose), &mLast),
                "lgs_bb_optimize_pose_query");
    return summary_of(mLast);
}

ScanMatchingSummary ScanMatcherBranchBoundHip::OptimizePose(const DeviceGrid& gridMap,
                                                            const std::vector<DeviceGridPtr>& precompMaps,
                                                            const ScanDataPtr& scanData,
                                                            const RobotPose2D<double>& initialPose, double thr) const
{
    std::vector<const lgs_grid*> pyr;
    for (const auto& m : precompMaps) pyr.push_back(m->Handle());
    if ((int)pyr.size() != mParams.node_height_max + 1)
        throw Error(LGS_ERR_INVALID_ARG, "ScanMatcherBranchBoundHip: one precomputed map per node height needed");
    const lgs_scan* s = scanData->Handle();
    const lgs_pose2d p = to_c(initialPose);
    mDev->Check(lgs_bb_optimize_pose_batch(mDev->Handle(), gridMap.Handle(), pyr.data(), &mParams, &mCost, &s, &p,
                                           1, thr, &mLast),
                "lgs_bb_optimize_pose_batch");
    return summary_of(mLast);
}

std::vector<DeviceGridPtr> ScanMatcherBranchBoundHip::ComputeCoarserMaps(const DeviceGrid& g) const
{
    std::vector<DeviceGridPtr> out;
    std::vector<lgs_grid*> hs;
    for (int h = 0; h <= mParams.node_height_max; ++h) {
        out.push_back(std::make_shared<DeviceGrid>(mDev, g.NumCellsX(), g.NumCellsY(), g.MinX(), g.MinY(),
                                                   g.Resolution()));
        hs.push_back(const_cast<lgs_grid*>(out.back()->Handle()));
    }
    mDev->Check(lgs_grid_precompute_pyramid(mDev->Handle(), g.Handle(), mParams.node_height_max, hs.data()),
                "lgs_grid_precompute_pyramid");
    return out;
}

// ------------------------------------------------ ScanMatcherLinearSolverHip
ScanMatcherLinearSolverHip::ScanMatcherLinearSolverHip(DevicePtr dev, int numOfIterationsMax,
                                                       double convergenceThreshold, double usableRangeMin,
                                                       double usableRangeMax, double translationRegularizer,
                                                       double rotationRegularizer, double costUsableRangeMin,
                                                       double costUsableRangeMax)
    : mDev(std::move(dev))
{
    mParams = { numOfIterationsMax, convergenceThreshold, usableRangeMin, usableRangeMax,
                translationRegularizer, rotationRegularizer, costUsableRangeMin, costUsableRangeMax };
}

ScanMatchingSummary ScanMatcherLinearSolverHip::OptimizePose(const ScanMatchingQuery& q)
{
    mDev->Check(lgs_linsolve_optimize_pose(mDev->Handle(), q.mGridMap->Handle(), &mParams, q.mScanData->Handle(),
                                           to_c(q.mInitialPose), &mLast, nullptr),
                "lgs_linsolve_optimize_pose");
    ScanMatchingSummary o;
    o.mPoseFound = mLast.pose_found != 0;
    o.mNormalizedCost = mLast.normalized_cost;
    o.mInitialPose = from_c(mLast.initial_pose);
    o.mEstimatedPose = from_c(mLast.estimated_pose);
    o.mEstimatedCovariance = cov_of(mLast.covariance);
    return o;
}

// --------------------------------------------------------------- GridMapHip
GridMapHip::GridMapHip(DevicePtr dev, double resolution, int patchSize, int numCellsX, int numCellsY,
                       const RobotPose2D<double>& c)
    : mDev(std::move(dev))
{
    mDev->Check(lgs_map_create(mDev->Handle(), resolution, patchSize, numCellsX, numCellsY, c.mX, c.mY, &mMap),
                "lgs_map_create");
}

GridMapHip::~GridMapHip()
{
    if (mMap) lgs_map_destroy(mMap);
}

static lgs_builder_params bp_of(const GridMapBuilderParams& p)
{
    return { p.mUsableRangeMin, p.mUsableRangeMax, p.mProbHit, p.mProbMiss };
}

void GridMapHip::UpdateScan(const ScanData& scan, const RobotPose2D<double>& pose, const GridMapBuilderParams& p)
{
    const lgs_builder_params bp = bp_of(p);
    mDev->Check(lgs_map_update_scan(mDev->Handle(), mMap, scan.Handle(), to_c(pose), &bp), "lgs_map_update_scan");
}

void GridMapHip::ConstructMapFromScans(const std::vector<ScanDataPtr>& scans,
                                       const std::vector<RobotPose2D<double>>& poses,
                                       const GridMapBuilderParams& p)
{
    if (scans.size() != poses.size()) throw Error(LGS_ERR_INVALID_ARG, "ConstructMapFromScans: size mismatch");
    std::vector<const lgs_scan*> hs;
    std::vector<lgs_pose2d> ps;
    for (std::size_t i = 0; i < scans.size(); ++i) {
        hs.push_back(scans[i]->Handle());
        ps.push_back(to_c(poses[i]));
    }
    const lgs_builder_params bp = bp_of(p);
    mDev->Check(lgs_map_construct_from_scans(mDev->Handle(), mMap, hs.data(), ps.data(), (int)hs.size(), &bp),
                "lgs_map_construct_from_scans");
}

static void scan_arrays(const std::vector<ScanDataPtr>& scans, const std::vector<RobotPose2D<double>>& poses,
                        std::vector<const lgs_scan*>& hs, std::vector<lgs_pose2d>& ps, const char* what)
{
    if (scans.size() != poses.size()) throw Error(LGS_ERR_INVALID_ARG, std::string(what) + ": size mismatch");
    for (std::size_t i = 0; i < scans.size(); ++i) {
        hs.push_back(scans[i]->Handle());
        ps.push_back(to_c(poses[i]));
    }
}

void GridMapHip::AppendScan(GridMapHip& localMap, GridMapHip& latestMap, const std::vector<ScanDataPtr>& scans,
                            const std::vector<RobotPose2D<double>>& poses, const GridMapBuilderParams& p)
{
    if (localMap.mDev != latestMap.mDev) throw Error(LGS_ERR_INVALID_ARG, "AppendScan: maps of one device");
    std::vector<const lgs_scan*> hs;
    std::vector<lgs_pose2d> ps;
    scan_arrays(scans, poses, hs, ps, "AppendScan");
    const lgs_builder_params bp = bp_of(p);
    localMap.mDev->Check(lgs_map_append_scan(localMap.mDev->Handle(), localMap.mMap, latestMap.mMap, hs.data(),
                                             ps.data(), (int)hs.size(), &bp),
                         "lgs_map_append_scan");
}

void GridMapHip::ConstructMapsFromScans(const std::vector<GridMapHip*>& maps, const std::vector<int>& nodeIdxMin,
                                        const std::vector<int>& nodeIdxMax, const std::vector<ScanDataPtr>& scans,
                                        const std::vector<RobotPose2D<double>>& poses,
                                        const GridMapBuilderParams& p)
{
    if (maps.empty()) return;
    if (nodeIdxMin.size() != maps.size() || nodeIdxMax.size() != maps.size())
        throw Error(LGS_ERR_INVALID_ARG, "ConstructMapsFromScans: size mismatch");
    std::vector<const lgs_scan*> hs;
    std::vector<lgs_pose2d> ps;
    scan_arrays(scans, poses, hs, ps, "ConstructMapsFromScans");
    std::vector<lgs_map*> ms;
    for (GridMapHip* m : maps) {
        if (!m || m->mDev != maps[0]->mDev)
            throw Error(LGS_ERR_INVALID_ARG, "ConstructMapsFromScans: maps of one device");
        ms.push_back(m->mMap);
    }
    const lgs_builder_params bp = bp_of(p);
    const DevicePtr& dev = maps[0]->mDev;
    dev->Check(lgs_maps_construct_from_scans(dev->Handle(), ms.data(), nodeIdxMin.data(), nodeIdxMax.data(),
                                             (int)ms.size(), hs.data(), ps.data(), (int)hs.size(), &bp),
               "lgs_maps_construct_from_scans");
}

std::unique_ptr<GridMapHip> GridMapHip::ConstructGlobalMap(DevicePtr dev, double resolution, int patchSize,
                                                           const std::vector<ScanDataPtr>& scans,
                                                           const std::vector<RobotPose2D<double>>& poses,
                                                           const GridMapBuilderParams& p)
{
    std::vector<const lgs_scan*> hs;
    std::vector<lgs_pose2d> ps;
    scan_arrays(scans, poses, hs, ps, "ConstructGlobalMap");
    const lgs_builder_params bp = bp_of(p);
    lgs_map* m = nullptr;
    dev->Check(lgs_map_construct_global(dev->Handle(), resolution, patchSize, hs.data(), ps.data(), (int)hs.size(),
                                        &bp, &m),
               "lgs_map_construct_global");
    return std::unique_ptr<GridMapHip>(new GridMapHip(std::move(dev), m));
}

lgs_map_geometry GridMapHip::Geometry() const
{
    lgs_map_geometry g{};
    mDev->Check(lgs_map_get_geometry(mMap, &g), "lgs_map_get_geometry");
    return g;
}

DeviceGridPtr GridMapHip::Grid() const
{
    lgs_grid* g = nullptr;
    mDev->Check(lgs_map_grid(mMap, &g), "lgs_map_grid");
    const lgs_map_geometry geo = Geometry();
    return DeviceGridPtr(new DeviceGrid(mDev, g, geo.num_cells_x, geo.num_cells_y, geo.min_x, geo.min_y,
                                        geo.resolution));
}

void GridMapHip::Download(std::vector<double>* cells, std::vector<uint32_t>* hits,
                          std::vector<uint32_t>* misses) const
{
    const lgs_map_geometry g = Geometry();
    const std::size_t n = (std::size_t)g.num_cells_x * g.num_cells_y;
    if (cells) cells->resize(n);
    if (hits) hits->resize(n);
    if (misses) misses->resize(n);
    mDev->Check(lgs_map_download(mDev->Handle(), mMap, cells ? cells->data() : nullptr,
                                 hits ? hits->data() : nullptr, misses ? misses->data() : nullptr),
                "lgs_map_download");
}

// ------------------------------------------ LoopDetectorRealTimeCorrelativeHip
LoopDetectorRealTimeCorrelativeHip::LoopDetectorRealTimeCorrelativeHip(
    std::shared_ptr<ScanMatcherRealTimeCorrelativeHip> m, double thr, std::vector<DevicePtr> extra)
    : mScanMatcher(std::move(m)), mScoreThreshold(thr), mExtraDevices(std::move(extra))
{
    for (const auto& d : mExtraDevices)
        if (!d) throw Error(LGS_ERR_INVALID_ARG, "LoopDetectorRealTimeCorrelativeHip: null device");
    if (!(thr > 0.0 && thr <= 1.0))   // the reference asserts this (:21-22)
        throw Error(LGS_ERR_INVALID_ARG, "LoopDetectorRealTimeCorrelativeHip: score threshold must be in (0, 1]");
}

void LoopDetectorRealTimeCorrelativeHip::Detect(std::vector<LoopDetectionQuery>& queries,
                                                std::vector<LoopDetectionResult>& results)
{
    results.clear();
    if (queries.empty()) return;
    const DevicePtr& dev = mScanMatcher->Dev();
    std::vector<lgs_loop_query> qs;
    std::vector<lgs_loop_candidate> cs;
    for (auto& q : queries) {
        if (!q.mPrecomputedMap)   // LocalMapInfo caches the coarse map (:52-60)
            q.mPrecomputedMap = std::make_shared<DeviceGrid>(mScanMatcher->ComputeCoarserMap(*q.mLocalMap));
        lgs_loop_query c{};
        c.map = q.mLocalMap->Handle();
        c.coarse = q.mPrecomputedMap->Handle();
        c.local_map_node_pose = to_c(q.mLocalMapNodePose);
        c.local_map_node_index = q.mLocalMapNodeIndex;
        c.first_candidate = (int)cs.size();
        c.num_candidates = (int)q.mPoseGraphNodes.size();
        qs.push_back(c);
        for (const auto& n : q.mPoseGraphNodes)
            cs.push_back(lgs_loop_candidate{ n.mScanData->Handle(), to_c(n.mPose), n.mIndex, 0 });
    }
    std::vector<lgs_loop_result> out(cs.size());
    std::vector<lgs_ctx*> ctxs{ dev->Handle() };
    for (const auto& d : mExtraDevices) ctxs.push_back(d->Handle());
    dev->Check(lgs_loop_detect_rtcsm_multi(ctxs.data(), (int)ctxs.size(), &mScanMatcher->Params(),
                                           &mScanMatcher->Cost(), mScoreThreshold, qs.data(), (int)qs.size(),
                                           cs.data(), (int)cs.size(), out.data()),
               "lgs_loop_detect_rtcsm_multi");
    for (const auto& r : out) {
        if (!r.found) continue;   // the reference appends only detected loops, in order (:77-88)
        LoopDetectionResult o;
        o.mRelativePose = from_c(r.relative_pose);
        o.mStartNodePose = from_c(r.start_node_pose);
        o.mStartNodeIdx = r.start_node_index;
        o.mEndNodeIdx = r.end_node_index;
        o.mEstimatedCovMat = cov_of(r.covariance);
        results.push_back(o);
    }
}

// ------------------------------------------------ LoopDetectorBranchBoundHip
LoopDetectorBranchBoundHip::LoopDetectorBranchBoundHip(std::shared_ptr<ScanMatcherBranchBoundHip> m, double thr)
    : mScanMatcher(std::move(m)), mScoreThreshold(thr)
{
    if (!(thr > 0.0 && thr <= 1.0))   // the reference asserts this (:18-19)
        throw Error(LGS_ERR_INVALID_ARG, "LoopDetectorBranchBoundHip: score threshold must be in (0, 1]");
}

void LoopDetectorBranchBoundHip::Detect(std::vector<LoopDetectionQuery>& queries,
                                        std::vector<LoopDetectionResult>& results)
{
    results.clear();
    if (queries.empty()) return;
    const DevicePtr& dev = mScanMatcher->Dev();
    std::vector<lgs_loop_query> qs;
    std::vector<lgs_loop_candidate> cs;
    for (auto& q : queries) {
        lgs_loop_query c{};
        c.map = q.mLocalMap->Handle();   // lgs_loop_detect_bb builds the pyramid (:45-55)
        c.local_map_node_pose = to_c(q.mLocalMapNodePose);
        c.local_map_node_index = q.mLocalMapNodeIndex;
        c.first_candidate = (int)cs.size();
        c.num_candidates = (int)q.mPoseGraphNodes.size();
        qs.push_back(c);
        for (const auto& n : q.mPoseGraphNodes)
            cs.push_back(lgs_loop_candidate{ n.mScanData->Handle(), to_c(n.mPose), n.mIndex, 0 });
    }
    std::vector<lgs_loop_result> out(cs.size());
    dev->Check(lgs_loop_detect_bb(dev->Handle(), &mScanMatcher->Params(), &mScanMatcher->Cost(), mScoreThreshold,
                                  qs.data(), (int)qs.size(), cs.data(), (int)cs.size(), out.data()),
               "lgs_loop_detect_bb");
    for (const auto& r : out) {
        if (!r.found) continue;   // only detected loops, in query -> node order (:61-84)
        LoopDetectionResult o;
        o.mRelativePose = from_c(r.relative_pose);
        o.mStartNodePose = from_c(r.start_node_pose);
        o.mStartNodeIdx = r.start_node_index;
        o.mEndNodeIdx = r.end_node_index;
        o.mEstimatedCovMat = cov_of(r.covariance);
        results.push_back(o);
    }
}

}  // namespace Hip
}  // namespace MyLidarGraphSlam
