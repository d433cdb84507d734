// lgs_slam_hip.hpp -- C++ host side of the MI355X hot path, mirroring the
// reference's plugin interfaces so a caller of Forrest-Z/my-lidar-graph-slam
// finds the same names, argument meanings and error behaviour.
//
//   reference (H/ = include/my_lidar_graph_slam/)          here
//   Mapping::ScanMatcher (H/mapping/scan_matcher.hpp:83-103) ScanMatcher
//   ScanMatchingQuery / ScanMatchingSummary (:20-77)        same names
//   ScanMatcherRealTimeCorrelative
//     (H/mapping/scan_matcher_real_time_correlative.hpp:15-48)
//                                                           ScanMatcherRealTimeCorrelativeHip
//   ScanMatcherLinearSolver (H/mapping/scan_matcher_linear_solver.hpp:15-56)
//                                                           ScanMatcherLinearSolverHip
//   GridMap<BinaryBayesGridCell> + GridMapBuilder's scan insert / ConstructMapFromScans
//     (H/grid_map/grid_map.hpp, C/mapping/grid_map_builder.cpp:98-332)
//                                                           GridMapHip
//   LoopDetectorRealTimeCorrelative::Detect
//     (C/mapping/loop_detector_real_time_correlative.cpp:26-125)
//                                                           LoopDetectorRealTimeCorrelativeHip
//
// Everything is a thin RAII layer over the C-ABI (include/lgs_hip.h); the
// compute runs in HIP kernels on the GPU.  Value types are self-contained
// (no Eigen): Matrix3d is a row-major std::array.  INTEGRATION.md shows the
// glue that plugs these classes into the reference itself (flattening its
// patch-based GridMapType into a dense DeviceGrid, Eigen conversions).
//
// Errors: every non-zero status of the C-ABI is thrown as lgs::hip::Error
// (std::runtime_error) with the context's message -- the reference uses
// asserts/exceptions for misuse; no exception crosses the C-ABI itself.
#pragma once

#include <array>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "lgs_hip.h"

namespace MyLidarGraphSlam {
namespace Hip {

struct Error : std::runtime_error {
    int status;
    Error(int s, const std::string& m) : std::runtime_error(m), status(s) {}
};

// H/pose.hpp RobotPose2D<double> (mX, mY, mTheta)
template <typename T>
struct RobotPose2D {
    T mX = 0, mY = 0, mTheta = 0;
    RobotPose2D() = default;
    RobotPose2D(T x, T y, T theta) : mX(x), mY(y), mTheta(theta) {}
};

// Eigen::Matrix3d stand-in (row-major)
struct Matrix3d {
    std::array<double, 9> m{};
    double operator()(int r, int c) const { return m[3 * r + c]; }
};

// One GPU + HIP stream + scratch (lgs_ctx).  One per matcher instance, like
// the reference's distinct frontend / loop-detector matchers.
class Device {
public:
    explicit Device(int device = 0);
    ~Device();
    Device(const Device&) = delete;
    Device& operator=(const Device&) = delete;
    lgs_ctx* Handle() const { return mCtx; }
    void Check(int status, const char* what) const;
    void Synchronize() const;

private:
    lgs_ctx* mCtx = nullptr;
};
using DevicePtr = std::shared_ptr<Device>;

// GridMapBase<double> flattened to a dense row-major fp64 grid in HBM
// (cell (x, y) at y*w + x; 0.0 = Unknown = unallocated patch).
class DeviceGrid {
public:
    DeviceGrid(DevicePtr dev, int w, int h, double minX, double minY, double res);
    DeviceGrid(DevicePtr dev, const std::vector<double>& cells, int w, int h, double minX, double minY,
               double res);
    ~DeviceGrid();
    DeviceGrid(const DeviceGrid&) = delete;
    DeviceGrid& operator=(const DeviceGrid&) = delete;
    DeviceGrid(DeviceGrid&& o) noexcept;
    void Upload(const std::vector<double>& cells);
    // GridMapType ingest without Flatten: patches[py * npx + px] =
    // PatchAt(px, py).Data() or nullptr (lgs_grid_upload_patches); the grid
    // must be npx*patchSize x npy*patchSize
    void UploadPatches(const void* const* patches, int npx, int npy, int patchSize, int cellBytes = 16,
                       int valueOffset = 8);
    std::vector<double> Download() const;
    int NumCellsX() const { return mW; }
    int NumCellsY() const { return mH; }
    double Resolution() const { return mRes; }
    double MinX() const { return mMinX; }
    double MinY() const { return mMinY; }
    const lgs_grid* Handle() const { return mGrid; }
    const DevicePtr& Dev() const { return mDev; }

private:
    friend class GridMapHip;
    DeviceGrid(DevicePtr dev, lgs_grid* borrowed, int w, int h, double minX, double minY, double res);
    DevicePtr mDev;
    lgs_grid* mGrid = nullptr;
    bool mBorrowed = false;
    int mW = 0, mH = 0;
    double mMinX = 0, mMinY = 0, mRes = 0;
};
using DeviceGridPtr = std::shared_ptr<const DeviceGrid>;

// Sensor::ScanData<double> (H/sensor/sensor_data.hpp:65-158), uploaded once.
class ScanData {
public:
    ScanData(DevicePtr dev, const std::vector<double>& angles, const std::vector<double>& ranges,
             const RobotPose2D<double>& relPose = {}, double minRange = 0.0, double maxRange = 30.0);
    ~ScanData();
    ScanData(const ScanData&) = delete;
    ScanData& operator=(const ScanData&) = delete;
    std::size_t NumOfScans() const { return mRanges.size(); }
    const RobotPose2D<double>& RelativeSensorPose() const { return mRelPose; }
    const std::vector<double>& Ranges() const { return mRanges; }
    const std::vector<double>& Angles() const { return mAngles; }
    const lgs_scan* Handle() const { return mScan; }

private:
    friend class ScanInterpolatorHip;
    ScanData(DevicePtr dev, lgs_scan* adopted, const RobotPose2D<double>& relPose);  // takes ownership
    DevicePtr mDev;
    std::vector<double> mAngles, mRanges;
    RobotPose2D<double> mRelPose;
    lgs_scan* mScan = nullptr;
};
using ScanDataPtr = std::shared_ptr<const ScanData>;

// Mapping::ScanInterpolator (H/mapping/scan_interpolator.hpp,
// C/mapping/scan_interpolator.cpp:9-98): the interpolated scan is created
// device-resident directly.
class ScanInterpolatorHip {
public:
    ScanInterpolatorHip(DevicePtr dev, double distScans = 0.05, double distThresholdEmpty = 0.25)
        : mDev(std::move(dev)), mDistScans(distScans), mDistThresholdEmpty(distThresholdEmpty) {}
    ScanDataPtr Interpolate(const ScanDataPtr& scanData) const;

private:
    DevicePtr mDev;
    double mDistScans, mDistThresholdEmpty;
};

// H/mapping/scan_matcher.hpp:20-77
struct ScanMatchingQuery {
    ScanMatchingQuery(DeviceGridPtr gridMap, ScanDataPtr scanData, const RobotPose2D<double>& initialPose)
        : mGridMap(std::move(gridMap)), mScanData(std::move(scanData)), mInitialPose(initialPose) {}
    const DeviceGridPtr mGridMap;
    const ScanDataPtr mScanData;
    const RobotPose2D<double> mInitialPose;
};

struct ScanMatchingSummary {
    bool mPoseFound = false;
    double mNormalizedCost = 0.0;
    RobotPose2D<double> mInitialPose;
    RobotPose2D<double> mEstimatedPose;
    Matrix3d mEstimatedCovariance;
};

// Mapping::ScanMatcher (H/mapping/scan_matcher.hpp:83-103)
class ScanMatcher {
public:
    ScanMatcher() = default;
    virtual ~ScanMatcher() = default;
    ScanMatcher(const ScanMatcher&) = delete;
    ScanMatcher& operator=(const ScanMatcher&) = delete;
    virtual ScanMatchingSummary OptimizePose(const ScanMatchingQuery& queryInfo) = 0;
};
using ScanMatcherPtr = std::shared_ptr<ScanMatcher>;

// CostGreedyEndpoint members (the values the object ends up holding; the
// launcher passes (stddev, scale) into the (scale, stddev) slots, SURVEY
// finding 6 -- FromLauncherJson reproduces that).
struct CostGreedyEndpointParams {
    double mUsableRangeMin = 0.01, mUsableRangeMax = 20.0;
    double mHitAndMissedDist = 0.075, mOccupancyThreshold = 0.1;
    int mKernelSize = 1;
    double mScalingFactor = 0.05, mStandardDeviation = 1.0;
    static CostGreedyEndpointParams FromLauncherJson(double usableMin, double usableMax, double hitMissed,
                                                     double occThr, int kernelSize, double jsonStdDev,
                                                     double jsonScale);
};

// ScanMatcherRealTimeCorrelative (C/mapping/scan_matcher_real_time_correlative.cpp:14-256)
class ScanMatcherRealTimeCorrelativeHip final : public ScanMatcher {
public:
    ScanMatcherRealTimeCorrelativeHip(DevicePtr dev, const CostGreedyEndpointParams& costFunc,
                                      int lowResolution, double rangeX, double rangeY, double rangeTheta,
                                      double scanRangeMax);
    // OptimizePose(query): coarse map + search with threshold DBL_MIN (:31-47)
    ScanMatchingSummary OptimizePose(const ScanMatchingQuery& queryInfo) override;
    // the const overload used by loop detectors (:50-145)
    ScanMatchingSummary OptimizePose(const DeviceGrid& gridMap, const DeviceGrid& precompMap,
                                     const ScanDataPtr& scanData, const RobotPose2D<double>& initialPose,
                                     double normalizedScoreThreshold) const;
    // ComputeCoarserMap (:148-153)
    DeviceGrid ComputeCoarserMap(const DeviceGrid& gridMap) const;
    // full device summary of the last OptimizePose (diagnostics: score, window, ...)
    const lgs_rtcsm_summary& LastSummary() const { return mLast; }
    const lgs_rtcsm_params& Params() const { return mParams; }
    const lgs_cost_ge_params& Cost() const { return mCost; }
    const DevicePtr& Dev() const { return mDev; }

private:
    DevicePtr mDev;
    lgs_rtcsm_params mParams{};
    lgs_cost_ge_params mCost{};
    mutable lgs_rtcsm_summary mLast{};
};

// ScorePixelAccurate (C/mapping/score_function_pixel_accurate.cpp:9-17)
struct ScorePixelAccurateParams {
    double mUsableRangeMin = 0.01, mUsableRangeMax = 20.0;
};

// ScanMatcherBranchBound (C/mapping/scan_matcher_branch_bound.cpp:8-200): the
// device scores every node the reference's search can visit, the host
// replays the search.
class ScanMatcherBranchBoundHip final : public ScanMatcher {
public:
    ScanMatcherBranchBoundHip(DevicePtr dev, const ScorePixelAccurateParams& scoreFunc,
                              const CostGreedyEndpointParams& costFunc, int nodeHeightMax, double rangeX,
                              double rangeY, double rangeTheta, double scanRangeMax);
    // OptimizePose(query): pyramid + search with threshold DBL_MIN (:29-44)
    ScanMatchingSummary OptimizePose(const ScanMatchingQuery& queryInfo) override;
    // the const overload used by the loop detector (:47-154)
    ScanMatchingSummary OptimizePose(const DeviceGrid& gridMap, const std::vector<DeviceGridPtr>& precompMaps,
                                     const ScanDataPtr& scanData, const RobotPose2D<double>& initialPose,
                                     double normalizedScoreThreshold) const;
    // ComputeCoarserMaps (:157-165): heights 0..NodeHeightMax
    std::vector<DeviceGridPtr> ComputeCoarserMaps(const DeviceGrid& gridMap) const;
    const lgs_rtcsm_summary& LastSummary() const { return mLast; }
    const lgs_bb_params& Params() const { return mParams; }
    const lgs_cost_ge_params& Cost() const { return mCost; }
    const DevicePtr& Dev() const { return mDev; }

private:
    DevicePtr mDev;
    lgs_bb_params mParams{};
    lgs_cost_ge_params mCost{};
    mutable lgs_rtcsm_summary mLast{};
};

// ScanMatcherLinearSolver (C/mapping/scan_matcher_linear_solver.cpp:38-148)
// with CostSquareError(usableRangeMin, usableRangeMax).
class ScanMatcherLinearSolverHip final : public ScanMatcher {
public:
    ScanMatcherLinearSolverHip(DevicePtr dev, int numOfIterationsMax, double convergenceThreshold,
                               double usableRangeMin, double usableRangeMax, double translationRegularizer,
                               double rotationRegularizer, double costUsableRangeMin,
                               double costUsableRangeMax);
    ScanMatchingSummary OptimizePose(const ScanMatchingQuery& queryInfo) override;
    const lgs_linsolve_summary& LastSummary() const { return mLast; }

private:
    DevicePtr mDev;
    lgs_linsolve_params mParams{};
    lgs_linsolve_summary mLast{};
};

// GridMap<BinaryBayesGridCell<double>> with cells on the device and the
// reference's geometry; UpdateScan = GridMapBuilder::UpdateGridMap's insert of
// one scan into the current local map (:149-186), ConstructMapFromScans =
// :227-332 (the latest map).
struct GridMapBuilderParams {
    double mUsableRangeMin = 0.01, mUsableRangeMax = 20.0;
    double mProbHit = 0.6, mProbMiss = 0.45;
};

class GridMapHip {
public:
    GridMapHip(DevicePtr dev, double resolution, int patchSize, int numCellsX, int numCellsY,
               const RobotPose2D<double>& centerPos = {});
    ~GridMapHip();
    GridMapHip(const GridMapHip&) = delete;
    GridMapHip& operator=(const GridMapHip&) = delete;
    void UpdateScan(const ScanData& scan, const RobotPose2D<double>& robotPose, const GridMapBuilderParams& p);
    void ConstructMapFromScans(const std::vector<ScanDataPtr>& scans,
                               const std::vector<RobotPose2D<double>>& robotPoses,
                               const GridMapBuilderParams& p);
    // GridMapBuilder::AppendScan (C/mapping/grid_map_builder.cpp:48-59): the
    // newest scan (scans.back() at robotPoses.back()) into `localMap` as
    // UpdateScan does, and `latestMap` rebuilt from all of `scans` as
    // ConstructMapFromScans does -- one fused device pass for both maps.
    static void AppendScan(GridMapHip& localMap, GridMapHip& latestMap, const std::vector<ScanDataPtr>& scans,
                           const std::vector<RobotPose2D<double>>& robotPoses, const GridMapBuilderParams& p);
    // GridMapBuilder::AfterLoopClosure's rebuild of every local map
    // (C/mapping/grid_map_builder.cpp:62-80): maps[i] from the pose-graph
    // nodes nodeIdxMin[i]..nodeIdxMax[i] of (scans, robotPoses), one fused
    // device pass for all maps.
    static void ConstructMapsFromScans(const std::vector<GridMapHip*>& maps, const std::vector<int>& nodeIdxMin,
                                       const std::vector<int>& nodeIdxMax, const std::vector<ScanDataPtr>& scans,
                                       const std::vector<RobotPose2D<double>>& robotPoses,
                                       const GridMapBuilderParams& p);
    // GridMapBuilder::ConstructGlobalMap (C/mapping/grid_map_builder.cpp:83-95)
    static std::unique_ptr<GridMapHip> ConstructGlobalMap(DevicePtr dev, double resolution, int patchSize,
                                                          const std::vector<ScanDataPtr>& scans,
                                                          const std::vector<RobotPose2D<double>>& robotPoses,
                                                          const GridMapBuilderParams& p);
    lgs_map_geometry Geometry() const;
    // non-owning view of the current cells (valid until the next geometry change)
    DeviceGridPtr Grid() const;
    void Download(std::vector<double>* cells, std::vector<uint32_t>* hits, std::vector<uint32_t>* misses) const;
    lgs_map* Handle() const { return mMap; }
    const DevicePtr& Dev() const { return mDev; }

private:
    GridMapHip(DevicePtr dev, lgs_map* map) : mDev(std::move(dev)), mMap(map) {}
    DevicePtr mDev;
    lgs_map* mMap = nullptr;
};

// LoopDetectionQuery / LoopDetectionResult (H/mapping/loop_detector.hpp:26-87)
struct LoopCandidateNode {
    ScanDataPtr mScanData;
    RobotPose2D<double> mPose;
    int mIndex = 0;
};
struct LoopDetectionQuery {
    std::vector<LoopCandidateNode> mPoseGraphNodes;
    DeviceGridPtr mLocalMap;
    std::shared_ptr<DeviceGrid> mPrecomputedMap;   // LocalMapInfo::mPrecomputedMaps[0]; filled lazily
    RobotPose2D<double> mLocalMapNodePose;
    int mLocalMapNodeIndex = 0;
};
struct LoopDetectionResult {
    RobotPose2D<double> mRelativePose;
    RobotPose2D<double> mStartNodePose;
    int mStartNodeIdx = 0;
    int mEndNodeIdx = 0;
    Matrix3d mEstimatedCovMat;
};

class LoopDetectorRealTimeCorrelativeHip {
public:
    // extraDevices: more GPUs of this process to shard the candidates over
    // (lgs_loop_detect_rtcsm_multi); the matcher's own device is shard 0 and
    // holds the queries' maps and scans.  Results are the same with or without.
    LoopDetectorRealTimeCorrelativeHip(std::shared_ptr<ScanMatcherRealTimeCorrelativeHip> scanMatcher,
                                       double scoreThreshold, std::vector<DevicePtr> extraDevices = {});
    // Detect (:26-92): coarse maps computed once per query, every node matched,
    // found ones appended in query -> node order.
    void Detect(std::vector<LoopDetectionQuery>& queries, std::vector<LoopDetectionResult>& results);
    int NumDevices() const { return 1 + (int)mExtraDevices.size(); }

private:
    std::shared_ptr<ScanMatcherRealTimeCorrelativeHip> mScanMatcher;
    double mScoreThreshold;
    std::vector<DevicePtr> mExtraDevices;
};

// LoopDetectorBranchBound (C/mapping/loop_detector_branch_bound.cpp:10-117):
// pyramids computed per query (LocalMapInfo caches them, :45-55), every node
// matched, found ones appended in query -> node order.
class LoopDetectorBranchBoundHip {
public:
    LoopDetectorBranchBoundHip(std::shared_ptr<ScanMatcherBranchBoundHip> scanMatcher, double scoreThreshold);
    void Detect(std::vector<LoopDetectionQuery>& queries, std::vector<LoopDetectionResult>& results);

private:
    std::shared_ptr<ScanMatcherBranchBoundHip> mScanMatcher;
    double mScoreThreshold;
};

}  // namespace Hip
}  // namespace MyLidarGraphSlam
