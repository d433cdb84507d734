// adapter_test.cpp -- exercises the reference-shaped C++ classes
// (my-lidar-graph-slam_amd/host/lgs_slam_hip.hpp) on the GPU and compares them
// with the CPU oracle (oracle/lgs_oracle.h; test infrastructure, linked here
// only).  Scenes are synthetic: a walled room with boxes, analytic ray cast.
// Prints one line per check; exit status 1 if any check fails.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <memory>
#include <random>
#include <string>
#include <vector>

#include "lgs_oracle.h"
#include "lgs_slam_hip.hpp"

using namespace MyLidarGraphSlam::Hip;

namespace {

int g_failed = 0;

void check(bool ok, const std::string& name, const std::string& detail = "")
{
    std::printf("[%s] %s%s%s\n", ok ? " OK " : "FAIL", name.c_str(), detail.empty() ? "" : ": ", detail.c_str());
    if (!ok) ++g_failed;
}

struct Seg { double x0, y0, x1, y1; };

std::vector<Seg> make_world(unsigned seed)
{
    const double h = 12.0;
    std::vector<Seg> s = { { -h, -h, h, -h }, { h, -h, h, h }, { h, h, -h, h }, { -h, h, -h, -h } };
    std::mt19937_64 rng(seed);
    std::uniform_real_distribution<double> size(0.2, 2.0), pos(-h + 1.2, h - 1.2);
    int boxes = 0;
    while (boxes < 30) {
        const double w = size(rng), d = size(rng), cx = pos(rng), cy = pos(rng);
        const double x0 = cx - w / 2, x1 = cx + w / 2, y0 = cy - d / 2, y1 = cy + d / 2;
        if (x1 > -2.5 && x0 < 2.5 && y1 > -2.5 && y0 < 2.5) continue;
        s.push_back({ x0, y0, x1, y0 });
        s.push_back({ x1, y0, x1, y1 });
        s.push_back({ x1, y1, x0, y1 });
        s.push_back({ x0, y1, x0, y0 });
        ++boxes;
    }
    return s;
}

std::vector<double> beam_angles(int n)
{
    const double fov = 270.0 * M_PI / 180.0;
    std::vector<double> a(n);
    for (int i = 0; i < n; ++i) a[i] = -fov / 2 + i * (fov / (n - 1));
    return a;
}

std::vector<double> ray_cast(const std::vector<Seg>& w, double x, double y, double th, const std::vector<double>& ang)
{
    std::vector<double> r(ang.size(), 30.0);
    for (std::size_t i = 0; i < ang.size(); ++i) {
        const double dx = std::cos(th + ang[i]), dy = std::sin(th + ang[i]);
        for (const Seg& s : w) {
            const double ex = s.x1 - s.x0, ey = s.y1 - s.y0;
            const double den = dx * ey - dy * ex;
            if (std::fabs(den) < 1e-12) continue;
            const double t = ((s.x0 - x) * ey - (s.y0 - y) * ex) / den;
            const double u = ((s.x0 - x) * dy - (s.y0 - y) * dx) / den;
            if (t > 0 && u >= 0 && u <= 1 && t < r[i]) r[i] = t;
        }
    }
    return r;
}

orc_scan oscan(const ScanData& s)
{
    orc_scan o{};
    o.ranges = s.Ranges().data();
    o.angles = s.Angles().data();
    o.n = (int)s.NumOfScans();
    o.rel_sensor_pose = { s.RelativeSensorPose().mX, s.RelativeSensorPose().mY, s.RelativeSensorPose().mTheta };
    o.min_range = 0.0;
    o.max_range = 30.0;
    return o;
}

bool same_pose(const RobotPose2D<double>& a, const orc_pose& b)
{
    return a.mX == b.x && a.mY == b.y && a.mTheta == b.theta;
}

bool same_pose(const RobotPose2D<double>& a, const RobotPose2D<double>& b)
{
    return a.mX == b.mX && a.mY == b.mY && a.mTheta == b.mTheta;
}

std::string fmt_pose(const RobotPose2D<double>& a, const orc_pose& b)
{
    char buf[256];
    std::snprintf(buf, sizeof(buf), "gpu (%.17g %.17g %.17g) oracle (%.17g %.17g %.17g)", a.mX, a.mY, a.mTheta,
                  b.x, b.y, b.theta);
    return buf;
}

}  // namespace

int main()
{
    std::shared_ptr<Device> dev;
    try {
        dev = std::make_shared<Device>(0);
    } catch (const Error& e) {
        std::printf("no GPU: %s\n", e.what());
        return 77;   // skip: the adapter and the C-ABI loaded, there is no device to run on
    }
    const auto world = make_world(42);
    const auto ang = beam_angles(361);
    const GridMapBuilderParams bp;   // 0.01 / 20.0 / 0.6 / 0.45
    const orc_builder_params obp = { bp.mUsableRangeMin, bp.mUsableRangeMax, bp.mProbHit, bp.mProbMiss };

    // ---- GridMapHip: UpdateGridMap-style inserts vs the oracle (local map growth)
    std::vector<RobotPose2D<double>> poses;
    for (int k = 0; k < 6; ++k) {
        const double phi = -0.6 + 0.24 * k;
        poses.push_back({ std::cos(phi), std::sin(phi), phi + M_PI / 2 });
    }
    std::vector<ScanDataPtr> scans;
    for (const auto& p : poses)
        scans.push_back(std::make_shared<ScanData>(dev, ang, ray_cast(world, p.mX, p.mY, p.mTheta, ang)));
    GridMapHip local(dev, 0.05, 64, 100, 100);
    orc_map om{};
    orc_map_init(&om, 0.05, 64, 100, 100, 0.0, 0.0);
    for (std::size_t k = 0; k < poses.size(); ++k) {
        local.UpdateScan(*scans[k], poses[k], bp);
        const orc_scan os = oscan(*scans[k]);
        orc_integrate_scan(&om, { poses[k].mX, poses[k].mY, poses[k].mTheta }, &os, &obp);
    }
    {
        std::vector<double> c;
        std::vector<uint32_t> h, m;
        local.Download(&c, &h, &m);
        const lgs_map_geometry g = local.Geometry();
        const std::size_t n = (std::size_t)om.w * om.h;
        bool ok = g.num_cells_x == om.w && g.num_cells_y == om.h && g.min_x == om.min_x && g.min_y == om.min_y &&
                  c.size() == n && std::memcmp(c.data(), om.cells, n * sizeof(double)) == 0 &&
                  std::memcmp(h.data(), om.hit_count, n * 4) == 0 && std::memcmp(m.data(), om.miss_count, n * 4) == 0;
        check(ok, "GridMapHip::UpdateScan x6 == oracle (cells, hit/miss counts, geometry)",
              std::to_string(g.num_cells_x) + "x" + std::to_string(g.num_cells_y));
    }

    // ---- ConstructMapFromScans (latest map)
    GridMapHip latest(dev, 0.05, 64, 64, 64);
    latest.ConstructMapFromScans(scans, poses, bp);
    orc_map ol{};
    orc_map_init(&ol, 0.05, 64, 64, 64, 0.0, 0.0);
    {
        std::vector<orc_node> nodes;
        std::vector<orc_scan> oss;
        for (std::size_t k = 0; k < scans.size(); ++k) oss.push_back(oscan(*scans[k]));
        for (std::size_t k = 0; k < scans.size(); ++k)
            nodes.push_back({ { poses[k].mX, poses[k].mY, poses[k].mTheta }, oss[k] });
        orc_construct_map_from_scans(&ol, nodes.data(), (int)nodes.size(), &obp);
        std::vector<double> c;
        latest.Download(&c, nullptr, nullptr);
        const std::size_t n = (std::size_t)ol.w * ol.h;
        check(c.size() == n && std::memcmp(c.data(), ol.cells, n * sizeof(double)) == 0,
              "GridMapHip::ConstructMapFromScans == oracle");
    }

    // ---- ScanInterpolatorHip vs the oracle (launcher defaults 0.05 / 0.25)
    {
        const ScanInterpolatorHip interp(dev);
        bool ok = true;
        std::size_t total = 0;
        for (const auto& sc : scans) {
            const ScanDataPtr out = interp.Interpolate(sc);
            std::vector<double> orr(4 * sc->NumOfScans() + 16), oa(orr.size());
            const int m = orc_scan_interpolate(sc->Ranges().data(), sc->Angles().data(), (int)sc->NumOfScans(), 0.05,
                                               0.25, orr.data(), oa.data(), (int)orr.size());
            ok = ok && m == (int)out->NumOfScans() &&
                 std::memcmp(orr.data(), out->Ranges().data(), sizeof(double) * m) == 0 &&
                 std::memcmp(oa.data(), out->Angles().data(), sizeof(double) * m) == 0;
            total += out->NumOfScans();
        }
        check(ok, "ScanInterpolatorHip::Interpolate == oracle", std::to_string(total) + " points from 6 scans");
    }

    // ---- AfterLoopClosure (two local maps, overlapping node ranges) and ConstructGlobalMap
    {
        std::vector<orc_scan> oss;
        for (std::size_t k = 0; k < scans.size(); ++k) oss.push_back(oscan(*scans[k]));
        auto oracle_construct = [&](orc_map* o, int lo, int hi) {
            std::vector<orc_node> nodes;
            for (int k = lo; k <= hi; ++k) nodes.push_back({ { poses[k].mX, poses[k].mY, poses[k].mTheta }, oss[k] });
            orc_construct_map_from_scans(o, nodes.data(), (int)nodes.size(), &obp);
        };
        auto same = [](const GridMapHip& g, const orc_map& o) {
            std::vector<double> c;
            std::vector<uint32_t> h, m;
            g.Download(&c, &h, &m);
            const lgs_map_geometry geo = g.Geometry();
            const std::size_t n = (std::size_t)o.w * o.h;
            return geo.num_cells_x == o.w && geo.num_cells_y == o.h && geo.min_x == o.min_x &&
                   geo.min_y == o.min_y && c.size() == n && std::memcmp(c.data(), o.cells, n * sizeof(double)) == 0 &&
                   std::memcmp(h.data(), o.hit_count, n * 4) == 0 && std::memcmp(m.data(), o.miss_count, n * 4) == 0;
        };
        GridMapHip second(dev, 0.05, 64, 0, 0, poses[2]);
        orc_map o2{};
        orc_map_init(&o2, 0.05, 64, 0, 0, poses[2].mX, poses[2].mY);
        GridMapHip::ConstructMapsFromScans({ &local, &second }, { 0, 2 }, { 5, 3 }, scans, poses, bp);
        oracle_construct(&om, 0, 5);
        oracle_construct(&o2, 2, 3);
        check(same(local, om) && same(second, o2), "GridMapHip::ConstructMapsFromScans (AfterLoopClosure) == oracle");
        auto global = GridMapHip::ConstructGlobalMap(dev, 0.05, 64, scans, poses, bp);
        orc_map og{};
        orc_map_init(&og, 0.05, 64, 0, 0, 0.0, 0.0);
        oracle_construct(&og, 0, 5);
        check(same(*global, og), "GridMapHip::ConstructGlobalMap == oracle");
        orc_map_free(&o2);
        orc_map_free(&og);
    }

    // ---- ScanMatcherRealTimeCorrelativeHip::OptimizePose(query) on the latest map
    const auto cost = CostGreedyEndpointParams::FromLauncherJson(0.01, 20.0, 0.075, 0.1, 1, 0.05, 1.0);
    auto rtc = std::make_shared<ScanMatcherRealTimeCorrelativeHip>(dev, cost, 5, 0.6, 0.6, 0.4, 20.0);
    const orc_cost_ge oc = { cost.mUsableRangeMin, cost.mUsableRangeMax, cost.mHitAndMissedDist,
                             cost.mOccupancyThreshold, cost.mKernelSize, cost.mScalingFactor,
                             cost.mStandardDeviation };
    const orc_rtcsm_params orp = { 5, 0.6, 0.6, 0.4, 20.0 };
    const DeviceGridPtr lgrid = latest.Grid();
    const orc_grid og = { ol.cells, ol.w, ol.h, ol.min_x, ol.min_y, ol.res };
    std::mt19937_64 rng(7);
    std::uniform_real_distribution<double> jit(-0.1, 0.1);
    for (int t = 0; t < 5; ++t) {
        const RobotPose2D<double> truth(0.2 * t - 0.4, 0.1 * t, 0.3 * t);
        auto s = std::make_shared<ScanData>(dev, ang, ray_cast(world, truth.mX, truth.mY, truth.mTheta, ang));
        const RobotPose2D<double> init(truth.mX + jit(rng), truth.mY + jit(rng), truth.mTheta + jit(rng));
        const ScanMatchingSummary r = rtc->OptimizePose(ScanMatchingQuery(lgrid, s, init));
        const orc_scan os = oscan(*s);
        orc_summary o{};
        orc_rtcsm_optimize_pose_query(&og, &orp, &oc, &os, { init.mX, init.mY, init.mTheta }, &o);
        const bool ok = r.mPoseFound == (o.pose_found != 0) && same_pose(r.mEstimatedPose, o.estimated_pose) &&
                        std::fabs(r.mNormalizedCost - o.normalized_cost) <= 1e-5 * std::max(1.0, std::fabs(o.normalized_cost));
        check(ok, "RealTimeCorrelative OptimizePose(query) #" + std::to_string(t),
              fmt_pose(r.mEstimatedPose, o.estimated_pose));
    }

    // ---- ComputeCoarserMap + the const overload (threshold 0.3)
    {
        const DeviceGrid coarse = rtc->ComputeCoarserMap(*lgrid);
        std::vector<double> oc5((std::size_t)ol.w * ol.h);
        orc_precompute_grid_map(ol.cells, ol.w, ol.h, 5, oc5.data());
        const std::vector<double> dc = coarse.Download();
        check(std::memcmp(dc.data(), oc5.data(), oc5.size() * sizeof(double)) == 0, "ComputeCoarserMap == oracle");
        const orc_grid ocg = { oc5.data(), ol.w, ol.h, ol.min_x, ol.min_y, ol.res };
        auto s = std::make_shared<ScanData>(dev, ang, ray_cast(world, 0.3, -0.2, 0.5, ang));
        const ScanMatchingSummary r = rtc->OptimizePose(*lgrid, coarse, s, { 0.35, -0.25, 0.45 }, 0.3);
        const orc_scan os = oscan(*s);
        orc_summary o{};
        orc_rtcsm_optimize_pose(&og, &ocg, &orp, &oc, &os, { 0.35, -0.25, 0.45 }, 0.3, &o);
        check(r.mPoseFound == (o.pose_found != 0) && same_pose(r.mEstimatedPose, o.estimated_pose),
              "RealTimeCorrelative OptimizePose(grid, precomp, scan, pose, 0.3)",
              fmt_pose(r.mEstimatedPose, o.estimated_pose));
    }

    // ---- ScanMatcherLinearSolverHip (JSON defaults; end-to-end tolerance)
    {
        ScanMatcherLinearSolverHip ls(dev, 100, 1e-3, 0.01, 20.0, 1e-3, 1e-3, 0.01, 20.0);
        auto s = std::make_shared<ScanData>(dev, ang, ray_cast(world, 0.1, 0.05, 0.2, ang));
        const RobotPose2D<double> init(0.12, 0.03, 0.21);
        const ScanMatchingSummary r = ls.OptimizePose(ScanMatchingQuery(lgrid, s, init));
        const orc_linsolve_params olp = { 100, 1e-3, 0.01, 20.0, 1e-3, 1e-3, 0.01, 20.0 };
        const orc_scan os = oscan(*s);
        orc_summary o{};
        orc_linsolve_optimize_pose(&og, &olp, &os, { init.mX, init.mY, init.mTheta }, &o, nullptr);
        const double d = std::max({ std::fabs(r.mEstimatedPose.mX - o.estimated_pose.x),
                                    std::fabs(r.mEstimatedPose.mY - o.estimated_pose.y),
                                    std::fabs(r.mEstimatedPose.mTheta - o.estimated_pose.theta) });
        check(r.mPoseFound && d <= 1e-3, "LinearSolver OptimizePose(query) within 1e-3 of the oracle",
              fmt_pose(r.mEstimatedPose, o.estimated_pose));
    }

    // ---- LoopDetectorRealTimeCorrelativeHip::Detect vs the oracle's Detect loop
    {
        LoopDetectorRealTimeCorrelativeHip det(rtc, 0.35);   // sparse 361-beam latest map
        std::vector<LoopDetectionQuery> qs(2);
        std::vector<std::vector<double>> oracle_coarse;
        for (int q = 0; q < 2; ++q) {
            qs[q].mLocalMap = lgrid;
            qs[q].mLocalMapNodePose = poses[q];
            qs[q].mLocalMapNodeIndex = q;
            for (int j = 0; j < 4; ++j) {
                const RobotPose2D<double> truth(-0.5 + 0.3 * j, 0.2 * q - 0.1, 0.7 * j + q);
                LoopCandidateNode n;
                n.mScanData = std::make_shared<ScanData>(dev, ang, ray_cast(world, truth.mX, truth.mY, truth.mTheta, ang));
                n.mPose = { truth.mX + jit(rng), truth.mY + jit(rng), truth.mTheta + jit(rng) };
                n.mIndex = 100 + 10 * q + j;
                qs[q].mPoseGraphNodes.push_back(n);
            }
        }
        std::vector<LoopDetectionResult> res;
        det.Detect(qs, res);
        std::vector<double> oc5((std::size_t)ol.w * ol.h);
        orc_precompute_grid_map(ol.cells, ol.w, ol.h, 5, oc5.data());
        const orc_grid ocg = { oc5.data(), ol.w, ol.h, ol.min_x, ol.min_y, ol.res };
        std::vector<std::pair<int, orc_pose>> expect;
        for (const auto& q : qs)
            for (const auto& n : q.mPoseGraphNodes) {
                const orc_scan os = oscan(*n.mScanData);
                orc_summary o{};
                orc_rtcsm_optimize_pose(&og, &ocg, &orp, &oc, &os, { n.mPose.mX, n.mPose.mY, n.mPose.mTheta }, 0.35, &o);
                if (!o.pose_found) continue;
                const orc_pose lp = { q.mLocalMapNodePose.mX, q.mLocalMapNodePose.mY, q.mLocalMapNodePose.mTheta };
                expect.push_back({ n.mIndex, orc_inverse_compound(lp, o.estimated_pose) });
            }
        bool ok = res.size() == expect.size();
        for (std::size_t i = 0; ok && i < res.size(); ++i)
            ok = res[i].mEndNodeIdx == expect[i].first && same_pose(res[i].mRelativePose, expect[i].second);
        check(ok && !res.empty(), "LoopDetectorRealTimeCorrelative::Detect == oracle (" + std::to_string(res.size()) +
                                      " of 8 found)");
        // the same Detect sharded over two more contexts on this GPU (one host
        // thread each, maps peer-copied): identical results
        auto d2 = std::make_shared<Device>(0), d3 = std::make_shared<Device>(0);
        LoopDetectorRealTimeCorrelativeHip multi(rtc, 0.35, { d2, d3 });
        std::vector<LoopDetectionResult> mres;
        multi.Detect(qs, mres);
        bool same_all = mres.size() == res.size() && multi.NumDevices() == 3;
        for (std::size_t i = 0; same_all && i < res.size(); ++i) {
            const auto &a = res[i], &b = mres[i];
            same_all = a.mStartNodeIdx == b.mStartNodeIdx && a.mEndNodeIdx == b.mEndNodeIdx &&
                       same_pose(a.mRelativePose, b.mRelativePose) && same_pose(a.mStartNodePose, b.mStartNodePose) &&
                       a.mEstimatedCovMat.m == b.mEstimatedCovMat.m;
        }
        check(same_all, "LoopDetectorRealTimeCorrelativeHip over 3 devices == one device");
    }

    // ---- ScanMatcherBranchBoundHip (query + the loop overload) and LoopDetectorBranchBoundHip
    {
        const ScorePixelAccurateParams sp;   // 0.01 / 20.0
        auto bbm = std::make_shared<ScanMatcherBranchBoundHip>(dev, sp, cost, 3, 0.6, 0.6, 0.3, 20.0);
        const orc_bb_params obb = { 3, 0.6, 0.6, 0.3, 20.0, sp.mUsableRangeMin, sp.mUsableRangeMax };
        const RobotPose2D<double> truth(0.1, -0.05, 0.4);
        auto sc = std::make_shared<ScanData>(dev, ang, ray_cast(world, truth.mX, truth.mY, truth.mTheta, ang));
        const RobotPose2D<double> init(0.15, -0.02, 0.43);
        const ScanMatchingQuery q(lgrid, sc, init);
        const ScanMatchingSummary s = bbm->OptimizePose(q);
        const orc_scan os = oscan(*sc);
        orc_summary o{};
        orc_bb_optimize_pose_query(&og, &obb, &oc, &os, { init.mX, init.mY, init.mTheta }, &o);
        check(s.mPoseFound == (o.pose_found != 0) && same_pose(s.mEstimatedPose, o.estimated_pose) &&
                  bbm->LastSummary().score_max == o.score_max && bbm->LastSummary().fine_blocks == o.coarse_evals,
              "ScanMatcherBranchBound::OptimizePose(query) == oracle (pose, score, nodes visited)");
        // the loop overload with the matcher's own pyramid, threshold 0.35
        const auto pyr = bbm->ComputeCoarserMaps(*lgrid);
        const ScanMatchingSummary s2 = bbm->OptimizePose(*lgrid, pyr, sc, init, 0.35);
        std::vector<std::vector<double>> bufs(4, std::vector<double>((std::size_t)ol.w * ol.h));
        std::vector<orc_grid> maps;
        for (int h = 0; h <= 3; ++h) {
            orc_precompute_grid_map(ol.cells, ol.w, ol.h, 1 << h, bufs[h].data());
            maps.push_back({ bufs[h].data(), ol.w, ol.h, ol.min_x, ol.min_y, ol.res });
        }
        orc_summary o2{};
        orc_bb_optimize_pose(&og, maps.data(), &obb, &oc, &os, { init.mX, init.mY, init.mTheta }, 0.35, &o2);
        check(s2.mPoseFound == (o2.pose_found != 0) && same_pose(s2.mEstimatedPose, o2.estimated_pose) &&
                  bbm->LastSummary().fine_blocks == o2.coarse_evals,
              "ScanMatcherBranchBound::OptimizePose(map, pyramid, .., 0.35) == oracle");
        LoopDetectorBranchBoundHip det(bbm, 0.35);
        std::vector<LoopDetectionQuery> qs(1);
        qs[0].mLocalMap = lgrid;
        qs[0].mLocalMapNodePose = { 0.05, 0.0, 0.1 };
        qs[0].mLocalMapNodeIndex = 3;
        for (int j = 0; j < 3; ++j) {
            LoopCandidateNode nd;
            const RobotPose2D<double> tr(0.1 * j - 0.1, 0.05 * j, 0.2 * j);
            nd.mScanData = std::make_shared<ScanData>(dev, ang, ray_cast(world, tr.mX, tr.mY, tr.mTheta, ang));
            nd.mPose = { tr.mX + jit(rng), tr.mY + jit(rng), tr.mTheta + jit(rng) };
            nd.mIndex = 200 + j;
            qs[0].mPoseGraphNodes.push_back(nd);
        }
        std::vector<LoopDetectionResult> res;
        det.Detect(qs, res);
        std::vector<std::pair<int, orc_pose>> expect;
        for (const auto& n : qs[0].mPoseGraphNodes) {
            const orc_scan ns = oscan(*n.mScanData);
            orc_summary o3{};
            orc_bb_optimize_pose(&og, maps.data(), &obb, &oc, &ns, { n.mPose.mX, n.mPose.mY, n.mPose.mTheta }, 0.35,
                                 &o3);
            if (!o3.pose_found) continue;
            expect.push_back({ n.mIndex, orc_inverse_compound({ 0.05, 0.0, 0.1 }, o3.estimated_pose) });
        }
        bool ok = res.size() == expect.size();
        for (std::size_t i = 0; ok && i < res.size(); ++i)
            ok = res[i].mEndNodeIdx == expect[i].first && same_pose(res[i].mRelativePose, expect[i].second);
        check(ok && !res.empty(), "LoopDetectorBranchBound::Detect == oracle (" + std::to_string(res.size()) +
                                      " of 3 found)");
    }

    // ---- error behaviour: status -> exception
    {
        bool threw = false;
        try {
            DeviceGrid g(dev, 4, 4, 0, 0, 0.05);
            g.Upload(std::vector<double>(3));
        } catch (const Error& e) {
            threw = e.status == LGS_ERR_INVALID_ARG;
        }
        check(threw, "DeviceGrid::Upload size mismatch throws Error(LGS_ERR_INVALID_ARG)");
        threw = false;
        try {
            LoopDetectorRealTimeCorrelativeHip bad(rtc, 1.5);
        } catch (const Error&) {
            threw = true;
        }
        check(threw, "LoopDetector score threshold outside (0, 1] throws");
    }

    orc_map_free(&om);
    orc_map_free(&ol);
    std::printf("%s\n", g_failed ? "ADAPTER TESTS FAILED" : "ADAPTER TESTS PASSED");
    return g_failed ? 1 : 0;
}
