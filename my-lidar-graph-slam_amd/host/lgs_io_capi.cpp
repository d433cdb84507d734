// lgs_io_capi.cpp -- extern "C" entry points of include/lgs_io.h over the
// C++ classes of lgs_io.hpp / lgs_posegraph.hpp.  No exception crosses the ABI.
#include <cstring>
#include <sstream>

#include "lgs_io.h"
#include "lgs_io.hpp"
#include "lgs_posegraph.hpp"

using namespace MyLidarGraphSlam::Hip;

namespace {

Matrix3d to_mat(const double* a)
{
    Matrix3d m;
    for (int k = 0; k < 9; ++k) m.m[k] = a[k];
    return m;
}

std::vector<Mapping::PoseGraph::Edge> to_edges(const lgs_pose_graph_edge* e, int n)
{
    std::vector<Mapping::PoseGraph::Edge> v;
    v.reserve((size_t)n);
    for (int i = 0; i < n; ++i)
        v.emplace_back(e[i].start_node_index, e[i].end_node_index,
                       RobotPose2D<double>(e[i].relative_pose.x, e[i].relative_pose.y, e[i].relative_pose.theta),
                       to_mat(e[i].information));
    return v;
}

IO::MapSaver::Options to_options(const lgs_map_save_options* o)
{
    IO::MapSaver::Options s;
    if (!o) return s;
    s.mDrawTrajectory = o->draw_trajectory != 0;
    s.mTrajectoryNodeIdxMin = o->trajectory_node_index_min;
    s.mTrajectoryNodeIdxMax = o->trajectory_node_index_max;
    s.mDrawScans = o->draw_scan != 0 && o->scan != nullptr;
    s.mScanPose = RobotPose2D<double>(o->scan_pose.x, o->scan_pose.y, o->scan_pose.theta);
    if (o->scan) {
        s.mScanData.mRanges = o->scan->ranges;
        s.mScanData.mAngles = o->scan->angles;
        s.mScanData.mNumOfScans = o->scan->n;
        s.mScanData.mRelativeSensorPose =
            RobotPose2D<double>(o->scan->rel_sensor_pose.x, o->scan->rel_sensor_pose.y,
                                o->scan->rel_sensor_pose.theta);
    }
    s.mSaveMetadata = o->save_metadata != 0;
    return s;
}

std::vector<RobotPose2D<double>> to_poses(const lgs_pose2d* p, int n)
{
    std::vector<RobotPose2D<double>> v;
    v.reserve((size_t)std::max(0, n));
    for (int i = 0; i < n; ++i) v.emplace_back(p[i].x, p[i].y, p[i].theta);
    return v;
}

template <typename F>
int guarded(F&& f)
{
    try {
        return f();
    } catch (const Error& e) {
        return e.status;
    } catch (const std::bad_alloc&) {
        return LGS_ERR_OOM;
    } catch (const std::invalid_argument&) {
        return LGS_ERR_INVALID_ARG;
    } catch (const std::out_of_range&) {
        return LGS_ERR_INVALID_ARG;
    } catch (...) {
        return LGS_ERR_INTERNAL;
    }
}

}  // namespace

extern "C" long long lgs_carmen_load(const char* text, double* out, long long cap, char* ids, long long ids_cap,
                                     long long* ids_bytes, int* num_records)
{
    if (!text) return -1;
    try {
        std::istringstream in{ std::string(text) };
        std::vector<Sensor::SensorDataPtr> data;
        IO::Carmen::CarmenLogReader reader;
        if (!reader.Load(in, data)) return -1;
        std::vector<double> v;
        std::string names;
        for (const auto& d : data) {
            names += d->SensorId();
            names.push_back('\0');
            if (auto o = std::dynamic_pointer_cast<const Sensor::OdometryData>(d)) {
                const double rec[8] = { 0.0, o->TimeStamp(), o->Pose().mX, o->Pose().mY, o->Pose().mTheta,
                                        o->Velocity().mX, o->Velocity().mY, o->Velocity().mTheta };
                v.insert(v.end(), rec, rec + 8);
            } else if (auto s = std::dynamic_pointer_cast<const Sensor::ScanData>(d)) {
                const double rec[16] = { 1.0, s->TimeStamp(), (double)s->NumOfScans(), s->OdomPose().mX,
                                         s->OdomPose().mY, s->OdomPose().mTheta, s->Velocity().mX, s->Velocity().mY,
                                         s->Velocity().mTheta, s->RelativeSensorPose().mX,
                                         s->RelativeSensorPose().mY, s->RelativeSensorPose().mTheta, s->MinRange(),
                                         s->MaxRange(), s->MinAngle(), s->MaxAngle() };
                v.insert(v.end(), rec, rec + 16);
                v.insert(v.end(), s->Angles().begin(), s->Angles().end());
                v.insert(v.end(), s->Ranges().begin(), s->Ranges().end());
            }
        }
        if (num_records) *num_records = (int)data.size();
        if (ids_bytes) *ids_bytes = (long long)names.size();
        if (out && cap > 0)
            std::memcpy(out, v.data(), sizeof(double) * (size_t)std::min<long long>(cap, (long long)v.size()));
        if (ids && ids_cap > 0) std::memcpy(ids, names.data(), std::min<size_t>((size_t)ids_cap, names.size()));
        return (long long)v.size();
    } catch (...) {
        return -1;
    }
}

extern "C" int lgs_pose_graph_optimize_lm(lgs_pose_graph_lm_params* p, lgs_pose2d* poses, int n,
                                          const lgs_pose_graph_edge* edges, int m, int* iterations,
                                          double* total_error)
{
    if (!p || n < 0 || m < 0 || (n > 0 && !poses) || (m > 0 && !edges) || p->num_iterations_max < 0)
        return LGS_ERR_INVALID_ARG;
    return guarded([&] {
        auto loss = Mapping::CreateLossFunction(p->loss_kind, p->loss_scale);
        if (!loss || (p->solver != LGS_LM_SPARSE_CHOLESKY && p->solver != LGS_LM_CONJUGATE_GRADIENT))
            return LGS_ERR_INVALID_ARG;
        Mapping::PoseGraphOptimizerLM opt(p->solver == LGS_LM_SPARSE_CHOLESKY
                                              ? Mapping::PoseGraphOptimizerLM::SolverType::SparseCholesky
                                              : Mapping::PoseGraphOptimizerLM::SolverType::ConjugateGradient,
                                          p->num_iterations_max, p->error_tolerance, p->lambda, loss);
        std::vector<Mapping::PoseGraph::Node> nodes;
        nodes.reserve((size_t)n);
        for (int i = 0; i < n; ++i) nodes.emplace_back(i, RobotPose2D<double>(poses[i].x, poses[i].y, poses[i].theta));
        opt.Optimize(nodes, to_edges(edges, m));
        for (int i = 0; i < n; ++i) {
            poses[i].x = nodes[i].Pose().mX;
            poses[i].y = nodes[i].Pose().mY;
            poses[i].theta = nodes[i].Pose().mTheta;
        }
        p->lambda = opt.Lambda();
        if (iterations) *iterations = opt.LastIterations();
        if (total_error) *total_error = opt.LastTotalError();
        return LGS_OK;
    });
}

extern "C" int lgs_robust_loss(int kind, double scale, const double* t, int n, double* out)
{
    if (n < 0 || (n > 0 && (!t || !out))) return LGS_ERR_INVALID_ARG;
    auto f = Mapping::CreateLossFunction(kind, scale);
    if (!f) return LGS_ERR_INVALID_ARG;
    for (int i = 0; i < n; ++i) {
        out[2 * i] = f->Loss(t[i]);
        out[2 * i + 1] = f->Weight(t[i]);
    }
    return LGS_OK;
}

extern "C" int lgs_map_draw_image(lgs_ctx* ctx, const lgs_map* map, const lgs_pose2d* poses, int n,
                                  const lgs_map_save_options* o, uint8_t* rgb, size_t cap, int* w, int* h)
{
    if (!ctx || !map || !w || !h || n < 0 || (n > 0 && !poses)) return LGS_ERR_INVALID_ARG;
    return guarded([&] {
        std::vector<uint8_t> img;
        int a[12];
        if (!IO::MapSaver::Instance()->DrawImage(ctx, map, to_poses(poses, n), to_options(o), img, *w, *h, a))
            return LGS_ERR_INVALID_ARG;
        if (rgb && cap >= img.size()) std::memcpy(rgb, img.data(), img.size());
        return LGS_OK;
    });
}

extern "C" int lgs_map_save(lgs_ctx* ctx, const lgs_map* map, const lgs_pose2d* poses, int n,
                            const lgs_map_save_options* o, const char* file_name)
{
    if (!ctx || !map || !file_name || n < 0 || (n > 0 && !poses)) return LGS_ERR_INVALID_ARG;
    return guarded([&] {
        IO::MapSaver::Options opt = to_options(o);
        opt.mFileName = file_name;
        return IO::MapSaver::Instance()->SaveMapCore(ctx, map, to_poses(poses, n), opt) ? LGS_OK
                                                                                         : LGS_ERR_INVALID_ARG;
    });
}

extern "C" int lgs_pose_graph_save(const int* idx, const lgs_pose2d* poses, const double* ts, int n,
                                   const lgs_pose_graph_edge* edges, int m, const char* file_name)
{
    if (!file_name || n < 0 || m < 0 || (n > 0 && (!idx || !poses || !ts)) || (m > 0 && !edges))
        return LGS_ERR_INVALID_ARG;
    return guarded([&] {
        std::vector<Mapping::PoseGraph::Node> nodes;
        nodes.reserve((size_t)n);
        for (int i = 0; i < n; ++i)
            nodes.emplace_back(idx[i], RobotPose2D<double>(poses[i].x, poses[i].y, poses[i].theta), ts[i]);
        return IO::MapSaver::Instance()->SavePoseGraph(nodes, to_edges(edges, m), file_name) ? LGS_OK
                                                                                             : LGS_ERR_INTERNAL;
    });
}

extern "C" int lgs_png_write_rgb8(const char* file_name, const uint8_t* rgb, int w, int h)
{
    if (!file_name || !rgb || w <= 0 || h <= 0) return LGS_ERR_INVALID_ARG;
    return guarded([&] { return IO::WritePngRgb8(file_name, rgb, w, h) ? LGS_OK : LGS_ERR_INTERNAL; });
}
