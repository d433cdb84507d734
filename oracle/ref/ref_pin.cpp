// ref_pin.cpp -- test infrastructure ONLY (never linked into the product).
//
// Pins the CPU oracle (oracle/lgs_oracle.c) and the host restatements against
// the reference ITSELF, for the parts of the reference that compile in this
// image without any stand-in: the reference's own headers and sources are
// included / compiled in place from /root/reference (oracle/ref/Makefile),
// with the reference's compiler flags (-O3, no -march: R/CMakeLists.txt:33-36).
// Everything else of the reference includes <Eigen/Core> (through
// H/util.hpp) or Boost and is unbuildable here.
//
// Entry points (extern "C", plain arrays, no reference types):
//   ref_compound / ref_inverse_compound / ref_move_backward
//       H/pose.hpp:150-206 (Compound, InverseCompound, MoveBackward)
//   ref_hit_points
//       Sensor::ScanData<double>::HitPoint, H/sensor/sensor_data.hpp:162-173
//   ref_hit_and_missed_points
//       Sensor::ScanData<double>::HitAndMissedPoint, :177-198
//   ref_bayes_sequence
//       BinaryBayesGridCell<double>::Update, H/grid_map/binary_bayes_grid_cell.hpp:75-119
//   ref_score_pixel_accurate
//       ScorePixelAccurate::Score, C/mapping/score_function_pixel_accurate.cpp:20-77,
//       over a dense grid behind the reference's own GridMapBase<double>
//       interface (H/grid_map/grid_map_base.hpp:13-114).  The grid's index and
//       value semantics restate GridMap::WorldCoordinateToGridCellIndex
//       (H/grid_map/grid_map.hpp:779-790) and GridMap::Value with a default
//       (:858-873): that part is harness, the scoring loop is the reference's.
//   ref_loss
//       the robust loss functions, C/mapping/robust_loss_function.cpp:17-188
//       and LossSquared (H/mapping/robust_loss_function.hpp:36-50)
//   ref_carmen_load
//       IO::Carmen::CarmenLogReader::Load, C/io/carmen/carmen_reader.cpp:11-503
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <memory>
#include <sstream>
#include <string>
#include <vector>

#include "my_lidar_graph_slam/grid_map/binary_bayes_grid_cell.hpp"
#include "my_lidar_graph_slam/grid_map/grid_map_base.hpp"
#include "my_lidar_graph_slam/io/carmen/carmen_reader.hpp"
#include "my_lidar_graph_slam/mapping/robust_loss_function.hpp"
#include "my_lidar_graph_slam/mapping/score_function_pixel_accurate.hpp"
#include "my_lidar_graph_slam/pose.hpp"
#include "my_lidar_graph_slam/sensor/sensor_data.hpp"

using namespace MyLidarGraphSlam;

namespace {

RobotPose2D<double> P(const double* p) { return RobotPose2D<double>(p[0], p[1], p[2]); }
void put(const RobotPose2D<double>& p, double* out)
{
    out[0] = p.mX;
    out[1] = p.mY;
    out[2] = p.mTheta;
}

Sensor::ScanDataPtr<double> make_scan(const double* ranges, const double* angles, int n, double min_range,
                                      double max_range)
{
    std::vector<double> a(angles, angles + n), r(ranges, ranges + n);
    const double amin = n ? angles[0] : 0.0, amax = n ? angles[n - 1] : 0.0;
    const RobotPose2D<double> zero(0.0, 0.0, 0.0);
    return std::make_shared<Sensor::ScanData<double>>("ref", 0.0, zero, zero, zero, min_range, max_range, amin,
                                                      amax, std::move(a), std::move(r));
}

// Dense row-major grid behind the reference's GridMapBase<double> interface
// (cell (x, y) at y * w + x; out of bounds -> the default value).
class DenseGrid final : public GridMapBase<double> {
public:
    DenseGrid(const double* cells, int w, int h, double min_x, double min_y, double res)
        : mCells(cells), mW(w), mH(h), mMin(min_x, min_y), mRes(res) {}
    double UnknownValue() const override { return 0.0; }
    bool IsInside(int x, int y) const override { return x >= 0 && x < mW && y >= 0 && y < mH; }
    bool IsInside(const Point2D<int>& i) const override { return IsInside(i.mX, i.mY); }
    bool IsInside(double x, double y) const override { return IsInside(WorldCoordinateToGridCellIndex(x, y)); }
    bool IsInside(const Point2D<double>& p) const override { return IsInside(p.mX, p.mY); }
    bool IsAllocated(int x, int y) const override { return IsInside(x, y); }
    bool IsAllocated(const Point2D<int>& i) const override { return IsInside(i); }
    Point2D<double> GridCellIndexToWorldCoordinate(int x, int y) const override
    {
        return Point2D<double>(mMin.mX + mRes * x, mMin.mY + mRes * y);
    }
    Point2D<double> GridCellIndexToWorldCoordinate(const Point2D<int>& i) const override
    {
        return GridCellIndexToWorldCoordinate(i.mX, i.mY);
    }
    // H/grid_map/grid_map.hpp:779-790: floor((pos - minPos) / resolution)
    Point2D<int> WorldCoordinateToGridCellIndex(double x, double y) const override
    {
        return Point2D<int>(static_cast<int>(std::floor((x - mMin.mX) / mRes)),
                            static_cast<int>(std::floor((y - mMin.mY) / mRes)));
    }
    Point2D<int> WorldCoordinateToGridCellIndex(const Point2D<double>& p) const override
    {
        return WorldCoordinateToGridCellIndex(p.mX, p.mY);
    }
    Point2D<double> WorldCoordinateToGridCellIndexFloat(double x, double y) const override
    {
        return Point2D<double>((x - mMin.mX) / mRes, (y - mMin.mY) / mRes);
    }
    Point2D<double> WorldCoordinateToGridCellIndexFloat(const Point2D<double>& p) const override
    {
        return WorldCoordinateToGridCellIndexFloat(p.mX, p.mY);
    }
    double Value(int x, int y) const override { return mCells[(size_t)y * mW + x]; }
    double Value(const Point2D<int>& i) const override { return Value(i.mX, i.mY); }
    double Value(int x, int y, double d) const override { return IsInside(x, y) ? Value(x, y) : d; }
    double Value(const Point2D<int>& i, double d) const override { return Value(i.mX, i.mY, d); }
    double Distance(int x0, int y0, int x1, int y1) const override
    {
        return std::hypot((x1 - x0) * mRes, (y1 - y0) * mRes);
    }
    double Distance(const Point2D<int>& a, const Point2D<int>& b) const override
    {
        return Distance(a.mX, a.mY, b.mX, b.mY);
    }
    double SquaredDistance(int x0, int y0, int x1, int y1) const override
    {
        const double dx = (x1 - x0) * mRes, dy = (y1 - y0) * mRes;
        return dx * dx + dy * dy;
    }
    double SquaredDistance(const Point2D<int>& a, const Point2D<int>& b) const override
    {
        return SquaredDistance(a.mX, a.mY, b.mX, b.mY);
    }
    double Resolution() const override { return mRes; }
    int NumOfGridCellsX() const override { return mW; }
    int NumOfGridCellsY() const override { return mH; }
    double MapSizeX() const override { return mW * mRes; }
    double MapSizeY() const override { return mH * mRes; }
    const Point2D<double>& MinPos() const override { return mMin; }

private:
    const double* mCells;
    int mW, mH;
    Point2D<double> mMin;
    double mRes;
};

}  // namespace

extern "C" {

void ref_compound(const double* s, const double* d, double* out) { put(Compound(P(s), P(d)), out); }
void ref_inverse_compound(const double* s, const double* e, double* out) { put(InverseCompound(P(s), P(e)), out); }
void ref_move_backward(const double* e, const double* d, double* out) { put(MoveBackward(P(e), P(d)), out); }

// xy[2*i], xy[2*i+1] = HitPoint(sensorPose, i)
void ref_hit_points(const double* ranges, const double* angles, int n, const double* sensor_pose, double* xy)
{
    auto s = make_scan(ranges, angles, n, 0.0, 1e9);
    for (int i = 0; i < n; ++i) {
        const Point2D<double> p = s->HitPoint(P(sensor_pose), (size_t)i);
        xy[2 * i] = p.mX;
        xy[2 * i + 1] = p.mY;
    }
}

// hm[4*i .. 4*i+3] = (hit x, hit y, missed x, missed y)
void ref_hit_and_missed_points(const double* ranges, const double* angles, int n, const double* sensor_pose,
                               double dist, double* hm)
{
    auto s = make_scan(ranges, angles, n, 0.0, 1e9);
    for (int i = 0; i < n; ++i) {
        Point2D<double> h, m;
        s->HitAndMissedPoint(P(sensor_pose), (size_t)i, dist, h, m);
        hm[4 * i] = h.mX;
        hm[4 * i + 1] = h.mY;
        hm[4 * i + 2] = m.mX;
        hm[4 * i + 3] = m.mY;
    }
}

// values[k] = the cell value after the k-th Update(probs[k]) of a fresh cell
void ref_bayes_sequence(const double* probs, int n, double* values)
{
    BinaryBayesGridCell<double> c;
    for (int k = 0; k < n; ++k) {
        c.Update(probs[k]);
        values[k] = c.Value();
    }
}

// ScorePixelAccurate::Score -> (score, normalized score, match rate)
void ref_score_pixel_accurate(const double* cells, int w, int h, double min_x, double min_y, double res,
                              const double* ranges, const double* angles, int n, double scan_min_range,
                              double scan_max_range, double usable_min, double usable_max,
                              const double* sensor_pose, double* out3)
{
    DenseGrid g(cells, w, h, min_x, min_y, res);
    auto s = make_scan(ranges, angles, n, scan_min_range, scan_max_range);
    Mapping::ScorePixelAccurate f(usable_min, usable_max);
    Mapping::ScoreFunction::Summary sum{};
    f.Score(g, s, P(sensor_pose), sum);
    out3[0] = sum.mScore;
    out3[1] = sum.mNormalizedScore;
    out3[2] = sum.mMatchRate;
}

// kind: 0 Huber, 1 Cauchy, 2 Fair, 3 GemanMcClure, 4 Welsch, 5 DCS, 6 Squared;
// out[2*i] = Loss(t[i]), out[2*i+1] = Weight(t[i])
int ref_loss(int kind, double scale, const double* t, int n, double* out)
{
    std::unique_ptr<Mapping::LossFunction> f;
    switch (kind) {
    case 0: f.reset(new Mapping::LossHuber(scale)); break;
    case 1: f.reset(new Mapping::LossCauchy(scale)); break;
    case 2: f.reset(new Mapping::LossFair(scale)); break;
    case 3: f.reset(new Mapping::LossGemanMcClure(scale)); break;
    case 4: f.reset(new Mapping::LossWelsch(scale)); break;
    case 5: f.reset(new Mapping::LossDCS(scale)); break;
    case 6: f.reset(new Mapping::LossSquared()); break;
    default: return -1;
    }
    for (int i = 0; i < n; ++i) {
        out[2 * i] = f->Loss(t[i]);
        out[2 * i + 1] = f->Weight(t[i]);
    }
    return 0;
}

// CarmenLogReader::Load over `text`.  Records are written as a flat fp64
// stream, one record after another:
//   odometry: 0, timestamp, x, y, theta, vx, vy, vtheta
//   scan:     1, timestamp, n, odom x y theta, vel x y theta, rel x y theta,
//             minRange, maxRange, minAngle, maxAngle, angles[n], ranges[n]
// and the sensor ids, NUL-terminated one after another, into ids.  Returns
// the number of doubles of the stream (at most cap are written), or -1.
long long ref_carmen_load(const char* text, double* out, long long cap, char* ids, long long ids_cap,
                          int* num_records)
{
    std::istringstream in{ std::string(text) };
    std::vector<Sensor::SensorDataPtr> data;
    IO::Carmen::CarmenLogReader reader;
    if (!reader.Load(in, data)) return -1;
    std::vector<double> v;
    std::string names;
    for (const auto& d : data) {
        names += d->SensorId();
        names.push_back('\0');
        if (auto o = std::dynamic_pointer_cast<const Sensor::OdometryData<double>>(d)) {
            const double rec[8] = { 0.0, o->TimeStamp(), o->Pose().mX, o->Pose().mY, o->Pose().mTheta,
                                    o->Velocity().mX, o->Velocity().mY, o->Velocity().mTheta };
            v.insert(v.end(), rec, rec + 8);
        } else if (auto s = std::dynamic_pointer_cast<const Sensor::ScanData<double>>(d)) {
            const double rec[16] = { 1.0, s->TimeStamp(), (double)s->NumOfScans(),
                                     s->OdomPose().mX, s->OdomPose().mY, s->OdomPose().mTheta,
                                     s->Velocity().mX, s->Velocity().mY, s->Velocity().mTheta,
                                     s->RelativeSensorPose().mX, s->RelativeSensorPose().mY,
                                     s->RelativeSensorPose().mTheta, s->MinRange(), s->MaxRange(),
                                     s->MinAngle(), s->MaxAngle() };
            v.insert(v.end(), rec, rec + 16);
            v.insert(v.end(), s->Angles().begin(), s->Angles().end());
            v.insert(v.end(), s->Ranges().begin(), s->Ranges().end());
        }
    }
    if (num_records) *num_records = (int)data.size();
    if (out && cap > 0)
        std::memcpy(out, v.data(), sizeof(double) * (size_t)std::min<long long>(cap, (long long)v.size()));
    if (ids && ids_cap > 0) std::memcpy(ids, names.data(), std::min<size_t>((size_t)ids_cap, names.size()));
    return (long long)v.size();
}

}  // extern "C"
