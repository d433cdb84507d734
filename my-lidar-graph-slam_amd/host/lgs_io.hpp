// lgs_io.hpp -- input logs and map output, host C++ with
// the reference's class names:
//
//   reference (H/ = include/my_lidar_graph_slam/, C/ = src/my_lidar_graph_slam/)   here
//   Sensor::SensorData / OdometryData / ScanData (H/sensor/sensor_data.hpp)       Sensor::SensorData /
//                                                                                 OdometryData / ScanData
//   IO::Carmen::CarmenLogReader (H/io/carmen/carmen_reader.hpp,
//     C/io/carmen/carmen_reader.cpp:11-530)                                       same
//   IO::MapSaver (H/io/map_saver.hpp, C/io/map_saver.cpp:25-532)                  same, over GridMapHip
//
// The map image is drawn on the device (lgs_map_render_gray_region: DrawMap
// of the actual map size, GridMap::ComputeActualMapSize from the device's
// patch-allocation flags); the trajectory and scan overlays, the PNG encoding
// (zlib) and the JSON files are host work.  JSON is written the way
// boost::property_tree::write_json writes the reference's ptrees: every value
// a string, numbers with max_digits10 significant digits, 4-space indentation.
#pragma once

#include <istream>
#include <map>
#include <memory>
#include <string>
#include <unordered_map>
#include <vector>

#include "lgs_posegraph.hpp"
#include "lgs_slam_hip.hpp"

namespace MyLidarGraphSlam {
namespace Hip {
namespace Sensor {

// H/sensor/sensor_data.hpp:18-60
class SensorData {
public:
    SensorData(const std::string& sensorId, double timeStamp) : mSensorId(sensorId), mTimeStamp(timeStamp) {}
    virtual ~SensorData() = default;
    const std::string& SensorId() const { return mSensorId; }
    double TimeStamp() const { return mTimeStamp; }

private:
    std::string mSensorId;
    double mTimeStamp;
};
using SensorDataPtr = std::shared_ptr<SensorData>;

// OdometryData<double> (H/sensor/sensor_data.hpp:160-200 area)
class OdometryData final : public SensorData {
public:
    OdometryData(const std::string& sensorId, double timeStamp, const RobotPose2D<double>& pose,
                 const RobotPose2D<double>& velocity)
        : SensorData(sensorId, timeStamp), mPose(pose), mVelocity(velocity) {}
    const RobotPose2D<double>& Pose() const { return mPose; }
    const RobotPose2D<double>& Velocity() const { return mVelocity; }

private:
    RobotPose2D<double> mPose, mVelocity;
};
using OdometryDataPtr = std::shared_ptr<OdometryData>;

// Host-side ScanData<double> (H/sensor/sensor_data.hpp:65-158) as the log
// reader produces it; Upload() makes the device-resident Hip::ScanData the
// matchers and map builders take.
class ScanData final : public SensorData {
public:
    ScanData(const std::string& sensorId, double timeStamp, const RobotPose2D<double>& odomPose,
             const RobotPose2D<double>& velocity, const RobotPose2D<double>& relPose, double minRange,
             double maxRange, double minAngle, double maxAngle, std::vector<double>&& angles,
             std::vector<double>&& ranges)
        : SensorData(sensorId, timeStamp), mOdomPose(odomPose), mVelocity(velocity), mRelPose(relPose),
          mMinRange(minRange), mMaxRange(maxRange), mMinAngle(minAngle), mMaxAngle(maxAngle),
          mAngles(std::move(angles)), mRanges(std::move(ranges)) {}
    const RobotPose2D<double>& OdomPose() const { return mOdomPose; }
    const RobotPose2D<double>& Velocity() const { return mVelocity; }
    const RobotPose2D<double>& RelativeSensorPose() const { return mRelPose; }
    double MinRange() const { return mMinRange; }
    double MaxRange() const { return mMaxRange; }
    double MinAngle() const { return mMinAngle; }
    double MaxAngle() const { return mMaxAngle; }
    std::size_t NumOfScans() const { return mRanges.size(); }
    const std::vector<double>& Angles() const { return mAngles; }
    const std::vector<double>& Ranges() const { return mRanges; }
    // device-resident copy for the HIP matchers / map builders
    Hip::ScanDataPtr Upload(DevicePtr dev) const;

private:
    RobotPose2D<double> mOdomPose, mVelocity, mRelPose;
    double mMinRange, mMaxRange, mMinAngle, mMaxAngle;
    std::vector<double> mAngles, mRanges;
};
using ScanDataPtr = std::shared_ptr<ScanData>;

}  // namespace Sensor

namespace IO {
namespace Carmen {

// C/io/carmen/carmen_reader.cpp: PARAM, ODOM, RAWLASER1-4, ROBOTLASER1-2,
// FLASER/RLASER and LASER3/4 records, everything else ignored; fields are
// read with the same std::istringstream extractions, so malformed lines
// parse exactly as they do in the reference.
class CarmenLogReader final {
public:
    bool Load(std::istream& inputStream, std::vector<Sensor::SensorDataPtr>& sensorData);

private:
    enum class DataType { None = 0, Param, Odom, TruePos, RawLaser, RobotLaser, OldFrontLaser, OldRearLaser,
                          OldOtherLaser };
    using ParamMapType = std::unordered_map<std::string, std::string>;

    void ReadLine(const std::string& sensorId, DataType dataType, std::istringstream& strStream,
                  ParamMapType& paramMap, std::vector<Sensor::SensorDataPtr>& sensorData);
    void ReadParameter(std::istringstream& strStream, ParamMapType& paramMap);
    Sensor::OdometryDataPtr ReadOdometryData(const std::string& sensorId, std::istringstream& strStream);
    Sensor::ScanDataPtr ReadRawLaserData(const std::string& sensorId, std::istringstream& strStream);
    Sensor::ScanDataPtr ReadRobotLaserData(const std::string& sensorId, std::istringstream& strStream);
    Sensor::ScanDataPtr ReadOldLaserData(const std::string& sensorId, std::istringstream& strStream,
                                         const ParamMapType& paramMap, bool withPoses);
    static double GuessAngleRange(int numReadings);
    static double GuessAngleIncrement(int numReadings);
    static DataType ToDataType(const std::string& dataTypeStr);
};

}  // namespace Carmen

// C/io/map_saver.cpp.  Maps are GridMapHip (cells on the device); the
// precomputed maps of a local map are DeviceGrids of its geometry.
struct LocalMapInfo {
    std::shared_ptr<GridMapHip> mMap;
    int mPoseGraphNodeIdxMin = 0;
    int mPoseGraphNodeIdxMax = 0;
    std::map<int, DeviceGridPtr> mPrecomputedMaps;   // node height -> window-max map (patch size of mMap)
};

class MapSaver final {
public:
    static MapSaver* Instance();

    // :32-53
    bool SaveMap(const GridMapHip& globalMap, const std::vector<Mapping::PoseGraph::Node>& poseGraphNodes,
                 const std::string& fileName, bool drawTrajectory, bool saveMetadata) const;
    // :56-120 (<fileName>.posegraph.json)
    bool SavePoseGraph(const std::vector<Mapping::PoseGraph::Node>& poseGraphNodes,
                       const std::vector<Mapping::PoseGraph::Edge>& poseGraphEdges,
                       const std::string& fileName) const;
    // :123-156
    bool SaveLocalMaps(const std::vector<LocalMapInfo>& localMaps,
                       const std::vector<Mapping::PoseGraph::Node>& poseGraphNodes, bool drawTrajectory,
                       bool saveMetadata, const std::string& fileName) const;
    // :159-178
    bool SaveLatestMap(const GridMapHip& latestMap, const std::vector<Mapping::PoseGraph::Node>& poseGraphNodes,
                       bool drawTrajectory, int trajectoryNodeIdxMin, int trajectoryNodeIdxMax, bool saveMetadata,
                       const std::string& fileName) const;
    // :181-202
    bool SaveLocalMapAndScan(const LocalMapInfo& localMapInfo,
                             const std::vector<Mapping::PoseGraph::Node>& poseGraphNodes,
                             const RobotPose2D<double>& scanPose, const Hip::ScanData& scanData, bool drawTrajectory,
                             bool saveMetadata, const std::string& fileName) const;
    // :205-228
    bool SaveLatestMapAndScan(const GridMapHip& latestMap, const std::vector<Mapping::PoseGraph::Node>& poseGraphNodes,
                              const RobotPose2D<double>& scanPose, const Hip::ScanData& scanData, bool drawTrajectory,
                              int trajectoryNodeIdxMin, int trajectoryNodeIdxMax, bool saveMetadata,
                              const std::string& fileName) const;
    // :231-275 (<fileName>-<window>.png per precomputed map)
    bool SavePrecomputedGridMaps(const LocalMapInfo& localMapInfo,
                                 const std::vector<Mapping::PoseGraph::Node>& poseGraphNodes,
                                 const std::string& fileName) const;

    // a scan to draw: host ranges/angles and its relative sensor pose
    struct ScanView {
        const double* mRanges = nullptr;
        const double* mAngles = nullptr;
        int mNumOfScans = 0;
        RobotPose2D<double> mRelativeSensorPose;
    };
    struct Options {   // MapSaver::Options (H/io/map_saver.hpp)
        bool mDrawTrajectory = false;
        int mTrajectoryNodeIdxMin = 0;
        int mTrajectoryNodeIdxMax = 0;
        bool mDrawScans = false;
        RobotPose2D<double> mScanPose;
        ScanView mScanData;
        bool mSaveMetadata = false;
        std::string mFileName;
    };
    // SaveMapCore's image (:413-463) without writing it: w x h RGB, rows
    // already flipped up-down; false if the map has no allocated patch.
    // actual = GridMap::ComputeActualMapSize (lgs_map_actual_size's layout).
    bool DrawImage(lgs_ctx* ctx, const lgs_map* map, const std::vector<RobotPose2D<double>>& nodePoses,
                   const Options& opt, std::vector<uint8_t>& rgb, int& w, int& h, int actual[12]) const;
    // SaveMapCore (:413-496): <mFileName>.png (+ .json metadata)
    bool SaveMapCore(lgs_ctx* ctx, const lgs_map* map, const std::vector<RobotPose2D<double>>& nodePoses,
                     const Options& saveOptions) const;

private:
    MapSaver() = default;
    bool SaveMapCore(const GridMapHip& gridMap, const std::vector<Mapping::PoseGraph::Node>& poseGraphNodes,
                     const Options& saveOptions) const;
};

// 8-bit RGB PNG (no interlace, filter 0, zlib), `rgb` rows top to bottom
bool WritePngRgb8(const std::string& fileName, const uint8_t* rgb, int w, int h);

}  // namespace IO
}  // namespace Hip
}  // namespace MyLidarGraphSlam
