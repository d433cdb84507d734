// lgs_io.cpp -- Carmen log reader, MapSaver (PNG + JSON), see lgs_io.hpp.
#include "lgs_io.hpp"

#include <zlib.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <climits>
#include <fstream>
#include <limits>
#include <sstream>
#include <stdexcept>

namespace MyLidarGraphSlam {
namespace Hip {

Hip::ScanDataPtr Sensor::ScanData::Upload(DevicePtr dev) const
{
    return std::make_shared<Hip::ScanData>(std::move(dev), mAngles, mRanges, mRelPose, mMinRange, mMaxRange);
}

namespace IO {
namespace Carmen {

// ---------------------------------------------------------------------------
// CarmenLogReader (C/io/carmen/carmen_reader.cpp)
// ---------------------------------------------------------------------------
bool CarmenLogReader::Load(std::istream& in, std::vector<Sensor::SensorDataPtr>& sensorData)
{
    // :11-42.  The sensor id lives across lines: a line whose first extraction
    // fails (empty or blank) is read again as the previous record type, as in
    // the reference.
    sensorData.clear();
    ParamMapType paramMap;
    std::string line, sensorId;
    while (std::getline(in, line)) {
        std::istringstream str{ line };
        if (!str) continue;
        str >> sensorId;
        ReadLine(sensorId, ToDataType(sensorId), str, paramMap, sensorData);
    }
    return true;
}

void CarmenLogReader::ReadLine(const std::string& sensorId, DataType type, std::istringstream& str,
                               ParamMapType& paramMap, std::vector<Sensor::SensorDataPtr>& out)
{
    // :45-109
    switch (type) {
    case DataType::Param: ReadParameter(str, paramMap); break;
    case DataType::Odom: out.emplace_back(ReadOdometryData(sensorId, str)); break;
    case DataType::RawLaser: out.emplace_back(ReadRawLaserData(sensorId, str)); break;
    case DataType::RobotLaser: out.emplace_back(ReadRobotLaserData(sensorId, str)); break;
    case DataType::OldFrontLaser:
    case DataType::OldRearLaser: out.emplace_back(ReadOldLaserData(sensorId, str, paramMap, true)); break;
    case DataType::OldOtherLaser: out.emplace_back(ReadOldLaserData(sensorId, str, paramMap, false)); break;
    default: break;
    }
}

void CarmenLogReader::ReadParameter(std::istringstream& str, ParamMapType& paramMap)
{
    // :112-132 (the first value of a name is kept: unordered_map::insert)
    if (!str) return;
    std::string name, value;
    str >> name;
    if (str) str >> value;
    paramMap.insert(std::make_pair(name, value));
}

namespace {

struct Header {
    std::string host;
    double ipcTime = 0.0, loggerTime = 0.0;
};

void read_header(std::istringstream& str, Header& h) { str >> h.ipcTime >> h.host >> h.loggerTime; }

void read_values(std::istringstream& str, int n, std::vector<double>& v)
{
    v.reserve(static_cast<std::size_t>(std::max(0, n)));
    double x = 0.0;
    for (int i = 0; i < n; ++i) {
        str >> x;
        v.emplace_back(x);
    }
}

std::vector<double> beam_angles(double start, double step, int n)
{
    std::vector<double> a;
    a.reserve(static_cast<std::size_t>(std::max(0, n)));
    for (int i = 0; i < n; ++i) a.emplace_back(start + step * i);
    return a;
}

}  // namespace

Sensor::OdometryDataPtr CarmenLogReader::ReadOdometryData(const std::string& sensorId, std::istringstream& str)
{
    // :135-160: x y theta tv rv accel ipc_time host logger_time
    Header h;
    RobotPose2D<double> pose(0.0, 0.0, 0.0), vel(0.0, 0.0, 0.0);
    double accel = 0.0;
    str >> pose.mX >> pose.mY >> pose.mTheta;
    str >> vel.mX >> vel.mTheta;
    str >> accel;
    read_header(str, h);
    return std::make_shared<Sensor::OdometryData>(sensorId, h.ipcTime, pose, vel);
}

Sensor::ScanDataPtr CarmenLogReader::ReadRawLaserData(const std::string& sensorId, std::istringstream& str)
{
    // :163-236: type start fov res maxRange accuracy remission n ranges[n] m remissions[m] header
    Header h;
    int laserType = 0, remissionMode = 0, n = 0, m = 0;
    double start = 0.0, fov = 0.0, res = 0.0, maxRange = 0.0, accuracy = 0.0, rem = 0.0;
    str >> laserType >> start >> fov >> res >> maxRange >> accuracy >> remissionMode;
    str >> n;
    if (n < 0) throw std::length_error("CarmenLogReader: negative number of readings");
    std::vector<double> ranges;
    read_values(str, n, ranges);
    str >> m;
    for (int i = 0; i < m; ++i) str >> rem;
    read_header(str, h);
    const double maxAngle = start + res * static_cast<double>(n - 1);
    const RobotPose2D<double> zero(0.0, 0.0, 0.0);
    return std::make_shared<Sensor::ScanData>(sensorId, h.ipcTime, zero, zero, zero, 0.0, maxRange, start, maxAngle,
                                              beam_angles(start, res, n), std::move(ranges));
}

Sensor::ScanDataPtr CarmenLogReader::ReadRobotLaserData(const std::string& sensorId, std::istringstream& str)
{
    // :239-316: ... ranges[n] laser pose, robot pose, tv rv, safety fields, header
    Header h;
    int laserType = 0, remissionMode = 0, n = 0;
    double start = 0.0, fov = 0.0, res = 0.0, maxRange = 0.0, accuracy = 0.0;
    RobotPose2D<double> laser(0.0, 0.0, 0.0), robot(0.0, 0.0, 0.0), vel(0.0, 0.0, 0.0);
    double fwd = 0.0, side = 0.0, turn = 0.0;
    str >> laserType >> start >> fov >> res >> maxRange >> accuracy >> remissionMode;
    str >> n;
    if (n < 0) throw std::length_error("CarmenLogReader: negative number of readings");
    std::vector<double> ranges;
    read_values(str, n, ranges);
    str >> laser.mX >> laser.mY >> laser.mTheta;
    str >> robot.mX >> robot.mY >> robot.mTheta;
    str >> vel.mX >> vel.mTheta;
    str >> fwd >> side >> turn;
    read_header(str, h);
    const double maxAngle = start + res * static_cast<double>(n - 1);
    return std::make_shared<Sensor::ScanData>(sensorId, h.ipcTime, robot, vel, Mapping::InverseCompound(robot, laser),
                                              0.0, maxRange, start, maxAngle, beam_angles(start, res, n),
                                              std::move(ranges));
}

Sensor::ScanDataPtr CarmenLogReader::ReadOldLaserData(const std::string& sensorId, std::istringstream& str,
                                                      const ParamMapType& paramMap, bool withPoses)
{
    // FLASER / RLASER (:319-394, withPoses) and LASER3/4 (:397-460): n ranges[n]
    // [laser pose, robot pose, header]; geometry from the PARAM records or guessed
    Header h;
    int n = 0;
    RobotPose2D<double> laser(0.0, 0.0, 0.0), robot(0.0, 0.0, 0.0);
    str >> n;
    if (n < 0) throw std::length_error("CarmenLogReader: negative number of readings");
    std::vector<double> ranges;
    read_values(str, n, ranges);
    if (withPoses) {
        str >> laser.mX >> laser.mY >> laser.mTheta;
        str >> robot.mX >> robot.mY >> robot.mTheta;
        read_header(str, h);
    }
    const auto minR = paramMap.find("Laser.MinRange");
    const double minRange = (minR != paramMap.end()) ? std::stod(minR->second) : 0.0;
    const auto maxR = paramMap.find("Laser.MaxRange");
    const double maxRange = (maxR != paramMap.end()) ? std::stod(maxR->second) : 80.0;
    const auto inc = paramMap.find("Laser.AngleIncrement");
    const double angleIncrement = (inc != paramMap.end()) ? std::stod(inc->second) : GuessAngleIncrement(n);
    const auto minA = paramMap.find("Laser.MinAngle");
    const double minAngle = (minA != paramMap.end()) ? std::stod(minA->second) : (-M_PI_2);
    const auto maxA = paramMap.find("Laser.MaxAngle");
    const double maxAngle = (maxA != paramMap.end()) ? std::stod(maxA->second)
                            : (inc != paramMap.end()) ? minAngle + angleIncrement * static_cast<double>(n)
                                                      : minAngle + GuessAngleRange(n);
    const RobotPose2D<double> zero(0.0, 0.0, 0.0);
    return std::make_shared<Sensor::ScanData>(sensorId, h.ipcTime, withPoses ? robot : zero, zero,
                                              withPoses ? Mapping::InverseCompound(robot, laser) : zero, minRange,
                                              maxRange, minAngle, maxAngle, beam_angles(minAngle, angleIncrement, n),
                                              std::move(ranges));
}

double CarmenLogReader::GuessAngleRange(int n)
{
    // :463-481
    switch (n) {
    case 181: return M_PI;
    case 180: return M_PI * 179.0 / 180.0;
    case 361: return M_PI;
    case 360: return M_PI * 179.5 / 180.0;
    case 401: return M_PI * 100.0 / 180.0;
    case 400: return M_PI * 99.75 / 180.0;
    default: return M_PI;
    }
}

double CarmenLogReader::GuessAngleIncrement(int n)
{
    // :484-503
    switch (n) {
    case 181:
    case 180: return M_PI / 180.0;
    case 361:
    case 360: return M_PI / 360.0;
    case 401:
    case 400: return M_PI / 720.0;
    default: return CarmenLogReader::GuessAngleRange(n) / static_cast<double>(n - 1);
    }
}

CarmenLogReader::DataType CarmenLogReader::ToDataType(const std::string& s)
{
    // :506-530
    static const std::unordered_map<std::string, DataType> kTypes{
        { "PARAM", DataType::Param },          { "ODOM", DataType::Odom },
        { "TRUEPOS", DataType::TruePos },      { "RAWLASER1", DataType::RawLaser },
        { "RAWLASER2", DataType::RawLaser },   { "RAWLASER3", DataType::RawLaser },
        { "RAWLASER4", DataType::RawLaser },   { "ROBOTLASER1", DataType::RobotLaser },
        { "ROBOTLASER2", DataType::RobotLaser }, { "FLASER", DataType::OldFrontLaser },
        { "RLASER", DataType::OldRearLaser },  { "LASER3", DataType::OldOtherLaser },
        { "LASER4", DataType::OldOtherLaser },
    };
    const auto it = kTypes.find(s);
    return (it != kTypes.end()) ? it->second : DataType::None;
}

}  // namespace Carmen

// ---------------------------------------------------------------------------
// JSON the way boost::property_tree::write_json prints a ptree
// ---------------------------------------------------------------------------
namespace {

struct PTree {
    std::string data;
    std::vector<std::pair<std::string, PTree>> children;

    PTree& walk(const std::string& path)   // ptree::put / add_child path creation
    {
        PTree* t = this;
        size_t pos = 0;
        while (true) {
            const size_t dot = path.find('.', pos);
            const std::string key = path.substr(pos, dot == std::string::npos ? std::string::npos : dot - pos);
            PTree* next = nullptr;
            for (auto& c : t->children)
                if (c.first == key) {
                    next = &c.second;
                    break;
                }
            if (!next) {
                t->children.emplace_back(key, PTree{});
                next = &t->children.back().second;
            }
            t = next;
            if (dot == std::string::npos) return *t;
            pos = dot + 1;
        }
    }
    template <typename T> void put(const std::string& path, const T& v) { walk(path).data = str(v); }
    void add_child(const std::string& path, const PTree& child)
    {
        const size_t dot = path.rfind('.');
        PTree& parent = (dot == std::string::npos) ? *this : walk(path.substr(0, dot));
        parent.children.emplace_back(dot == std::string::npos ? path : path.substr(dot + 1), child);
    }
    void push_back(const PTree& child) { children.emplace_back("", child); }

    // boost's stream translator: floating point with max_digits10 digits
    static std::string str(double v)
    {
        std::ostringstream o;
        o.precision(std::numeric_limits<double>::max_digits10);
        o << v;
        return o.str();
    }
    template <typename T> static std::string str(const T& v)
    {
        std::ostringstream o;
        o << v;
        return o.str();
    }
};

std::string escape(const std::string& s)
{
    std::string o;
    for (unsigned char c : s) {
        if (c == 0x20 || c == 0x21 || (c >= 0x23 && c <= 0x2E) || (c >= 0x30 && c <= 0x5B) || c >= 0x5D) {
            o.push_back((char)c);
        } else if (c == '\b') o += "\\b";
        else if (c == '\f') o += "\\f";
        else if (c == '\n') o += "\\n";
        else if (c == '\r') o += "\\r";
        else if (c == '\t') o += "\\t";
        else if (c == '/') o += "\\/";
        else if (c == '"') o += "\\\"";
        else if (c == '\\') o += "\\\\";
        else {
            char buf[8];
            std::snprintf(buf, sizeof buf, "\\u%04X", (unsigned)c);
            o += buf;
        }
    }
    return o;
}

void write_json_node(std::ostream& os, const PTree& t, int indent)
{
    if (indent > 0 && t.children.empty()) {
        os << '"' << escape(t.data) << '"';
        return;
    }
    const bool array = indent > 0 && std::all_of(t.children.begin(), t.children.end(),
                                                 [](const std::pair<std::string, PTree>& c) { return c.first.empty(); });
    os << (array ? '[' : '{') << '\n';
    for (size_t i = 0; i < t.children.size(); ++i) {
        os << std::string(4 * (indent + 1), ' ');
        if (!array) os << '"' << escape(t.children[i].first) << "\": ";
        write_json_node(os, t.children[i].second, indent + 1);
        if (i + 1 < t.children.size()) os << ',';
        os << '\n';
    }
    os << std::string(4 * indent, ' ') << (array ? ']' : '}');
}

bool write_json(const std::string& fileName, const PTree& t)
{
    std::ofstream f(fileName);
    if (!f) return false;
    write_json_node(f, t, 0);
    f << std::endl;
    return (bool)f;
}

inline int world_to_cell(double p, double minPos, double res) { return (int)std::floor((p - minPos) / res); }

// Bresenham (H/util.hpp:256-303): start cell first, then one cell per step
// along the major axis (|2dx| > |2dy|, else y), error init dMinor - dMajor/2
void bresenham(int x0, int y0, int x1, int y1, std::vector<std::pair<int, int>>& out)
{
    out.clear();
    const int sx = (x1 - x0 < 0) ? -1 : 1, sy = (y1 - y0 < 0) ? -1 : 1;
    const int dx = std::abs((x1 - x0) * 2), dy = std::abs((y1 - y0) * 2);
    int x = x0, y = y0;
    out.emplace_back(x, y);
    if (dx > dy) {
        for (int err = dy - dx / 2; x != x1;) {
            if (err >= 0) y += sy, err -= dx;
            x += sx, err += dy;
            out.emplace_back(x, y);
        }
    } else {
        for (int err = dx - dy / 2; y != y1;) {
            if (err >= 0) x += sx, err -= dy;
            y += sy, err += dx;
            out.emplace_back(x, y);
        }
    }
}

inline void fill_block(std::vector<uint8_t>& rgb, int w, int h, int x, int y, int s, uint8_t r, uint8_t g, uint8_t b)
{
    for (int yy = y; yy < y + s; ++yy)
        for (int xx = x; xx < x + s; ++xx) {
            if (xx < 0 || xx >= w || yy < 0 || yy >= h) continue;
            uint8_t* p = &rgb[3 * ((size_t)yy * w + xx)];
            p[0] = r, p[1] = g, p[2] = b;
        }
}

void put_u32(std::vector<uint8_t>& v, uint32_t x)
{
    v.push_back((uint8_t)(x >> 24)), v.push_back((uint8_t)(x >> 16)), v.push_back((uint8_t)(x >> 8)),
        v.push_back((uint8_t)x);
}

void put_chunk(std::vector<uint8_t>& png, const char* type, const uint8_t* data, size_t n)
{
    put_u32(png, (uint32_t)n);
    const size_t at = png.size();
    png.insert(png.end(), type, type + 4);
    if (n) png.insert(png.end(), data, data + n);
    put_u32(png, (uint32_t)crc32(0L, png.data() + at, (uInt)(n + 4)));
}

}  // namespace

bool WritePngRgb8(const std::string& fileName, const uint8_t* rgb, int w, int h)
{
    if (w <= 0 || h <= 0) return false;
    std::vector<uint8_t> raw((size_t)h * (1 + 3 * (size_t)w));
    for (int y = 0; y < h; ++y) {
        uint8_t* row = &raw[(size_t)y * (1 + 3 * (size_t)w)];
        row[0] = 0;   // filter type None
        std::memcpy(row + 1, rgb + (size_t)y * 3 * w, 3 * (size_t)w);
    }
    uLongf zn = compressBound((uLong)raw.size());
    std::vector<uint8_t> z(zn);
    if (compress2(z.data(), &zn, raw.data(), (uLong)raw.size(), Z_DEFAULT_COMPRESSION) != Z_OK) return false;
    std::vector<uint8_t> png = { 0x89, 'P', 'N', 'G', '\r', '\n', 0x1a, '\n' };
    uint8_t ihdr[13];
    const uint32_t W = (uint32_t)w, H = (uint32_t)h;
    ihdr[0] = W >> 24, ihdr[1] = W >> 16, ihdr[2] = W >> 8, ihdr[3] = W;
    ihdr[4] = H >> 24, ihdr[5] = H >> 16, ihdr[6] = H >> 8, ihdr[7] = H;
    ihdr[8] = 8, ihdr[9] = 2, ihdr[10] = 0, ihdr[11] = 0, ihdr[12] = 0;   // 8-bit RGB
    put_chunk(png, "IHDR", ihdr, 13);
    put_chunk(png, "IDAT", z.data(), zn);
    put_chunk(png, "IEND", nullptr, 0);
    std::ofstream f(fileName, std::ios::binary);
    if (!f) return false;
    f.write((const char*)png.data(), (std::streamsize)png.size());
    return (bool)f;
}

// ---------------------------------------------------------------------------
// MapSaver (C/io/map_saver.cpp)
// ---------------------------------------------------------------------------
MapSaver* MapSaver::Instance()
{
    static MapSaver theInstance;
    return &theInstance;
}

namespace {

void check(lgs_ctx* ctx, int status, const char* what)
{
    if (status != LGS_OK) throw Error(status, std::string(what) + ": " + lgs_ctx_last_error(ctx));
}

std::vector<RobotPose2D<double>> poses_of(const std::vector<Mapping::PoseGraph::Node>& nodes)
{
    std::vector<RobotPose2D<double>> p;
    p.reserve(nodes.size());
    for (const auto& n : nodes) p.push_back(n.Pose());
    return p;
}

MapSaver::ScanView view_of(const Hip::ScanData& s)
{
    MapSaver::ScanView v;
    v.mRanges = s.Ranges().data();
    v.mAngles = s.Angles().data();
    v.mNumOfScans = (int)s.NumOfScans();
    v.mRelativeSensorPose = s.RelativeSensorPose();
    return v;
}

}  // namespace

bool MapSaver::DrawImage(lgs_ctx* ctx, const lgs_map* map, const std::vector<RobotPose2D<double>>& nodes,
                         const Options& opt, std::vector<uint8_t>& rgb, int& w, int& h, int a[12]) const
{
    int allocated = 0;
    check(ctx, lgs_map_actual_size(ctx, map, &allocated, a), "lgs_map_actual_size");
    if (!allocated) return false;   // the reference's bounds are INT_MAX/INT_MIN here
    w = a[10], h = a[11];
    const int gx0 = a[4], gy0 = a[5], gx1 = a[6], gy1 = a[7];
    // DrawMap (:278-317) of the actual map size on the device, rows bottom-up
    std::vector<uint8_t> gray((size_t)w * h);
    check(ctx, lgs_map_render_gray_region(ctx, map, gx0, gy0, w, h, 0, gray.data()), "lgs_map_render_gray_region");
    std::vector<uint8_t> img((size_t)w * h * 3);
    for (size_t i = 0; i < gray.size(); ++i) img[3 * i] = img[3 * i + 1] = img[3 * i + 2] = gray[i];
    lgs_map_geometry g{};
    check(ctx, lgs_map_get_geometry(map, &g), "lgs_map_get_geometry");
    std::vector<std::pair<int, int>> line;
    if (opt.mDrawTrajectory) {
        // DrawTrajectory (:320-362): 2x2 red dots along the Bresenham lines
        // between consecutive nodes
        const int lo = opt.mTrajectoryNodeIdxMin, hi = opt.mTrajectoryNodeIdxMax;
        if (lo < 0 || lo >= (int)nodes.size() || hi < 0 || hi >= (int)nodes.size())
            throw Error(LGS_ERR_INVALID_ARG, "MapSaver: trajectory node index out of range");
        int px = world_to_cell(nodes[lo].mX, g.min_x, g.resolution);
        int py = world_to_cell(nodes[lo].mY, g.min_y, g.resolution);
        for (int i = lo + 1; i <= hi; ++i) {
            const int cx = world_to_cell(nodes[i].mX, g.min_x, g.resolution);
            const int cy = world_to_cell(nodes[i].mY, g.min_y, g.resolution);
            bresenham(px, py, cx, cy, line);
            for (const auto& c : line) {
                if (c.first < gx0 || c.first >= gx1 - 1 || c.second < gy0 || c.second >= gy1 - 1) continue;
                fill_block(img, w, h, c.first - gx0, c.second - gy0, 2, 255, 0, 0);
            }
            px = cx, py = cy;
        }
    }
    if (opt.mDrawScans) {
        // DrawScan (:365-410): a 3x3 green pose marker (the reference bounds its
        // y index by gridCellIdxMax.mX, :380) and 2x2 blue hit points
        const int sx = world_to_cell(opt.mScanPose.mX, g.min_x, g.resolution);
        const int sy = world_to_cell(opt.mScanPose.mY, g.min_y, g.resolution);
        if (sx >= gx0 && sx < gx1 - 2 && sy >= gy0 && sy < gx1 - 2)
            fill_block(img, w, h, sx - gx0, sy - gy0, 3, 0, 255, 0);
        const ScanView& sv = opt.mScanData;
        const RobotPose2D<double> sp = Mapping::Compound(opt.mScanPose, sv.mRelativeSensorPose);
        for (int i = 0; i < sv.mNumOfScans; ++i) {
            double sinT, cosT;
            sincos(sp.mTheta + sv.mAngles[i], &sinT, &cosT);   // ScanData::HitPoint (H/sensor/sensor_data.hpp:162-173)
            const int ix = world_to_cell(sp.mX + sv.mRanges[i] * cosT, g.min_x, g.resolution);
            const int iy = world_to_cell(sp.mY + sv.mRanges[i] * sinT, g.min_y, g.resolution);
            if (ix < gx0 || ix >= gx1 - 1 || iy < gy0 || iy >= gy1 - 1) continue;
            fill_block(img, w, h, ix - gx0, iy - gy0, 2, 0, 0, 255);
        }
    }
    // flipped_up_down_view (:455-462)
    rgb.resize(img.size());
    for (int y = 0; y < h; ++y)
        std::memcpy(&rgb[(size_t)y * w * 3], &img[(size_t)(h - 1 - y) * w * 3], (size_t)w * 3);
    return true;
}

bool MapSaver::SaveMapCore(lgs_ctx* ctx, const lgs_map* map, const std::vector<RobotPose2D<double>>& nodes,
                           const Options& opt) const
{
    // :413-496
    std::vector<uint8_t> rgb;
    int w = 0, h = 0, a[12];
    if (!DrawImage(ctx, map, nodes, opt, rgb, w, h, a)) return false;
    if (!WritePngRgb8(opt.mFileName + ".png", rgb.data(), w, h)) return false;
    if (!opt.mSaveMetadata) return true;
    // SaveMapMetadata (:499-532): corners by GridCellIndexToWorldCoordinate (H/grid_map/grid_map.hpp:766-775)
    lgs_map_geometry g{};
    check(ctx, lgs_map_get_geometry(map, &g), "lgs_map_get_geometry");
    const double blx = g.min_x + g.resolution * a[4], bly = g.min_y + g.resolution * a[5];
    const double trx = g.min_x + g.resolution * a[6], try_ = g.min_y + g.resolution * a[7];
    PTree t;
    t.put("Map.Resolution", g.resolution);
    t.put("Map.PatchSize", g.patch_size);
    t.put("Map.WidthInPatches", a[8]);
    t.put("Map.HeightInPatches", a[9]);
    t.put("Map.WidthInGridCells", a[10]);
    t.put("Map.HeightInGridCells", a[11]);
    t.put("Map.BottomLeft.X", blx);
    t.put("Map.BottomLeft.Y", bly);
    t.put("Map.TopRight.X", trx);
    t.put("Map.TopRight.Y", try_);
    t.put("Map.PoseGraphNodeIdxMin", static_cast<std::size_t>(opt.mTrajectoryNodeIdxMin));
    t.put("Map.PoseGraphNodeIdxMax", static_cast<std::size_t>(opt.mTrajectoryNodeIdxMax));
    return write_json(opt.mFileName + ".json", t);
}

bool MapSaver::SaveMapCore(const GridMapHip& gridMap, const std::vector<Mapping::PoseGraph::Node>& nodes,
                           const Options& opt) const
{
    return SaveMapCore(gridMap.Dev()->Handle(), gridMap.Handle(), poses_of(nodes), opt);
}

bool MapSaver::SaveMap(const GridMapHip& globalMap, const std::vector<Mapping::PoseGraph::Node>& nodes,
                       const std::string& fileName, bool drawTrajectory, bool saveMetadata) const
{
    if (nodes.empty()) throw std::invalid_argument("MapSaver::SaveMap: pose graph is empty");   // :39-40
    Options o;
    o.mDrawTrajectory = drawTrajectory;
    o.mTrajectoryNodeIdxMin = 0;
    o.mTrajectoryNodeIdxMax = (int)nodes.size() - 1;
    o.mSaveMetadata = saveMetadata;
    o.mFileName = fileName;
    return SaveMapCore(globalMap, nodes, o);
}

bool MapSaver::SavePoseGraph(const std::vector<Mapping::PoseGraph::Node>& nodes,
                             const std::vector<Mapping::PoseGraph::Edge>& edges, const std::string& fileName) const
{
    // :56-120
    PTree root, nodesTree, edgesTree;
    for (const auto& node : nodes) {
        PTree n;
        n.put("Index", node.Index());
        n.put("Pose.X", node.Pose().mX);
        n.put("Pose.Y", node.Pose().mY);
        n.put("Pose.Theta", node.Pose().mTheta);
        n.put("TimeStamp", node.TimeStamp());
        nodesTree.push_back(n);
    }
    root.add_child("PoseGraph.Nodes", nodesTree);
    for (const auto& edge : edges) {
        PTree e, info;
        e.put("StartNodeIdx", edge.StartNodeIndex());
        e.put("EndNodeIdx", edge.EndNodeIndex());
        e.put("RelativePose.X", edge.RelativePose().mX);
        e.put("RelativePose.Y", edge.RelativePose().mY);
        e.put("RelativePose.Theta", edge.RelativePose().mTheta);
        for (int i = 0; i < 3; ++i)   // upper triangle, row by row
            for (int j = i; j < 3; ++j) {
                PTree v;
                v.data = PTree::str(edge.InformationMatrix()(i, j));
                info.push_back(v);
            }
        e.add_child("InformationMatrix", info);
        edgesTree.push_back(e);
    }
    root.add_child("PoseGraph.Edges", edgesTree);
    return write_json(fileName + ".posegraph.json", root);
}

bool MapSaver::SaveLocalMaps(const std::vector<LocalMapInfo>& localMaps,
                             const std::vector<Mapping::PoseGraph::Node>& nodes, bool drawTrajectory,
                             bool saveMetadata, const std::string& fileName) const
{
    // :123-156
    for (size_t i = 0; i < localMaps.size(); ++i) {
        const auto& lm = localMaps[i];
        Options o;
        o.mDrawTrajectory = drawTrajectory;
        o.mTrajectoryNodeIdxMin = lm.mPoseGraphNodeIdxMin;
        o.mTrajectoryNodeIdxMax = lm.mPoseGraphNodeIdxMax;
        o.mSaveMetadata = saveMetadata;
        o.mFileName = fileName + "-localmap-" + std::to_string(i);
        if (!SaveMapCore(*lm.mMap, nodes, o)) return false;
    }
    return true;
}

bool MapSaver::SaveLatestMap(const GridMapHip& latestMap, const std::vector<Mapping::PoseGraph::Node>& nodes,
                             bool drawTrajectory, int idxMin, int idxMax, bool saveMetadata,
                             const std::string& fileName) const
{
    // :159-178
    Options o;
    o.mDrawTrajectory = drawTrajectory;
    o.mTrajectoryNodeIdxMin = idxMin;
    o.mTrajectoryNodeIdxMax = idxMax;
    o.mSaveMetadata = saveMetadata;
    o.mFileName = fileName + "-latest-map";
    return SaveMapCore(latestMap, nodes, o);
}

bool MapSaver::SaveLocalMapAndScan(const LocalMapInfo& lm, const std::vector<Mapping::PoseGraph::Node>& nodes,
                                   const RobotPose2D<double>& scanPose, const Hip::ScanData& scan,
                                   bool drawTrajectory, bool saveMetadata, const std::string& fileName) const
{
    // :181-202
    Options o;
    o.mDrawTrajectory = drawTrajectory;
    o.mTrajectoryNodeIdxMin = lm.mPoseGraphNodeIdxMin;
    o.mTrajectoryNodeIdxMax = lm.mPoseGraphNodeIdxMax;
    o.mDrawScans = true;
    o.mScanPose = scanPose;
    o.mScanData = view_of(scan);
    o.mSaveMetadata = saveMetadata;
    o.mFileName = fileName;
    return SaveMapCore(*lm.mMap, nodes, o);
}

bool MapSaver::SaveLatestMapAndScan(const GridMapHip& latestMap, const std::vector<Mapping::PoseGraph::Node>& nodes,
                                    const RobotPose2D<double>& scanPose, const Hip::ScanData& scan,
                                    bool drawTrajectory, int idxMin, int idxMax, bool saveMetadata,
                                    const std::string& fileName) const
{
    // :205-228
    Options o;
    o.mDrawTrajectory = drawTrajectory;
    o.mTrajectoryNodeIdxMin = idxMin;
    o.mTrajectoryNodeIdxMax = idxMax;
    o.mDrawScans = true;
    o.mScanPose = scanPose;
    o.mScanData = view_of(scan);
    o.mSaveMetadata = saveMetadata;
    o.mFileName = fileName;
    return SaveMapCore(latestMap, nodes, o);
}

bool MapSaver::SavePrecomputedGridMaps(const LocalMapInfo& lm, const std::vector<Mapping::PoseGraph::Node>&,
                                       const std::string& fileName) const
{
    // :231-275: each precomputed map copied into a fresh occupancy map of the
    // same geometry (GridMap::Update of a fresh cell stores clamp(value),
    // H/grid_map/binary_bayes_grid_cell.hpp:75-82, and allocates its patch),
    // then drawn without trajectory, scans or metadata.  The pyramid is on the
    // device; it is read back once per map (host work off the hot path).
    const lgs_map_geometry g = lm.mMap->Geometry();
    const int ps = g.patch_size;
    for (const auto& pm : lm.mPrecomputedMaps) {
        const DeviceGrid& grid = *pm.second;
        if (grid.NumCellsX() != g.num_cells_x || grid.NumCellsY() != g.num_cells_y)
            throw std::invalid_argument("MapSaver: precomputed map geometry differs from its local map");
        const std::vector<double> cells = grid.Download();
        const int W = g.num_cells_x, npx = g.num_patches_x, npy = g.num_patches_y;
        std::vector<uint8_t> alloc((size_t)npx * npy, 0);
        for (int y = 0; y < g.num_cells_y; ++y)
            for (int x = 0; x < W; ++x)
                if (cells[(size_t)y * W + x] != 0.0) alloc[(size_t)(y / ps) * npx + x / ps] = 1;
        int pminx = INT_MAX, pminy = INT_MAX, pmaxx = INT_MIN, pmaxy = INT_MIN;
        for (int y = 0; y < npy; ++y)
            for (int x = 0; x < npx; ++x)
                if (alloc[(size_t)y * npx + x]) {
                    pminx = std::min(pminx, x), pminy = std::min(pminy, y);
                    pmaxx = std::max(pmaxx, x), pmaxy = std::max(pmaxy, y);
                }
        if (pmaxx < 0) return false;   // nothing allocated: undefined in the reference
        const int w = (pmaxx + 1 - pminx) * ps, h = (pmaxy + 1 - pminy) * ps;
        std::vector<uint8_t> rgb((size_t)w * h * 3, 192);
        for (int py = pminy; py <= pmaxy; ++py)
            for (int px = pminx; px <= pmaxx; ++px) {
                if (!alloc[(size_t)py * npx + px]) continue;
                for (int yy = 0; yy < ps; ++yy)
                    for (int xx = 0; xx < ps; ++xx) {
                        const double raw = cells[(size_t)(py * ps + yy) * W + px * ps + xx];
                        if (raw == 0.0) continue;   // never updated: Unknown
                        const double v = (raw < 1e-3) ? 1e-3 : (0.999 < raw) ? 0.999 : raw;
                        const uint8_t gray = (uint8_t)((1.0 - v) * 255.0);
                        const int iy = h - 1 - ((py - pminy) * ps + yy);   // flipped
                        uint8_t* p = &rgb[3 * ((size_t)iy * w + (size_t)((px - pminx) * ps + xx))];
                        p[0] = p[1] = p[2] = gray;
                    }
            }
        const int winSize = 1 << pm.first;
        if (!WritePngRgb8(fileName + "-" + std::to_string(winSize) + ".png", rgb.data(), w, h)) return false;
    }
    return true;
}

}  // namespace IO
}  // namespace Hip
}  // namespace MyLidarGraphSlam
