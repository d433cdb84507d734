// k_raycast.hip -- K3: Bresenham ray-cast + binary Bayes occupancy update on MI355X,
// and the reference's GridMap geometry (patches, Resize/Expand) around it.
//
// Restates GridMapBuilder's integration loop (C/mapping/grid_map_builder.cpp:167-186
// and :292-329): per beam, the cells of Bresenham(sensorCell, hitCell) minus the
// last are updated with pMiss, then the hit cell with pHit
// (BinaryBayesGridCell::Update, H/grid_map/binary_bayes_grid_cell.hpp:75-119).
// The update is order-dependent (clamped odds products), so the device keeps the
// reference's order exactly:
//
//   host       hit points with glibc sin/cos (bit-exact), bounding box, map
//              geometry (Expand/Resize), sensor/hit cells, ray lengths + offsets
//   k_emit     one thread per ray walks Bresenham (H/util.hpp:256-303) and emits
//              a 64-bit key (cell << 32 | ray << 1 | is_hit) per visited cell;
//              a ray visits a cell at most once, so (cell, ray) is unique
//   sort       hipcub radix sort on the key: each cell's updates become a
//              contiguous run ordered by ray = the reference's update order
//   k_apply    one thread per run applies the Bayes updates sequentially and
//              counts hits/misses
#include "lgs_internal.hpp"

#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cfloat>
#include <cstring>

using namespace lgs;

struct lgs_map {
    lgs_ctx* ctx = nullptr;
    int device = 0;
    double res = 0;
    int ps = 0;
    int npx = 0, npy = 0;
    int w = 0, h = 0;
    double min_x = 0, min_y = 0;
    double* d_cells = nullptr;
    uint32_t* d_hit = nullptr;
    uint32_t* d_miss = nullptr;
    lgs_grid view;
};

namespace {

constexpr double kPMin = 1e-3;
constexpr double kPMax = 1.0 - kPMin;

__device__ __forceinline__ double clampv(double v, double lo, double hi)
{
    return (v < lo) ? lo : (hi < v) ? hi : v;  // std::clamp
}

// BinaryBayesGridCell::Update (H/grid_map/binary_bayes_grid_cell.hpp:75-119)
__device__ __forceinline__ double bayes_update(double v, double p)
{
    if (v == 0.0) return clampv(p, kPMin, kPMax);
    const double co = clampv(v, kPMin, kPMax);
    const double cp = clampv(p, kPMin, kPMax);
    const double o = (co / (1.0 - co)) * (cp / (1.0 - cp));
    return clampv(clampv(o / (1.0 + o), kPMin, kPMax), kPMin, kPMax);
}

struct Ray {
    int sx, sy, hx, hy;
};

// One thread per ray: Bresenham walk (H/util.hpp:256-303), start cell
// inclusive, end (hit) cell last.
__global__ __launch_bounds__(64) void k_emit(const int4* __restrict__ rays,
                                             const long long* __restrict__ offs, int nrays,
                                             int W, int H, unsigned long long* __restrict__ keys,
                                             int* __restrict__ outside)
{
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= nrays) return;
    const int4 ry = rays[r];
    unsigned long long* out = keys + offs[r];
    int deltaX = ry.z - ry.x;
    int deltaY = ry.w - ry.y;
    const int stepX = (deltaX < 0) ? -1 : 1;
    const int stepY = (deltaY < 0) ? -1 : 1;
    int nx = ry.x, ny = ry.y;
    deltaX = abs(deltaX * 2);
    deltaY = abs(deltaY * 2);
    const unsigned long long tag = (unsigned long long)r << 1;
    int bad = 0;
    auto emit = [&](int x, int y, unsigned long long hit) {
        const bool in = (unsigned)x < (unsigned)W && (unsigned)y < (unsigned)H;
        bad |= !in;
        const unsigned long long cell = in ? (unsigned long long)y * W + x : 0ull;
        *out++ = (cell << 32) | tag | hit;
    };
    if (deltaX > deltaY) {
        int err = deltaY - deltaX / 2;
        while (nx != ry.z) {
            emit(nx, ny, 0ull);
            if (err >= 0) {
                ny += stepY;
                err -= deltaX;
            }
            nx += stepX;
            err += deltaY;
        }
    } else {
        int err = deltaX - deltaY / 2;
        while (ny != ry.w) {
            emit(nx, ny, 0ull);
            if (err >= 0) {
                nx += stepX;
                err -= deltaY;
            }
            ny += stepY;
            err += deltaX;
        }
    }
    emit(nx, ny, 1ull);  // == (hx, hy): the hit cell, updated last
    if (bad) atomicAdd(outside, 1);
}

// One thread per run of equal cells in the sorted keys.  The run is walked in
// batches of 8 keys loaded together (one memory latency per batch instead of
// per key).  BinaryBayesGridCell::Update is applied in order; odds(p) is the
// same constant the reference recomputes every time, and an update that maps
// a saturated value onto itself (v == 1e-3 under a miss with odds(pMiss) <= 1,
// v == 1 - 1e-3 under a hit) is skipped after the kernel has checked on the
// device that it is an exact fixed point -- long runs (cells next to the
// sensor) are mostly such updates.
constexpr int kApplyBatch = 8;

__global__ __launch_bounds__(256) void k_apply(const unsigned long long* __restrict__ keys,
                                               long long n, double* __restrict__ cells,
                                               uint32_t* __restrict__ hits,
                                               uint32_t* __restrict__ misses, double p_hit,
                                               double p_miss)
{
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const unsigned long long k = keys[i];
    const unsigned cell = (unsigned)(k >> 32);
    if (i > 0 && (unsigned)(keys[i - 1] >> 32) == cell) return;
    const bool miss_fixed = bayes_update(kPMin, p_miss) == kPMin;
    const bool hit_fixed = bayes_update(kPMax, p_hit) == kPMax;
    double v = cells[cell];
    uint32_t nh = 0, nm = 0;
    for (long long j = i;; j += kApplyBatch) {
        unsigned long long kb[kApplyBatch];
        if (j + kApplyBatch <= n) {
#pragma unroll
            for (int t = 0; t < kApplyBatch; ++t) kb[t] = keys[j + t];
        } else {
#pragma unroll
            for (int t = 0; t < kApplyBatch; ++t) kb[t] = (j + t < n) ? keys[j + t] : ~0ull;
        }
        bool end = false;
#pragma unroll
        for (int t = 0; t < kApplyBatch; ++t) {
            if (!end && (unsigned)(kb[t] >> 32) != cell) end = true;
            if (!end) {
                if (kb[t] & 1ull) {
                    if (!(hit_fixed && v == kPMax)) v = bayes_update(v, p_hit);
                    ++nh;
                } else {
                    if (!(miss_fixed && v == kPMin)) v = bayes_update(v, p_miss);
                    ++nm;
                }
            }
        }
        if (end) break;
    }
    cells[cell] = v;
    hits[cell] += nh;
    misses[cell] += nm;
}

// ---------------------------------------------------------------------------
// host: geometry restated from H/grid_map/grid_map.hpp
// ---------------------------------------------------------------------------
inline void world_to_cell(const lgs_map* m, double x, double y, int& ix, int& iy)
{
    // WorldCoordinateToGridCellIndex (:779-790)
    ix = (int)std::floor((x - m->min_x) / m->res);
    iy = (int)std::floor((y - m->min_y) / m->res);
}

inline int cell_to_patch(int idx, int ps) { return (idx < 0) ? (idx / ps - 1) : (idx / ps); }  // :905-915

void map_alloc(lgs_map* m, int w, int h, double** cells, uint32_t** hit, uint32_t** miss)
{
    const size_t n = std::max<size_t>(1, (size_t)w * (size_t)h);
    *cells = nullptr;
    *hit = *miss = nullptr;
    if (hipMalloc(cells, n * sizeof(double)) != hipSuccess ||
        hipMalloc(hit, n * sizeof(uint32_t)) != hipSuccess ||
        hipMalloc(miss, n * sizeof(uint32_t)) != hipSuccess) {
        hipFree(*cells);
        hipFree(*hit);
        throw Error(LGS_ERR_OOM, "hipMalloc failed for map");
    }
    hipStream_t st = m->ctx->stream;
    LGS_HIP_CHECK(hipMemsetAsync(*cells, 0, n * sizeof(double), st));
    LGS_HIP_CHECK(hipMemsetAsync(*hit, 0, n * sizeof(uint32_t), st));
    LGS_HIP_CHECK(hipMemsetAsync(*miss, 0, n * sizeof(uint32_t), st));
}

void map_sync_view(lgs_map* m)
{
    m->view.ctx = m->ctx;
    m->view.device = m->device;
    m->view.d = m->d_cells;
    m->view.w = m->w;
    m->view.h = m->h;
    m->view.min_x = m->min_x;
    m->view.min_y = m->min_y;
    m->view.res = m->res;
    m->view.owned = false;
    m->view.map_view = true;
}

// Resize (:652-711): patches overlapping the new range keep their cells.
void map_resize(lgs_map* m, double minX, double minY, double maxX, double maxY)
{
    int cminx, cminy, cmaxx, cmaxy;
    world_to_cell(m, minX, minY, cminx, cminy);
    world_to_cell(m, maxX, maxY, cmaxx, cmaxy);
    const int ps = m->ps;
    const int pminx = cell_to_patch(cminx, ps), pminy = cell_to_patch(cminy, ps);
    const int pmaxx = cell_to_patch(cmaxx, ps), pmaxy = cell_to_patch(cmaxy, ps);
    const int npx = std::max(0, pmaxx - pminx + 1);
    const int npy = std::max(0, pmaxy - pminy + 1);
    const int nw = npx * ps, nh = npy * ps;
    double* cells;
    uint32_t *hit, *miss;
    map_alloc(m, nw, nh, &cells, &hit, &miss);
    const int x0 = std::max(0, pminx), y0 = std::max(0, pminy);
    const int x1 = std::min(m->npx, pmaxx + 1), y1 = std::min(m->npy, pmaxy + 1);
    if (x1 > x0 && y1 > y0) {
        const size_t cw = (size_t)(x1 - x0) * ps, ch = (size_t)(y1 - y0) * ps;
        const size_t ox = (size_t)x0 * ps, oy = (size_t)y0 * ps;
        const size_t nx = (size_t)(x0 - pminx) * ps, ny = (size_t)(y0 - pminy) * ps;
        hipStream_t st = m->ctx->stream;
        LGS_HIP_CHECK(hipMemcpy2DAsync(cells + ny * nw + nx, nw * sizeof(double),
                                       m->d_cells + oy * m->w + ox, m->w * sizeof(double),
                                       cw * sizeof(double), ch, hipMemcpyDeviceToDevice, st));
        LGS_HIP_CHECK(hipMemcpy2DAsync(hit + ny * nw + nx, nw * sizeof(uint32_t),
                                       m->d_hit + oy * m->w + ox, m->w * sizeof(uint32_t),
                                       cw * sizeof(uint32_t), ch, hipMemcpyDeviceToDevice, st));
        LGS_HIP_CHECK(hipMemcpy2DAsync(miss + ny * nw + nx, nw * sizeof(uint32_t),
                                       m->d_miss + oy * m->w + ox, m->w * sizeof(uint32_t),
                                       cw * sizeof(uint32_t), ch, hipMemcpyDeviceToDevice, st));
    }
    LGS_HIP_CHECK(hipStreamSynchronize(m->ctx->stream));
    hipFree(m->d_cells);
    hipFree(m->d_hit);
    hipFree(m->d_miss);
    m->d_cells = cells;
    m->d_hit = hit;
    m->d_miss = miss;
    m->npx = npx;
    m->npy = npy;
    m->w = nw;
    m->h = nh;
    m->min_x += (pminx * ps) * m->res;
    m->min_y += (pminy * ps) * m->res;
    map_sync_view(m);
}

bool map_inside(const lgs_map* m, double x, double y)
{
    int ix, iy;
    world_to_cell(m, x, y, ix, iy);
    return (ix >= 0 && ix < m->w) && (iy >= 0 && iy < m->h);
}

// Expand (:714-736)
void map_expand(lgs_map* m, double minX, double minY, double maxX, double maxY, double step)
{
    if (map_inside(m, minX, minY) && map_inside(m, maxX, maxY)) return;
    double minPX = m->min_x + m->res * 0, minPY = m->min_y + m->res * 0;
    double maxPX = m->min_x + m->res * m->w, maxPY = m->min_y + m->res * m->h;
    minPX = (minX < minPX) ? minX - step : minPX;
    minPY = (minY < minPY) ? minY - step : minPY;
    maxPX = (maxX > maxPX) ? maxX + step : maxPX;
    maxPY = (maxY > maxPY) ? maxY + step : maxPY;
    map_resize(m, minPX, minPY, maxPX, maxPY);
}

void map_reset(lgs_map* m)
{
    const size_t n = std::max<size_t>(1, (size_t)m->w * (size_t)m->h);
    hipStream_t st = m->ctx->stream;
    LGS_HIP_CHECK(hipMemsetAsync(m->d_cells, 0, n * sizeof(double), st));
    LGS_HIP_CHECK(hipMemsetAsync(m->d_hit, 0, n * sizeof(uint32_t), st));
    LGS_HIP_CHECK(hipMemsetAsync(m->d_miss, 0, n * sizeof(uint32_t), st));
}

inline double smin(double a, double b) { return (b < a) ? b : a; }  // std::min
inline double smax(double a, double b) { return (a < b) ? b : a; }  // std::max

struct ScanHits {
    lgs_pose2d sensor;
    std::vector<double> xy;  // hit points (x, y) of the usable beams, beam order
};

// ComputeBoundingBoxAndScanPoints hit points (:335-380), glibc sin/cos
ScanHits scan_hits(const lgs_scan* s, lgs_pose2d robot, const lgs_builder_params* bp)
{
    ScanHits h;
    h.sensor = compound(robot, s->rel);
    const double minRange = smax(bp->usable_range_min, s->min_range);
    const double maxRange = smin(bp->usable_range_max, s->max_range);
    h.xy.reserve(2 * (size_t)s->n);
    for (int i = 0; i < s->n; ++i) {
        const double r = s->h_ranges[i];
        if (r >= maxRange || r <= minRange) continue;
        double sn, c;
        ref_sincos(h.sensor.theta + s->h_angles[i], sn, c);
        h.xy.push_back(h.sensor.x + r * c);
        h.xy.push_back(h.sensor.y + r * sn);
    }
    return h;
}

// Ray-cast the given scans (already in the map's geometry) in order.
void raycast(lgs_map* m, const std::vector<ScanHits>& scans, const lgs_builder_params* bp)
{
    lgs_ctx* ctx = m->ctx;
    hipStream_t st = ctx->stream;
    std::vector<int4> rays;
    std::vector<long long> offs;
    long long total = 0;
    for (const ScanHits& h : scans) {
        int sx, sy;
        world_to_cell(m, h.sensor.x, h.sensor.y, sx, sy);
        for (size_t k = 0; k + 1 < h.xy.size(); k += 2) {
            int hx, hy;
            world_to_cell(m, h.xy[k], h.xy[k + 1], hx, hy);
            rays.push_back(make_int4(sx, sy, hx, hy));
            offs.push_back(total);
            total += std::max(std::abs(hx - sx), std::abs(hy - sy)) + 1;
        }
    }
    const int nrays = (int)rays.size();
    if (nrays == 0) return;
    LGS_REQUIRE((size_t)m->w * m->h < (1ull << 32), "map too large for 32-bit cell keys");
    int4* d_rays = (int4*)ctx->ensure(S_RAY0, sizeof(int4) * nrays);
    long long* d_offs = (long long*)ctx->ensure(S_RAY1, sizeof(long long) * nrays);
    unsigned long long* d_keys = (unsigned long long*)ctx->ensure(S_RAY2, sizeof(unsigned long long) * total);
    unsigned long long* d_sorted = (unsigned long long*)ctx->ensure(S_RAY3, sizeof(unsigned long long) * total);
    int* d_bad = (int*)ctx->ensure(S_RAY4, 16);
    // stage rays + offsets through pinned memory (async copy)
    const size_t rb = sizeof(int4) * nrays, ob = sizeof(long long) * nrays;
    char* pin = (char*)ctx->ensure_pinned(rb + ob + 64);
    std::memcpy(pin, rays.data(), rb);
    std::memcpy(pin + rb, offs.data(), ob);
    LGS_HIP_CHECK(hipMemcpyAsync(d_rays, pin, rb, hipMemcpyHostToDevice, st));
    LGS_HIP_CHECK(hipMemcpyAsync(d_offs, pin + rb, ob, hipMemcpyHostToDevice, st));
    LGS_HIP_CHECK(hipMemsetAsync(d_bad, 0, sizeof(int), st));
    // algorithmic bytes: 8 B per emitted key (emit), 8 B key +
    // 16 B cell read/write per update (apply)
    int tok = ctx->timing_begin(K_RAY_EMIT, 8.0 * (double)total);
    hipLaunchKernelGGL(k_emit, dim3((nrays + 63) / 64), dim3(64), 0, st, d_rays, d_offs, nrays, m->w,
                       m->h, d_keys, d_bad);
    ctx->timing_end(tok);
    LGS_HIP_CHECK(hipGetLastError());
    int cell_bits = 1;
    while (cell_bits < 32 && (1ull << cell_bits) < (unsigned long long)m->w * m->h) ++cell_bits;
    size_t tbytes = 0;
    LGS_HIP_CHECK(hipcub::DeviceRadixSort::SortKeys(nullptr, tbytes, d_keys, d_sorted, (int)total, 0,
                                                    32 + cell_bits, st));
    void* temp = ctx->ensure(S_RAY5, tbytes);
    LGS_HIP_CHECK(hipcub::DeviceRadixSort::SortKeys(temp, tbytes, d_keys, d_sorted, (int)total, 0,
                                                    32 + cell_bits, st));
    tok = ctx->timing_begin(K_RAY_APPLY, 24.0 * (double)total);
    hipLaunchKernelGGL(k_apply, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, d_sorted, total,
                       m->d_cells, m->d_hit, m->d_miss, bp->prob_hit, bp->prob_miss);
    ctx->timing_end(tok);
    LGS_HIP_CHECK(hipGetLastError());
    int bad = 0;
    LGS_HIP_CHECK(hipMemcpyAsync(pin, d_bad, sizeof(int), hipMemcpyDeviceToHost, st));
    ctx->sync();
    if (ctx->profile) ctx->harvest();
    std::memcpy(&bad, pin, sizeof(int));
    if (bad) throw Error(LGS_ERR_INTERNAL, "ray cell outside the map geometry");
}

}  // namespace

extern "C" int lgs_map_create(lgs_ctx* ctx, double res, int ps, int ncx, int ncy, double cx, double cy,
                              lgs_map** out)
{
    if (!ctx || !out) return LGS_ERR_INVALID_ARG;
    *out = nullptr;
    return guarded(ctx, [&] {
        LGS_REQUIRE(res > 0.0 && ps > 0, "invalid map resolution / patch size");
        LGS_HIP_CHECK(hipSetDevice(ctx->device));
        // GridMap(res, patchSize, numCellsX, numCellsY, centerPos) (:337-391)
        lgs_map* m = new lgs_map();
        m->ctx = ctx;
        m->device = ctx->device;
        m->res = res;
        m->ps = ps;
        ncx = std::max(0, ncx);
        ncy = std::max(0, ncy);
        m->npx = (int)std::ceil((double)ncx / (double)ps);
        m->npy = (int)std::ceil((double)ncy / (double)ps);
        m->w = m->npx * ps;
        m->h = m->npy * ps;
        const double offX = (m->w % 2 == 0) ? (double)(m->w / 2) : ((double)(m->w / 2) + 0.5);
        const double offY = (m->h % 2 == 0) ? (double)(m->h / 2) : ((double)(m->h / 2) + 0.5);
        m->min_x = cx - offX * res;
        m->min_y = cy - offY * res;
        try {
            map_alloc(m, m->w, m->h, &m->d_cells, &m->d_hit, &m->d_miss);
        } catch (...) {
            delete m;
            throw;
        }
        map_sync_view(m);
        *out = m;
    });
}

extern "C" void lgs_map_destroy(lgs_map* m)
{
    if (!m) return;
    hipSetDevice(m->device);
    hipFree(m->d_cells);
    hipFree(m->d_hit);
    hipFree(m->d_miss);
    delete m;
}

extern "C" int lgs_map_get_geometry(const lgs_map* m, lgs_map_geometry* g)
{
    if (!m || !g) return LGS_ERR_INVALID_ARG;
    g->resolution = m->res;
    g->patch_size = m->ps;
    g->num_patches_x = m->npx;
    g->num_patches_y = m->npy;
    g->num_cells_x = m->w;
    g->num_cells_y = m->h;
    g->min_x = m->min_x;
    g->min_y = m->min_y;
    return LGS_OK;
}

extern "C" int lgs_map_grid(lgs_map* m, lgs_grid** out)
{
    if (!m || !out) return LGS_ERR_INVALID_ARG;
    *out = &m->view;
    return LGS_OK;
}

extern "C" int lgs_map_update_scan(lgs_ctx* ctx, lgs_map* m, const lgs_scan* scan, lgs_pose2d robot,
                                   const lgs_builder_params* bp)
{
    if (!ctx || !m || !scan || !bp) return LGS_ERR_INVALID_ARG;
    return guarded(ctx, [&] {
        LGS_HIP_CHECK(hipSetDevice(ctx->device));
        m->ctx = ctx;
        std::vector<ScanHits> hs(1, scan_hits(scan, robot, bp));
        // bounding box starts at the sensor position (:346-352)
        double blx = hs[0].sensor.x, bly = hs[0].sensor.y, trx = blx, try_ = bly;
        for (size_t k = 0; k + 1 < hs[0].xy.size(); k += 2) {
            blx = smin(blx, hs[0].xy[k]);
            bly = smin(bly, hs[0].xy[k + 1]);
            trx = smax(trx, hs[0].xy[k]);
            try_ = smax(try_, hs[0].xy[k + 1]);
        }
        map_expand(m, blx, bly, trx, try_, 5.0);  // :157-158 (default enlargeStep)
        raycast(m, hs, bp);
    });
}

extern "C" int lgs_map_construct_from_scans(lgs_ctx* ctx, lgs_map* m, const lgs_scan* const* scans,
                                            const lgs_pose2d* poses, int n,
                                            const lgs_builder_params* bp)
{
    if (!ctx || !m || !bp || n < 0 || (n > 0 && (!scans || !poses))) return LGS_ERR_INVALID_ARG;
    return guarded(ctx, [&] {
        LGS_HIP_CHECK(hipSetDevice(ctx->device));
        m->ctx = ctx;
        // :234-285 -- note topRight starts at numeric_limits<double>::min()
        double blx = DBL_MAX, bly = DBL_MAX, trx = DBL_MIN, try_ = DBL_MIN;
        std::vector<ScanHits> hs;
        hs.reserve(n);
        for (int k = 0; k < n; ++k) {
            hs.push_back(scan_hits(scans[k], poses[k], bp));
            const ScanHits& h = hs.back();
            blx = smin(blx, h.sensor.x);
            bly = smin(bly, h.sensor.y);
            trx = smax(trx, h.sensor.x);
            try_ = smax(try_, h.sensor.y);
            for (size_t q = 0; q + 1 < h.xy.size(); q += 2) {
                blx = smin(blx, h.xy[q]);
                bly = smin(bly, h.xy[q + 1]);
                trx = smax(trx, h.xy[q]);
                try_ = smax(try_, h.xy[q + 1]);
            }
        }
        map_resize(m, blx, bly, trx, try_);  // :288-289
        map_reset(m);                        // :290
        raycast(m, hs, bp);                  // :293-329
    });
}

extern "C" int lgs_map_download(lgs_ctx* ctx, const lgs_map* m, double* cells, uint32_t* hit,
                                uint32_t* miss)
{
    if (!ctx || !m) return LGS_ERR_INVALID_ARG;
    return guarded(ctx, [&] {
        const size_t n = (size_t)m->w * m->h;
        if (!n) return;
        hipStream_t st = ctx->stream;
        if (cells)
            LGS_HIP_CHECK(hipMemcpyAsync(cells, m->d_cells, n * sizeof(double), hipMemcpyDeviceToHost, st));
        if (hit)
            LGS_HIP_CHECK(hipMemcpyAsync(hit, m->d_hit, n * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
        if (miss)
            LGS_HIP_CHECK(hipMemcpyAsync(miss, m->d_miss, n * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
        LGS_HIP_CHECK(hipStreamSynchronize(st));
    });
}
