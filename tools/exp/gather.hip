// Per-wave random-gather rate: one wave per CU (grid = 256), each lane loads
// 16 B at a pseudo-random 32-B aligned offset of a 12 MB buffer; 32 lanes
// share a line pattern like k_coarse_rows (2 lanes per line).  Modes:
// 0 = global_load_dwordx4 into registers, depth D in flight; 1 = global_load_lds
// dwordx4 with counted waits.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef __attribute__((address_space(3))) void lds_void_t;
typedef const __attribute__((address_space(1))) void gbl_void_t;
constexpr unsigned wimm(unsigned vm, unsigned lgkm) { return (vm & 15u) | (7u << 4) | ((lgkm & 15u) << 8) | ((vm >> 4) << 14); }

__device__ __forceinline__ unsigned hsh(unsigned x) { x ^= x >> 16; x *= 0x7feb352d; x ^= x >> 15; x *= 0x846ca68b; x ^= x >> 16; return x; }

template <int MODE>
__global__ __launch_bounds__(64) void k(const double* buf, unsigned nlines, int iters, double* out, long long* t)
{
    extern __shared__ __attribute__((aligned(16))) double lds[];
    const int lane = threadIdx.x;
    double acc = 0;
    const long long w0 = wall_clock64();
    if constexpr (MODE == 0) {
        double4 r[8];
        for (int i = 0; i < iters; i += 8) {
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const unsigned line = hsh((blockIdx.x * 1000003u) ^ ((i + j) * 64 + (lane >> 1))) % nlines;
                const double* p = buf + (size_t)line * 4 + (lane & 1) * 2;
                r[j].x = p[0]; r[j].y = p[1];
            }
#pragma unroll
            for (int j = 0; j < 8; ++j) acc += r[j].x + r[j].y;
        }
    } else {
        constexpr int RING = 12;
        for (int i = 0; i < iters + RING; ++i) {
            if (i >= RING) {
                __builtin_amdgcn_s_waitcnt(wimm(RING - 1, 15));
                acc += lds[((i - RING) % RING) * 128 + lane];
                __builtin_amdgcn_s_waitcnt(wimm(63, 0));
            }
            if (i < iters) {
                const unsigned line = hsh((blockIdx.x * 1000003u) ^ (i * 64 + (lane >> 1))) % nlines;
                const double* p = buf + (size_t)line * 4 + (lane & 1) * 2;
                __builtin_amdgcn_global_load_lds((gbl_void_t*)p, (lds_void_t*)(lds + (i % RING) * 128), 16, 0, 0);
            }
        }
        __builtin_amdgcn_s_waitcnt(wimm(0, 15));
    }
    const long long w1 = wall_clock64();
    out[blockIdx.x * 64 + lane] = acc;
    if (lane == 0) t[blockIdx.x] = w1 - w0;
}

int main()
{
    const size_t bytes = 12u << 20;
    double* buf; double* out; long long* t;
    hipMalloc(&buf, bytes); hipMemset(buf, 0, bytes);
    hipMalloc(&out, 256 * 64 * 8); hipMalloc(&t, 256 * 8);
    const unsigned nlines = bytes / 32;
    const int iters = 512;
    for (int grid : {1, 256}) {
        for (int mode = 0; mode < 2; ++mode) {
            for (int rep = 0; rep < 2; ++rep) {
                if (mode == 0) hipLaunchKernelGGL(k<0>, dim3(grid), dim3(64), 0, 0, buf, nlines, iters, out, t);
                else hipLaunchKernelGGL(k<1>, dim3(grid), dim3(64), 12 * 128 * 8, 0, buf, nlines, iters, out, t);
                hipDeviceSynchronize();
            }
            long long h[256];
            hipMemcpy(h, t, grid * 8, hipMemcpyDeviceToHost);
            double avg = 0; for (int i = 0; i < grid; ++i) avg += h[i]; avg /= grid;
            printf("grid %3d mode %s: %.1f ns per 64-lane 16B gather instruction (%.2f us total)\n", grid,
                   mode ? "glds " : "vgprs", 10.0 * avg / iters, 0.01 * avg);
        }
    }
    return 0;
}
