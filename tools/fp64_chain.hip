// Microbenchmark: the latency of a dependent fp64 add
// chain on one wave of gfx950, operands (a) in registers, (b) read from LDS in
// 64-term blocks ahead of the adds (k_linsolve_split's seq_add_staged), for
// 1, 13 and 64 active lanes.  Prints ns per dependent add (s_memrealtime,
// 100 MHz).  Build: hipcc -O3 --offload-arch=gfx950 -ffp-contract=off
// tools/fp64_chain.hip -o tools/fp64_chain
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int kN = 1088;   // 17 blocks of 64 terms (a config-3 scan's 1081 beams)

__global__ void chain_regs(const double* __restrict__ x, double* out, unsigned long long* t, int active, int reps)
{
    const int lane = threadIdx.x;
    double v[64];
#pragma unroll
    for (int q = 0; q < 64; ++q) v[q] = x[q * 64 + lane];
    double s = 0.0;
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    if (lane < active) {
        for (int r = 0; r < reps * (kN / 64); ++r) {
#pragma unroll
            for (int q = 0; q < 64; ++q) s = s + v[q];   // no reassociation (-fno-fast-math): 64 dependent adds
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    out[lane] = s;
    if (lane == 0) {
        t[0] = t0;
        t[1] = t1;
    }
}

__global__ void chain_lds(const double* __restrict__ x, double* out, unsigned long long* t, int active, int reps)
{
    __shared__ double row[kN];
    const int lane = threadIdx.x;
    for (int i = lane; i < kN; i += 64) row[i] = x[i];
    __syncthreads();
    double s = 0.0;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    if (lane < active) {
        for (int r = 0; r < reps; ++r)
            for (int g = 0; g < kN / 64; ++g) {
                const double* b = row + g * 64;
                double2 v[32];
#pragma unroll
                for (int q = 0; q < 32; ++q) v[q] = *(const double2*)(b + 2 * q);
#pragma unroll
                for (int q = 0; q < 32; ++q) {
                    s = s + v[q].x;
                    s = s + v[q].y;
                }
            }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    out[lane] = s;
    if (lane == 0) {
        t[0] = t0;
        t[1] = t1;
    }
}

int main()
{
    double *x, *out;
    unsigned long long* t;
    if (hipMalloc(&x, sizeof(double) * 64 * 64) != hipSuccess || hipMalloc(&out, sizeof(double) * 64) != hipSuccess ||
        hipMalloc(&t, 16) != hipSuccess)
        return 1;
    double hx[64 * 64];
    for (int i = 0; i < 64 * 64; ++i) hx[i] = 1.0 / (i + 3);
    if (hipMemcpy(x, hx, sizeof(hx), hipMemcpyHostToDevice) != hipSuccess) return 1;
    const int reps = 50;   // 50 passes of a 1088-term chain (a 50-iteration refine)
    for (int mode = 0; mode < 2; ++mode)
        for (int active : { 1, 13, 64 }) {
            for (int warm = 0; warm < 2; ++warm) {
                if (mode == 0)
                    hipLaunchKernelGGL(chain_regs, dim3(1), dim3(64), 0, 0, x, out, t, active, reps);
                else
                    hipLaunchKernelGGL(chain_lds, dim3(1), dim3(64), 0, 0, x, out, t, active, reps);
                if (hipDeviceSynchronize() != hipSuccess) return 2;
            }
            unsigned long long ht[2];
            if (hipMemcpy(ht, t, 16, hipMemcpyDeviceToHost) != hipSuccess) return 1;
            const double ns = (double)(ht[1] - ht[0]) * 10.0 / ((double)reps * kN);
            printf("{\"operands\": \"%s\", \"active_lanes\": %d, \"ns_per_dependent_add\": %.3f, \"chain_us_1081\": %.2f}\n",
                   mode == 0 ? "registers" : "lds_blocks_of_64", active, ns, ns * 1081 / 1000.0);
        }
    return 0;
}
