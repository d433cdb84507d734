// Dependent-chain latency of v_add_f64 / v_add_f32 (one wave), via wall_clock64 (100 MHz) and clock64.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(double* out, float* outf, long long* t, int n, double x)
{
    double s = x;
    long long c0 = clock64(), w0 = wall_clock64();
    for (int i = 0; i < n; ++i) {
#pragma unroll
        for (int j = 0; j < 16; ++j) s += x * (j + 1);   // constants fold: dependent adds
    }
    long long c1 = clock64(), w1 = wall_clock64();
    float f = (float)x;
    for (int i = 0; i < n; ++i) {
#pragma unroll
        for (int j = 0; j < 16; ++j) f += (float)x * (j + 1);
    }
    long long c2 = clock64(), w2 = wall_clock64();
    if (threadIdx.x == 0) {
        t[0] = c1 - c0; t[1] = w1 - w0; t[2] = c2 - c1; t[3] = w2 - w1;
    }
    out[threadIdx.x] = s;
    outf[threadIdx.x] = f;
}
int main()
{
    double* d; float* f; long long* t;
    hipMalloc(&d, 64 * 8); hipMalloc(&f, 64 * 4); hipMalloc(&t, 32);
    const int n = 10000;
    for (int rep = 0; rep < 3; ++rep) {
        hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, f, t, n, 1e-3);
        long long h[4];
        hipMemcpy(h, t, 32, hipMemcpyDeviceToHost);
        const double adds = 16.0 * n;
        printf("f64 add: %.2f clk/add, %.3f ns/add; f32 add: %.2f clk/add, %.3f ns/add\n", h[0] / adds,
               10.0 * h[1] / adds, h[2] / adds, 10.0 * h[3] / adds);
    }
    return 0;
}
