// Dispatch-rate microbenchmark: N tiny kernels spread over S streams.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

__global__ void k_empty(int* p) { if (p && threadIdx.x == 1023) p[0] = 1; }

int main(int argc, char** argv)
{
    const int S = argc > 1 ? atoi(argv[1]) : 1;
    const int N = argc > 2 ? atoi(argv[2]) : 20000;
    const int G = argc > 3 ? atoi(argv[3]) : 1;
    const int B = argc > 4 ? atoi(argv[4]) : 64;
    const int threads = argc > 5 ? atoi(argv[5]) : 0;   // 1 = one host thread per stream
    std::vector<hipStream_t> st(S);
    for (auto& s : st) hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    for (int i = 0; i < 100; ++i) hipLaunchKernelGGL(k_empty, dim3(G), dim3(B), 0, st[i % S], nullptr);
    hipDeviceSynchronize();
    auto t0 = std::chrono::steady_clock::now();
    if (threads) {
        std::vector<std::thread> th;
        for (int s = 0; s < S; ++s)
            th.emplace_back([&, s] {
                for (int i = s; i < N; i += S) hipLaunchKernelGGL(k_empty, dim3(G), dim3(B), 0, st[s], nullptr);
                hipStreamSynchronize(st[s]);
            });
        for (auto& t : th) t.join();
    } else {
        for (int i = 0; i < N; ++i) hipLaunchKernelGGL(k_empty, dim3(G), dim3(B), 0, st[i % S], nullptr);
        hipDeviceSynchronize();
    }
    auto t1 = std::chrono::steady_clock::now();
    const double us = std::chrono::duration<double, std::micro>(t1 - t0).count();
    printf("streams=%d kernels=%d grid=%d block=%d threads=%d: %.2f us/kernel (%.0f kernels/s)\n", S, N, G, B,
           threads, us / N, N / us * 1e6);
    return 0;
}
