// Probe: effective shader clock and dependent-LDS-read latency of one lone wave (device plan diagnosis).
// A single wave runs a chain of dependent LDS reads; wall time (s_memrealtime, 100 MHz) and shader
// clocks (s_memtime / clock64) give the clock frequency and cycles per read.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void chain(int n, unsigned long long* out, int busy) {
    __shared__ unsigned idx[1024];
    for (int i = threadIdx.x; i < 1024; i += blockDim.x) idx[i] = (i * 37 + 11) & 1023;
    __syncthreads();
    if (blockIdx.x != 0 && !busy) return;
    const unsigned long long r0 = __builtin_amdgcn_s_memrealtime(), c0 = clock64();
    unsigned j = threadIdx.x & 1023;
    for (int i = 0; i < n; ++i) j = idx[j];
    const unsigned long long r1 = __builtin_amdgcn_s_memrealtime(), c1 = clock64();
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        out[0] = r1 - r0;
        out[1] = c1 - c0;
        out[2] = j;
    }
}

int main() {
    unsigned long long* d;
    hipMalloc(&d, 64);
    unsigned long long h[3];
    for (int busy = 0; busy < 2; ++busy)
        for (int rep = 0; rep < 3; ++rep) {
            const int n = 100000;
            hipLaunchKernelGGL(chain, dim3(busy ? 4096 : 1), dim3(64), 0, 0, n, d, busy);
            hipMemcpy(h, d, 24, hipMemcpyDeviceToHost);
            const double us = h[0] / 100.0;  // 100 MHz
            std::printf("busy=%d rep=%d: %d dependent LDS reads in %.1f us, %llu clocks -> %.2f GHz, %.1f clocks/read, %.1f ns/read\n",
                        busy, rep, n, us, h[1], h[1] / us / 1e3, (double)h[1] / n, us * 1e3 / n);
        }
    return 0;
}
