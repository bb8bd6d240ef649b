// Write-pattern probe (timing experiment, not part of libcovt): each wave owns one descriptor and
// writes its stream's output region front to back in 1 KiB steps (16 B per lane), like the decode
// kernels do, but computes nothing.  Compares the HBM rate of that pattern with a linear fill.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "covt.h"

typedef int32_t i32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void write_regions(const covt_stream_desc* __restrict__ d, const int64_t* __restrict__ nbytes,
                                                     int64_t n, uint8_t* __restrict__ out, int nt) {
    const int64_t sid = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (sid >= n) return;
    const int l = threadIdx.x & 63;
    uint8_t* o = out + d[sid].out_off;
    const int64_t nb = nbytes[sid];
    const i32x4 z = {l, 1, 2, 3};
    for (int64_t b = 0; b < nb; b += 1024) {
        const int64_t at = b + 16 * l;
        if (at < nb) {
            if (nt) __builtin_nontemporal_store(z, (i32x4*)(o + at));
            else *(i32x4*)(o + at) = z;
        }
    }
}

extern "C" int probe_write_regions(const void* d_desc, const void* d_nbytes, int64_t n, void* d_out, int nt, void* stream) {
    const int64_t blocks = (n + 3) / 4;
    hipLaunchKernelGGL(write_regions, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream,
                       (const covt_stream_desc*)d_desc, (const int64_t*)d_nbytes, n, (uint8_t*)d_out, nt);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}
