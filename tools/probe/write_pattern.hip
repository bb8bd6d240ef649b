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

// read + write: each wave streams its input slice (16 B per lane per step) while writing its output
// slice, in proportion, like a decoder with no compute
__global__ __launch_bounds__(256) void copy_regions(const uint8_t* __restrict__ in, const covt_stream_desc* __restrict__ d,
                                                    const int64_t* __restrict__ nbytes, int64_t n, uint8_t* __restrict__ out,
                                                    int nt, uint32_t* __restrict__ sink) {
    const int64_t sid = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (sid >= n) return;
    const int l = threadIdx.x & 63;
    uint8_t* o = out + d[sid].out_off;
    const uint8_t* ip = in + (d[sid].in_off & ~(uint64_t)15);
    const int64_t nb = nbytes[sid], ib = d[sid].byte_length;
    uint32_t acc = 0;
    int64_t r = 0;
    for (int64_t b = 0; b < nb; b += 1024) {
        // keep the read front proportional to the write front
        const int64_t rt = ib * (b + 1024) / (nb > 0 ? nb : 1);
        for (; r < rt; r += 1024) {
            const int64_t at = r + 16 * l;
            if (at < ib) {
                const i32x4 v = *(const i32x4*)(ip + at);
                acc += (uint32_t)(v.x ^ v.y ^ v.z ^ v.w);
            }
        }
        const int64_t at = b + 16 * l;
        const i32x4 z = {l, (int)acc, 2, 3};
        if (at < nb) {
            if (nt) __builtin_nontemporal_store(z, (i32x4*)(o + at));
            else *(i32x4*)(o + at) = z;
        }
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

extern "C" int probe_copy_regions(const void* d_in, const void* d_desc, const void* d_nbytes, int64_t n, void* d_out,
                                  int nt, void* d_sink, void* stream) {
    const int64_t blocks = (n + 3) / 4;
    hipLaunchKernelGGL(copy_regions, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, (const uint8_t*)d_in,
                       (const covt_stream_desc*)d_desc, (const int64_t*)d_nbytes, n, (uint8_t*)d_out, nt,
                       (uint32_t*)d_sink);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

extern "C" int probe_write_regions(const void* d_desc, const void* d_nbytes, int64_t n, void* d_out, int nt, void* stream) {
    const int64_t blocks = (n + 3) / 4;
    hipLaunchKernelGGL(write_regions, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream,
                       (const covt_stream_desc*)d_desc, (const int64_t*)d_nbytes, n, (uint8_t*)d_out, nt);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

// K consecutive descriptors per wave, one after the other (a wave writing a longer contiguous run when the
// slices are laid out in descriptor order); read+write form, input streamed in proportion per descriptor
__global__ __launch_bounds__(256) void copy_regions_multi(const uint8_t* __restrict__ in, const covt_stream_desc* __restrict__ d,
                                                          const int64_t* __restrict__ nbytes, int64_t n, uint8_t* __restrict__ out,
                                                          int K, uint32_t* __restrict__ sink) {
    const int64_t w = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int l = threadIdx.x & 63;
    uint32_t acc = 0;
    for (int64_t sid = w * K; sid < (w + 1) * K && sid < n; ++sid) {
        uint8_t* o = out + d[sid].out_off;
        const uint8_t* ip = in + (d[sid].in_off & ~(uint64_t)15);
        const int64_t nb = nbytes[sid], ib = d[sid].byte_length;
        int64_t r = 0;
        for (int64_t b = 0; b < nb; b += 1024) {
            const int64_t rt = ib * (b + 1024) / (nb > 0 ? nb : 1);
            for (; r < rt; r += 1024) {
                const int64_t at = r + 16 * l;
                if (at < ib) {
                    const i32x4 v = *(const i32x4*)(ip + at);
                    acc += (uint32_t)(v.x ^ v.y ^ v.z ^ v.w);
                }
            }
            const int64_t at = b + 16 * l;
            const i32x4 z = {l, (int)acc, 2, 3};
            if (at < nb) __builtin_nontemporal_store(z, (i32x4*)(o + at));
        }
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

extern "C" int probe_copy_regions_multi(const void* d_in, const void* d_desc, const void* d_nbytes, int64_t n, void* d_out,
                                        int K, void* d_sink, void* stream) {
    const int64_t waves = (n + K - 1) / K;
    const int64_t blocks = (waves + 3) / 4;
    hipLaunchKernelGGL(copy_regions_multi, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, (const uint8_t*)d_in,
                       (const covt_stream_desc*)d_desc, (const int64_t*)d_nbytes, n, (uint8_t*)d_out, K, (uint32_t*)d_sink);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}
