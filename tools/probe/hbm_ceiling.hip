// HBM ceiling probes (timing experiment, not part of libcovt).  Hand-written grid-stride kernels that
// move the decode launch's byte volumes with no decode at all:
//   k_store  -- 16 B per lane streaming stores over a linear buffer (the 4.5 GB output alone)
//   k_read   -- 16 B per lane streaming loads (the 0.9 GB input alone)
//   k_copy   -- proportional copy: each wave step loads 1 KiB of input and stores R KiB of output
//               (R = 5 for the bench batch: 0.9 GB in, 4.5 GB out)
// Every kernel takes its grid size from the caller so the sweep can find the best occupancy.
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef int32_t i32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void k_store(i32x4* __restrict__ out, int64_t n16, int nt) {
    const int64_t stride = (int64_t)gridDim.x * 256;
    const i32x4 z = {(int)threadIdx.x, 1, 2, 3};
    int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (nt) {
        for (; i + 3 * stride < n16; i += 4 * stride) {
            __builtin_nontemporal_store(z, out + i);
            __builtin_nontemporal_store(z, out + i + stride);
            __builtin_nontemporal_store(z, out + i + 2 * stride);
            __builtin_nontemporal_store(z, out + i + 3 * stride);
        }
        for (; i < n16; i += stride) __builtin_nontemporal_store(z, out + i);
    } else {
        for (; i + 3 * stride < n16; i += 4 * stride) {
            out[i] = z;
            out[i + stride] = z;
            out[i + 2 * stride] = z;
            out[i + 3 * stride] = z;
        }
        for (; i < n16; i += stride) out[i] = z;
    }
}

__global__ __launch_bounds__(256) void k_read(const i32x4* __restrict__ in, int64_t n16, uint32_t* __restrict__ sink) {
    const int64_t stride = (int64_t)gridDim.x * 256;
    uint32_t acc = 0;
    int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    for (; i + 3 * stride < n16; i += 4 * stride) {
        const i32x4 a = in[i], b = in[i + stride], c = in[i + 2 * stride], d = in[i + 3 * stride];
        acc += (uint32_t)(a.x ^ b.y ^ c.z ^ d.w);
    }
    for (; i < n16; i += stride) acc += (uint32_t)in[i].x;
    if (acc == 0x12345678u) sink[0] = acc;
}

// unit u = one wave step: input granules [64u, 64u+64), output granules [64Ru, 64R(u+1))
__global__ __launch_bounds__(256) void k_copy(const i32x4* __restrict__ in, int64_t n_units, int R, i32x4* __restrict__ out,
                                              int nt) {
    const int l = threadIdx.x & 63;
    const int64_t wave = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int64_t nwaves = (int64_t)gridDim.x * 4;
    for (int64_t u = wave; u < n_units; u += nwaves) {
        const i32x4 v = in[u * 64 + l];
        i32x4* o = out + u * 64 * R + l;
        for (int r = 0; r < R; ++r) {
            const i32x4 w = {v.x + r, v.y, v.z, v.w};
            if (nt) __builtin_nontemporal_store(w, o + 64 * r);
            else o[64 * r] = w;
        }
    }
}

// the same copy with D units per wave step: D 16-byte loads in flight per lane before the step's stores
// (k_copy keeps one; VERDICT r04: a probe with one load in flight per lane understates the read side)
template <int D>
__global__ __launch_bounds__(256) void k_copy_d(const i32x4* __restrict__ in, int64_t n_units, int R,
                                                i32x4* __restrict__ out) {
    const int l = threadIdx.x & 63;
    const int64_t wave = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int64_t nwaves = (int64_t)gridDim.x * 4;
    int64_t u = wave * D;
    for (; u + D <= n_units; u += nwaves * D) {
        i32x4 v[D];
#pragma unroll
        for (int d = 0; d < D; ++d) v[d] = __builtin_nontemporal_load(in + (u + d) * 64 + l);
#pragma unroll
        for (int d = 0; d < D; ++d) {
            i32x4* o = out + (u + d) * 64 * R + l;
            for (int r = 0; r < R; ++r) {
                const i32x4 w = {v[d].x + r, v[d].y, v[d].z, v[d].w};
                __builtin_nontemporal_store(w, o + 64 * r);
            }
        }
    }
    for (; u < n_units; ++u) {  // the last partial step (u + D > n_units here: one wave's units)
        const i32x4 v = in[u * 64 + l];
        for (int r = 0; r < R; ++r) __builtin_nontemporal_store(v, out + u * 64 * R + l + 64 * r);
    }
}

extern "C" int probe_copy_depth(const void* in, int64_t n_units, int R, void* out, int depth, int blocks, void* stream) {
    if (depth == 4)
        hipLaunchKernelGGL(k_copy_d<4>, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, (const i32x4*)in,
                           n_units, R, (i32x4*)out);
    else if (depth == 2)
        hipLaunchKernelGGL(k_copy_d<2>, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, (const i32x4*)in,
                           n_units, R, (i32x4*)out);
    else
        return -1;
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

extern "C" int probe_store(void* out, int64_t n16, int nt, int blocks, void* stream) {
    hipLaunchKernelGGL(k_store, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, (i32x4*)out, n16, nt);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

extern "C" int probe_read(const void* in, int64_t n16, void* sink, int blocks, void* stream) {
    hipLaunchKernelGGL(k_read, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, (const i32x4*)in, n16,
                       (uint32_t*)sink);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

extern "C" int probe_copy(const void* in, int64_t n_units, int R, void* out, int nt, int blocks, void* stream) {
    hipLaunchKernelGGL(k_copy, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, (const i32x4*)in, n_units, R,
                       (i32x4*)out, nt);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}
