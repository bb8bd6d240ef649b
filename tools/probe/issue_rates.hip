// Issue-rate probe for gfx950: how many VALU / SALU / mixed wave-instructions a CU retires per
// nanosecond with W waves per SIMD, each wave running independent (non-dependent) instruction
// streams.  Answers whether the decode families' SALU and VALU counts compete for one issue port.
//   hipcc -O3 --offload-arch=gfx950 -o /tmp/issue_rates tools/probe/issue_rates.hip && /tmp/issue_rates
#include <hip/hip_runtime.h>
#include <cstdio>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); return 1; } } while (0)

// MODE 0: 8 independent v_add per step; 1: 8 independent s_add; 2: 8 v_add + 8 s_add interleaved;
// 3: 8 v_add + 4 s_add; 4: dependent chain of v_add (latency); 5: dependent chain of s_add
template <int MODE>
__global__ void __launch_bounds__(256) probe(int* out, int iters) {
    uint32_t v0 = threadIdx.x, v1 = v0 + 1, v2 = v0 + 2, v3 = v0 + 3, v4 = v0 + 4, v5 = v0 + 5, v6 = v0 + 6, v7 = v0 + 7;
    uint32_t s0 = blockIdx.x, s1 = s0 + 1, s2 = s0 + 2, s3 = s0 + 3, s4 = s0 + 4, s5 = s0 + 5, s6 = s0 + 6, s7 = s0 + 7;
    const uint32_t k = iters;
    for (int i = 0; i < iters; ++i) {
#define VA(r) asm volatile("v_add_u32 %0, %0, %1" : "+v"(r) : "v"(k))
#define SA(r) asm volatile("s_mul_i32 %0, %0, %1" : "+s"(r) : "s"(k))
        if (MODE == 0) { VA(v0); VA(v1); VA(v2); VA(v3); VA(v4); VA(v5); VA(v6); VA(v7); }
        if (MODE == 1) { SA(s0); SA(s1); SA(s2); SA(s3); SA(s4); SA(s5); SA(s6); SA(s7); }
        if (MODE == 2) { VA(v0); SA(s0); VA(v1); SA(s1); VA(v2); SA(s2); VA(v3); SA(s3);
                         VA(v4); SA(s4); VA(v5); SA(s5); VA(v6); SA(s6); VA(v7); SA(s7); }
        if (MODE == 3) { VA(v0); VA(v1); SA(s0); VA(v2); VA(v3); SA(s1); VA(v4); VA(v5); SA(s2); VA(v6); VA(v7); SA(s3); }
        if (MODE == 4) { VA(v0); VA(v0); VA(v0); VA(v0); VA(v0); VA(v0); VA(v0); VA(v0); }
        if (MODE == 5) { SA(s0); SA(s0); SA(s0); SA(s0); SA(s0); SA(s0); SA(s0); SA(s0); }
    }
    out[blockIdx.x * 256 + threadIdx.x] = v0 + v1 + v2 + v3 + v4 + v5 + v6 + v7 + s0 + s1 + s2 + s3 + s4 + s5 + s6 + s7;
}

template <int MODE>
static int run(const char* name, int vpi, int spi, int* d, int cus) {
    const int iters = 20000;
    for (int wps : {1, 2, 4, 8}) {  // waves per SIMD: 4 waves per block, one block per SIMD-quad
        const int blocks = cus * wps;  // 4 waves per block -> wps waves on each of the CU's 4 SIMDs
        hipEvent_t a, b;
        CHECK(hipEventCreate(&a));
        CHECK(hipEventCreate(&b));
        probe<MODE><<<blocks, 256>>>(d, 100);
        CHECK(hipEventRecord(a));
        probe<MODE><<<blocks, 256>>>(d, iters);
        CHECK(hipEventRecord(b));
        CHECK(hipEventSynchronize(b));
        float ms = 0;
        CHECK(hipEventElapsedTime(&ms, a, b));
        const double waves = 4.0 * blocks;
        const double vi = waves * iters * vpi, si = waves * iters * spi;
        const double ns = ms * 1e6;
        printf("%-28s waves/SIMD %d: %8.3f ms  VALU %.3f  SALU %.3f  total %.3f wave-instr per CU per ns\n",
               name, wps, ms, vi / cus / ns, si / cus / ns, (vi + si) / cus / ns);
        CHECK(hipEventDestroy(a));
        CHECK(hipEventDestroy(b));
    }
    return 0;
}

int main() {
    hipDeviceProp_t p;
    CHECK(hipGetDeviceProperties(&p, 0));
    const int cus = p.multiProcessorCount;
    printf("CUs %d, clock %d kHz\n", cus, p.clockRate);
    int* d;
    CHECK(hipMalloc(&d, (size_t)cus * 8 * 256 * sizeof(int)));
    if (run<0>("8 indep v_add", 8, 0, d, cus)) return 1;
    if (run<1>("8 indep s_add", 0, 8, d, cus)) return 1;
    if (run<2>("8 v_add + 8 s_add", 8, 8, d, cus)) return 1;
    if (run<3>("8 v_add + 4 s_add", 8, 4, d, cus)) return 1;
    if (run<4>("dependent v_add chain", 8, 0, d, cus)) return 1;
    if (run<5>("dependent s_add chain", 0, 8, d, cus)) return 1;
    CHECK(hipFree(d));
    return 0;
}
