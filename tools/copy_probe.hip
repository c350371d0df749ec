// HBM streaming-copy variants (analysis aid for bench.py's measured_peaks): 2 GiB float4 copy, per variant
// (loads in flight per lane U, nontemporal or plain, workgroups per CU G) the best of 5 timed launches.
//   hipcc -O3 --offload-arch=gfx950 tools/copy_probe.hip -o tools/copy_probe && tools/copy_probe
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f4 __attribute__((ext_vector_type(4)));
template <int U, bool NT>
__global__ __launch_bounds__(256) void copyk(const f4* __restrict__ s, f4* __restrict__ d, long n) {
    const long stride = (long)gridDim.x * 256 * U;
    for (long b = (long)blockIdx.x * 256 * U + threadIdx.x; b < n; b += stride) {
        f4 v[U];
#pragma unroll
        for (int k = 0; k < U; ++k) {
            const long i = b + 256 * k;
            if (i < n) v[k] = NT ? __builtin_nontemporal_load(s + i) : s[i];
        }
#pragma unroll
        for (int k = 0; k < U; ++k) {
            const long i = b + 256 * k;
            if (i < n) { if (NT) __builtin_nontemporal_store(v[k], d + i); else d[i] = v[k]; }
        }
    }
}
template <int U, bool NT>
void run(const f4* s, f4* d, long n, int G, int cus) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    const int blocks = G * cus;
    copyk<U, NT><<<blocks, 256>>>(s, d, n);
    float best = 1e9;
    for (int r = 0; r < 5; ++r) {
        hipEventRecord(e0);
        copyk<U, NT><<<blocks, 256>>>(s, d, n);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1);
        if (ms < best) best = ms;
    }
    printf("U %d NT %d G %2d: %.1f GB/s\n", U, (int)NT, G, 2.0 * 16 * n / (best * 1e-3) / 1e9);
}
int main() {
    const long n = (1L << 31) / 16;
    f4 *s, *d;
    if (hipMalloc(&s, n * 16) || hipMalloc(&d, n * 16)) { printf("alloc failed\n"); return 1; }
    hipMemset(s, 0, n * 16); hipMemset(d, 0, n * 16);
    int cus = 0; hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    for (int G : {4, 8, 16, 32}) {
        run<4, true>(s, d, n, G, cus); run<4, false>(s, d, n, G, cus);
        run<8, true>(s, d, n, G, cus); run<8, false>(s, d, n, G, cus);
        run<2, false>(s, d, n, G, cus); run<1, false>(s, d, n, G, cus);
    }
    return 0;
}
