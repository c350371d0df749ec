// Probe of __builtin_amdgcn_global_load_lds semantics on gfx950 (dword and dwordx4):
// per-lane global source, LDS destination = wave-uniform base + lane * size.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

template <int SIZE>
__global__ void probe(const float* __restrict__ src, float* __restrict__ out, const int* __restrict__ perm) {
    __shared__ __attribute__((aligned(16))) float lds[1024 * 2];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (int i = threadIdx.x; i < 2048; i += blockDim.x) lds[i] = -1.f;
    __syncthreads();
    // each wave copies 64 "units" (SIZE bytes each) gathered through perm
    const float* g = src + perm[wave * 64 + lane] * (SIZE / 4);
    auto* dst = (void __attribute__((address_space(3)))*)(lds + wave * 64 * (SIZE / 4));
    if constexpr (SIZE == 4) __builtin_amdgcn_global_load_lds((const void*)g, dst, 4, 0, 0);
    else __builtin_amdgcn_global_load_lds((const void*)g, dst, 16, 0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int i = threadIdx.x; i < 4 * 64 * (SIZE / 4); i += blockDim.x) out[i] = lds[i];
}

int main() {
    const int n = 4096;
    float* h = (float*)malloc(n * 4);
    for (int i = 0; i < n; ++i) h[i] = (float)i;
    int hp[256];
    for (int i = 0; i < 256; ++i) hp[i] = (i * 37 + 11) % 256;
    float *d, *o;
    int* p;
    hipMalloc(&d, n * 4); hipMalloc(&o, 2048 * 4); hipMalloc(&p, 256 * 4);
    hipMemcpy(d, h, n * 4, hipMemcpyHostToDevice);
    hipMemcpy(p, hp, 256 * 4, hipMemcpyHostToDevice);
    float ho[2048];
    int bad = 0;
    probe<4><<<1, 256>>>(d, o, p);
    hipMemcpy(ho, o, 256 * 4, hipMemcpyDeviceToHost);
    for (int i = 0; i < 256; ++i) if (ho[i] != (float)hp[i]) { if (bad < 5) printf("dword mismatch %d: %f vs %d\n", i, ho[i], hp[i]); ++bad; }
    printf("dword: %s\n", bad ? "FAIL" : "ok");
    bad = 0;
    probe<16><<<1, 256>>>(d, o, p);
    hipMemcpy(ho, o, 1024 * 4, hipMemcpyDeviceToHost);
    for (int i = 0; i < 1024; ++i) { float want = (float)(hp[i / 4] * 4 + i % 4); if (ho[i] != want) { if (bad < 5) printf("x4 mismatch %d: %f vs %f\n", i, ho[i], want); ++bad; } }
    printf("dwordx4: %s\n", bad ? "FAIL" : "ok");
    hipError_t e = hipDeviceSynchronize();
    printf("status %s\n", hipGetErrorString(e));
    return 0;
}
