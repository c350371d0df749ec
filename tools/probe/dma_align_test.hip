#include <hip/hip_runtime.h>
typedef __attribute__((address_space(3))) void lds_void;
__global__ void k(const float* src, float* out, int mis) {
    __shared__ float lds[1024];
    for (int i = threadIdx.x; i < 1024; i += 64) lds[i] = -1.f;
    __syncthreads();
    const unsigned lds0 = (unsigned)(uintptr_t)(lds_void*)lds;
    const unsigned m0 = __builtin_amdgcn_readfirstlane(lds0);
    const float* g = src + mis + 4 * threadIdx.x;
    asm volatile("s_nop 0\n\tglobal_load_lds_dwordx4 %0, off" :: "v"(g), "{m0}"(m0) : "memory");
    __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(src), (short)0, 1 << 20, 0x00020000);
    const unsigned voff = 4u * (mis + 4 * threadIdx.x);
    const unsigned m1 = __builtin_amdgcn_readfirstlane(lds0 + 1024 * 2);
    asm volatile("s_nop 0\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds" :: "v"(voff), "s"(r), "{m0}"(m1) : "memory");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int i = threadIdx.x; i < 1024; i += 64) out[i] = lds[i];
}
#include <cstdio>
#include <vector>
int main() {
    const int n = 1 << 18;
    std::vector<float> h(n);
    for (int i = 0; i < n; ++i) h[i] = (float)i;
    float *src, *out;
    (void)hipMalloc(&src, n * 4); (void)hipMalloc(&out, 4096 * 4);
    (void)hipMemcpy(src, h.data(), n * 4, hipMemcpyHostToDevice);
    int bad = 0;
    for (int mis = 0; mis < 4; ++mis) {
        k<<<1, 64>>>(src, out, mis);
        std::vector<float> o(1024);
        if (hipMemcpy(o.data(), out, 1024 * 4, hipMemcpyDeviceToHost) != hipSuccess) { printf("copy failed\n"); return 1; }
        int eg = 0, eb = 0;
        for (int i = 0; i < 256; ++i) {
            if (o[i] != (float)(mis + i)) ++eg;
            if (o[512 + i] != (float)(mis + i)) ++eb;
        }
        printf("mis=%d global_lds_x4 errors %d (o[0..3]=%g %g %g %g) buffer_lds_x4 errors %d (o[512..515]=%g %g %g %g)\n", mis, eg,
               o[0], o[1], o[2], o[3], eb, o[512], o[513], o[514], o[515]);
        bad += eg + eb;
    }
    printf(bad ? "UNALIGNED-DMA-BROKEN\n" : "UNALIGNED-DMA-OK\n");
    return 0;
}
