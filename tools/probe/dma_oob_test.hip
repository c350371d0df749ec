#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef __attribute__((address_space(3))) void lds_void;
// buffer_load_dwordx4 ... lds with offsets straddling the range ends: per-dword or per-access bounds check?
__global__ void k(const float* src, float* out, int nrec_floats) {
    __shared__ float lds[256];
    for (int i = threadIdx.x; i < 256; i += 64) lds[i] = -1.f;
    __syncthreads();
    const unsigned lds0 = (unsigned)(uintptr_t)(lds_void*)lds;
    __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(src + 64), (short)0, 4 * nrec_floats, 0x00020000);
    // lane 0: offset -4 bytes (wraps to 0xFFFFFFFC); lane 1: 4 (n-2) (straddles the end); lane 2: 0; lane 3: 4 (n-1)
    int offs[4] = {-4, 4 * (nrec_floats - 2), 0, 4 * (nrec_floats - 1)};
    const unsigned voff = (unsigned)offs[threadIdx.x & 3];
    const unsigned m0 = __builtin_amdgcn_readfirstlane(lds0);
    asm volatile("s_nop 0\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds" :: "v"(voff), "s"(r), "{m0}"(m0) : "memory");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int i = threadIdx.x; i < 256; i += 64) out[i] = lds[i];
}
int main() {
    const int n = 4096;
    std::vector<float> h(n);
    for (int i = 0; i < n; ++i) h[i] = (float)(i - 64);
    float *src, *out;
    (void)hipMalloc(&src, n * 4); (void)hipMalloc(&out, 256 * 4);
    (void)hipMemcpy(src, h.data(), n * 4, hipMemcpyHostToDevice);
    k<<<1, 64>>>(src, out, 100);
    std::vector<float> o(256);
    (void)hipMemcpy(o.data(), out, 256 * 4, hipMemcpyDeviceToHost);
    const char* nm[4] = {"off -4 (cols -1..2)", "off 4(n-2) (n-2..n+1)", "off 0", "off 4(n-1) (n-1..n+2)"};
    for (int l = 0; l < 4; ++l) printf("%s: %g %g %g %g\n", nm[l], o[4 * l], o[4 * l + 1], o[4 * l + 2], o[4 * l + 3]);
    return 0;
}
