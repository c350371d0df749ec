// Library-wide C entry points: version and per-thread error reporting.
#include <stdarg.h>

#include <algorithm>

#include "pcx_common.h"

namespace pcx {

static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

int hip_status(hipError_t e, const char* what) {
    set_error("%s: %s", what, hipGetErrorString(e));
    return PCX_EHIP;
}

int num_cus() {  // compute units of the current device (cached per device; 256 on MI355X)
    static int cache[64] = {0};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
    if (!cache[dev]) {
        int n = 0;
        if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
        cache[dev] = n;
    }
    return cache[dev];
}

}  // namespace pcx

extern "C" int pcx_version(void) { return 100; }

extern "C" int pcx_last_error(char* buf, size_t n) {
    size_t len = strlen(pcx::g_err);
    if (buf && n) {
        size_t c = len < n - 1 ? len : n - 1;
        memcpy(buf, pcx::g_err, c);
        buf[c] = 0;
    }
    return (int)len;
}

namespace {
__device__ __forceinline__ uint64_t splitmix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
__global__ void dropout_mask_kernel(float* out, int64_t n, float p, float keep, uint64_t seed, uint64_t off) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint64_t r = splitmix64(seed ^ splitmix64(off + (uint64_t)i));
    float u = (float)(r >> 40) * (1.0f / 16777216.0f);
    out[i] = (u >= p) ? keep : 0.f;
}
}  // namespace

extern "C" int pcx_dropout_masks(float* out, int64_t n, float p, uint64_t seed, uint64_t offset,
                                 hipStream_t stream) {
    using namespace pcx;
    PCX_CHECK_ARG(out || n == 0, "dropout: NULL output");
    PCX_CHECK_ARG(p >= 0.f && p < 1.f, "dropout probability has to be between 0 and 1, but got %f", p);
    if (n == 0) return PCX_OK;
    dropout_mask_kernel<<<ceil_div(n, 256), 256, 0, stream>>>(out, n, p, 1.f / (1.f - p), seed, offset);
    PCX_LAUNCH_CHECK("dropout_mask_kernel");
    return PCX_OK;
}

// HBM probe (bench.py measured_peaks): dst = src, 16 bytes per lane, each lane moving 8 x 16 B of consecutive
// 4 KB blocks per pass (all eight loads issued before the stores), nontemporal; grid = 16 workgroups of 256
// per CU (the best of the variants tools/copy_probe.hip times: 5.68-5.75 TB/s on MI355X).  The achievable streaming rate an HBM-bound kernel is judged against (MI355X_MICROARCH.md: ~6.3 TB/s for
// a float4 copy), in place of torch's copy_.
namespace {
typedef float sc_f4 __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256) void stream_copy_kernel(const sc_f4* __restrict__ src, sc_f4* __restrict__ dst,
                                                         int64_t n4) {
    const int64_t stride = (int64_t)gridDim.x * 2048;
    for (int64_t base = (int64_t)blockIdx.x * 2048 + threadIdx.x; base < n4; base += stride) {
        sc_f4 v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int64_t i = base + 256 * k;
            if (i < n4) v[k] = __builtin_nontemporal_load(src + i);
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int64_t i = base + 256 * k;
            if (i < n4) __builtin_nontemporal_store(v[k], dst + i);
        }
    }
}
}  // namespace

extern "C" int pcx_stream_copy(const void* src, void* dst, size_t bytes, hipStream_t stream) {
    using namespace pcx;
    PCX_CHECK_ARG(src && dst, "stream_copy: NULL buffer");
    PCX_CHECK_ARG(bytes % 16 == 0 && ((uintptr_t)src & 15) == 0 && ((uintptr_t)dst & 15) == 0,
                  "stream_copy: 16-byte aligned buffers and sizes required");
    const int64_t n4 = (int64_t)(bytes / 16);
    if (n4 == 0) return PCX_OK;
    const int64_t blocks = std::min<int64_t>(ceil_div(n4, 2048), (int64_t)16 * num_cus());
    stream_copy_kernel<<<(unsigned)blocks, 256, 0, stream>>>(static_cast<const sc_f4*>(src),
                                                            static_cast<sc_f4*>(dst), n4);
    PCX_LAUNCH_CHECK("stream_copy_kernel");
    return PCX_OK;
}
