// Library-wide C entry points: version and per-thread error reporting.
#include <stdarg.h>

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
