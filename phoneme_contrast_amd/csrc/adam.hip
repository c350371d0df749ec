// torch.optim.Adam step over one flat fp32 parameter buffer (reference scripts/train.py:129-133:
// Adam(lr, weight_decay) -> coupled L2, betas (0.9, 0.999), eps 1e-8, bias correction).
// Streaming kernel: 16 B per lane per tensor, grid-stride, ~5 x 4 B of HBM traffic per element.
#include "pcx_common.h"

namespace pcx {
namespace {

__device__ __forceinline__ void adam1(float& p, float g, float& m, float& v, float lr_bc1,
                                      float b1, float b2, float inv_sqrt_bc2, float eps, float wd,
                                      float gs) {
    g = g * gs + wd * p;
    m = b1 * m + (1.f - b1) * g;
    v = b2 * v + (1.f - b2) * g * g;
    // torch: denom = sqrt(v) / sqrt(bc2) + eps ; p -= (lr / bc1) * m / denom
    float denom = sqrtf(v) * inv_sqrt_bc2 + eps;
    p -= lr_bc1 * m / denom;
}

__global__ __launch_bounds__(256) void adam_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                   float* __restrict__ m, float* __restrict__ v,
                                                   int64_t n, float lr_bc1, float b1, float b2,
                                                   float inv_sqrt_bc2, float eps, float wd, float gs) {
    const int64_t n4 = n / 4;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n4; e += stride) {
        float4 pp = ld4(p + 4 * e), gg = ld4(g + 4 * e), mm = ld4(m + 4 * e), vv = ld4(v + 4 * e);
        adam1(pp.x, gg.x, mm.x, vv.x, lr_bc1, b1, b2, inv_sqrt_bc2, eps, wd, gs);
        adam1(pp.y, gg.y, mm.y, vv.y, lr_bc1, b1, b2, inv_sqrt_bc2, eps, wd, gs);
        adam1(pp.z, gg.z, mm.z, vv.z, lr_bc1, b1, b2, inv_sqrt_bc2, eps, wd, gs);
        adam1(pp.w, gg.w, mm.w, vv.w, lr_bc1, b1, b2, inv_sqrt_bc2, eps, wd, gs);
        st4(p + 4 * e, pp);
        st4(m + 4 * e, mm);
        st4(v + 4 * e, vv);
    }
    for (int64_t e = 4 * n4 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += stride)
        adam1(p[e], g[e], m[e], v[e], lr_bc1, b1, b2, inv_sqrt_bc2, eps, wd, gs);
}

}  // namespace
}  // namespace pcx

extern "C" int pcx_adam_step(float* p, const float* g, float* m, float* v, int64_t n, int64_t step,
                             float lr, float beta1, float beta2, float eps, float weight_decay,
                             float grad_scale, hipStream_t stream) {
    using namespace pcx;
    PCX_CHECK_ARG(p && g && m && v, "adam: NULL buffer");
    PCX_CHECK_ARG(step >= 1, "adam: step must be >= 1");
    PCX_CHECK_ARG((((uintptr_t)p | (uintptr_t)g | (uintptr_t)m | (uintptr_t)v) & 15) == 0,
                  "adam: buffers must be 16-byte aligned");
    if (n <= 0) return PCX_OK;
    double bc1 = 1.0 - pow((double)beta1, (double)step);
    double bc2 = 1.0 - pow((double)beta2, (double)step);
    int blocks = (int)std::min<int64_t>(2048, std::max<int64_t>(1, (n / 4 + 255) / 256));
    adam_kernel<<<blocks, 256, 0, stream>>>(p, g, m, v, n, (float)(lr / bc1), beta1, beta2,
                                            (float)(1.0 / sqrt(bc2)), eps, weight_decay, grad_scale);
    PCX_LAUNCH_CHECK("adam_kernel");
    return PCX_OK;
}
