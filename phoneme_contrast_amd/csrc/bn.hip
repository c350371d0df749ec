// Train/eval BatchNorm finalisers (reference nn.BatchNorm2d at src/models/phoneme_cnn.py:37,40,48,
// 51,59,62 and the residual blocks).  The conv kernels leave per-block partial statistics; these
// kernels reduce them in a fixed order in float64 (deterministic, cancellation-safe), update the
// running statistics exactly as torch does (momentum 0.1, unbiased running variance,
// num_batches_tracked += 1) and emit the per-channel coefficients the next kernel's prologue uses.
#include "kernels.h"

namespace pcx {
namespace {

__device__ __forceinline__ double block_sum_d(double v, double* red) {
    const int tid = threadIdx.x;
    red[tid] = v;
    __syncthreads();
    for (int o = blockDim.x / 2; o > 0; o >>= 1) {
        if (tid < o) red[tid] += red[tid + o];
        __syncthreads();
    }
    double r = red[0];
    __syncthreads();
    return r;
}

// one block per channel, 1024 threads, 4 independent loads in flight per thread: the partial
// counts reach 64000 per channel (cnn_small L1/L2), and a 256-thread loop with one outstanding load
// per iteration was memory-latency bound (0.1-0.3 ms per launch)
__global__ __launch_bounds__(1024) void bn_fwd_finalize_kernel(BnFwdArgs a) {
    __shared__ double red[1024];
    const int c = blockIdx.x;
    const float g = a.gamma ? a.gamma[c] : 1.f;
    const float be = a.beta ? a.beta[c] : 0.f;
    const float bias = a.bias ? a.bias[c] : 0.f;
    if (!a.train) {
        if (threadIdx.x == 0) {
            float invstd = 1.f / sqrtf(a.rvar[c] + a.eps);
            float s = g * invstd;
            // stored conv output excludes the bias: y_true = y + bias
            a.cf[c] = make_float4(s, be - (a.rmean[c] - bias) * s, a.rmean[c] - bias, invstd);
        }
        return;
    }
    const float* s0 = a.part0 + (int64_t)c * a.nblk;
    const float* s1 = a.part1 + (int64_t)c * a.nblk;
    double sum = 0.0, n = 0.0;
    {
        const int st = blockDim.x;
        int i = threadIdx.x;
        for (; i + 3 * st < a.nblk; i += 4 * st) {
            const float x0 = s0[i], x1 = s0[i + st], x2 = s0[i + 2 * st], x3 = s0[i + 3 * st];
            const float n0 = a.partn[i], n1 = a.partn[i + st], n2 = a.partn[i + 2 * st], n3 = a.partn[i + 3 * st];
            sum += (double)x0 + (double)x1 + (double)x2 + (double)x3;
            n += (double)n0 + (double)n1 + (double)n2 + (double)n3;
        }
        for (; i < a.nblk; i += st) {
            sum += (double)s0[i];
            n += (double)a.partn[i];
        }
    }
    sum = block_sum_d(sum, red);
    n = block_sum_d(n, red);
    const double mean = sum / n;
    // M2 = sum_b [M2_b + n_b (mean_b - mean)^2]
    double m2 = 0.0;
    {
        const int st = blockDim.x;
        int i = threadIdx.x;
        auto term = [&](float sv, float mv, float nv) {
            const double nb = (double)nv;
            if (nb <= 0) return 0.0;
            const double d = (double)sv / nb - mean;
            return (double)mv + nb * d * d;
        };
        for (; i + 3 * st < a.nblk; i += 4 * st) {
            float sv[4], mv[4], nv[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                sv[u] = s0[i + u * st];
                mv[u] = s1[i + u * st];
                nv[u] = a.partn[i + u * st];
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) m2 += term(sv[u], mv[u], nv[u]);
        }
        for (; i < a.nblk; i += st) m2 += term(s0[i], s1[i], a.partn[i]);
    }
    m2 = block_sum_d(m2, red);
    if (threadIdx.x == 0) {
        double var = m2 / n;
        double invstd = 1.0 / sqrt(var + (double)a.eps);
        float s = (float)(g * invstd);
        a.cf[c] = make_float4(s, (float)(be - mean * g * invstd), (float)mean, (float)invstd);
        if (a.rmean) {
            double unb = n > 1 ? m2 / (n - 1) : m2;
            a.rmean[c] = (float)((1.0 - a.momentum) * a.rmean[c] + a.momentum * (mean + bias));
            a.rvar[c] = (float)((1.0 - a.momentum) * a.rvar[c] + a.momentum * unb);
        }
        if (c == 0 && a.nbt) a.nbt[0] += 1;
    }
}

__global__ __launch_bounds__(1024) void bn_bwd_finalize_kernel(BnBwdArgs a) {
    __shared__ double red[1024];
    const int c = blockIdx.x;
    const float* s0 = a.part0 + (int64_t)c * a.nblk;
    const float* s1 = a.part1 + (int64_t)c * a.nblk;
    double d0 = 0.0, d1 = 0.0;
    for (int i = threadIdx.x; i < a.nblk; i += blockDim.x) {
        d0 += (double)s0[i];
        d1 += (double)s1[i];
    }
    d0 = block_sum_d(d0, red);
    d1 = block_sum_d(d1, red);
    if (threadIdx.x == 0) {
        const float4 f = a.cf_fwd[c];
        const float g = a.gamma ? a.gamma[c] : 1.f;
        if (a.dbeta) a.dbeta[c] = (float)d0;
        if (a.dgamma) a.dgamma[c] = (float)d1;
        // dy = g*invstd*(dz - dbeta/N - xhat*dgamma/N),  xhat = (y - mean)*invstd
        float ac = g * f.w;
        a.cf[c] = make_float4(ac, (float)(d0 / a.count), (float)(d1 / a.count) * f.w, f.z);
    }
}

}  // namespace

int launch_bn_fwd_finalize(BnFwdArgs a, hipStream_t s) {
    bn_fwd_finalize_kernel<<<a.C, a.train ? 1024 : 64, 0, s>>>(a);
    PCX_LAUNCH_CHECK("bn_fwd_finalize_kernel");
    return PCX_OK;
}

int launch_bn_bwd_finalize(BnBwdArgs a, hipStream_t s) {
    bn_bwd_finalize_kernel<<<a.C, 1024, 0, s>>>(a);
    PCX_LAUNCH_CHECK("bn_bwd_finalize_kernel");
    return PCX_OK;
}

}  // namespace pcx
