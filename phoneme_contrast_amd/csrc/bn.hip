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
        if (a.zero) a.zero[c] = 0.f;
        // dy = g*invstd*(dz - dbeta/N - xhat*dgamma/N),  xhat = (y - mean)*invstd
        float ac = g * f.w;
        a.cf[c] = make_float4(ac, (float)(d0 / a.count), (float)(d1 / a.count) * f.w, f.z);
    }
}

// ---- split finalisers (round 6): one block per channel walked up to 131072 partials (cnn_small L1 / L2) in
// 32 dependent load rounds per pass on 32 CUs, 0.05-0.08 ms per launch; blocks (split, channel) now reduce
// <= SPLIT_R partials each (2 rounds of 4 loads per thread) and a second launch merges the splits per channel
// in split order (deterministic).  A split's result is parked in the first words of its own range of part1
// (forward: n, sum, M2 about the split mean as three float64) or part0 (backward: the two float64 sums):
// those ranges are read by that split's block only, before it writes, and the partials are scratch consumed
// by the finaliser alone.
constexpr int SPLIT_T = 512, SPLIT_R = 4096;

__device__ __forceinline__ void put_d(float* p, double v) {  // 4-byte aligned float64 store (two words)
    const unsigned long long u = __builtin_bit_cast(unsigned long long, v);
    reinterpret_cast<unsigned*>(p)[0] = (unsigned)u;
    reinterpret_cast<unsigned*>(p)[1] = (unsigned)(u >> 32);
}
__device__ __forceinline__ double get_d(const float* p) {
    const unsigned lo = reinterpret_cast<const unsigned*>(p)[0], hi = reinterpret_cast<const unsigned*>(p)[1];
    return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}

__global__ __launch_bounds__(SPLIT_T) void bn_fwd_split_kernel(BnFwdArgs a, int R) {
    __shared__ double red[SPLIT_T];
    const int sp = blockIdx.x, c = blockIdx.y;
    const int i0 = sp * R, i1 = min(a.nblk, i0 + R);
    const float* s0 = a.part0 + (int64_t)c * a.nblk;
    const float* s1 = a.part1 + (int64_t)c * a.nblk;
    constexpr int st = SPLIT_T;
    double sum = 0.0, n = 0.0;
    int i = i0 + threadIdx.x;
    for (; i + 3 * st < i1; i += 4 * st) {
        const float x0 = s0[i], x1 = s0[i + st], x2 = s0[i + 2 * st], x3 = s0[i + 3 * st];
        const float n0 = a.partn[i], n1 = a.partn[i + st], n2 = a.partn[i + 2 * st], n3 = a.partn[i + 3 * st];
        sum += (double)x0 + (double)x1 + (double)x2 + (double)x3;
        n += (double)n0 + (double)n1 + (double)n2 + (double)n3;
    }
    for (; i < i1; i += st) {
        sum += (double)s0[i];
        n += (double)a.partn[i];
    }
    sum = block_sum_d(sum, red);
    n = block_sum_d(n, red);
    const double mean = n > 0 ? sum / n : 0.0;
    auto term = [&](float sv, float mv, float nv) {
        const double nb = (double)nv;
        if (nb <= 0) return 0.0;
        const double d = (double)sv / nb - mean;
        return (double)mv + nb * d * d;
    };
    double m2 = 0.0;
    i = i0 + threadIdx.x;
    for (; i + 3 * st < i1; i += 4 * st) {
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
    for (; i < i1; i += st) m2 += term(s0[i], s1[i], a.partn[i]);
    m2 = block_sum_d(m2, red);  // (its barriers order every read of the range before the writes below)
    if (threadIdx.x == 0) {
        float* o = const_cast<float*>(s1) + i0;
        put_d(o, n);
        put_d(o + 2, sum);
        put_d(o + 4, m2);
    }
}

// merge of the splits of channel c in split order (Chan: M2 = sum M2_s + n_s (mean_s - mean)^2), then the
// coefficients and running statistics exactly as bn_fwd_finalize_kernel
__global__ __launch_bounds__(64) void bn_fwd_merge_kernel(BnFwdArgs a, int R, int S) {
    const int c = blockIdx.x;
    if (threadIdx.x) return;
    const float* s1 = a.part1 + (int64_t)c * a.nblk;
    double n = 0.0, sum = 0.0;
    for (int sp = 0; sp < S; ++sp) {
        n += get_d(s1 + sp * R);
        sum += get_d(s1 + sp * R + 2);
    }
    const double mean = sum / n;
    double m2 = 0.0;
    for (int sp = 0; sp < S; ++sp) {
        const double ns = get_d(s1 + sp * R);
        if (ns <= 0) continue;
        const double d = get_d(s1 + sp * R + 2) / ns - mean;
        m2 += get_d(s1 + sp * R + 4) + ns * d * d;
    }
    const float g = a.gamma ? a.gamma[c] : 1.f;
    const float be = a.beta ? a.beta[c] : 0.f;
    const float bias = a.bias ? a.bias[c] : 0.f;
    const double var = m2 / n;
    const double invstd = 1.0 / sqrt(var + (double)a.eps);
    const float s = (float)(g * invstd);
    a.cf[c] = make_float4(s, (float)(be - mean * g * invstd), (float)mean, (float)invstd);
    if (a.rmean) {
        const double unb = n > 1 ? m2 / (n - 1) : m2;
        a.rmean[c] = (float)((1.0 - a.momentum) * a.rmean[c] + a.momentum * (mean + bias));
        a.rvar[c] = (float)((1.0 - a.momentum) * a.rvar[c] + a.momentum * unb);
    }
    if (c == 0 && a.nbt) a.nbt[0] += 1;
}

__global__ __launch_bounds__(SPLIT_T) void bn_bwd_split_kernel(BnBwdArgs a, int R) {
    __shared__ double red[SPLIT_T];
    const int sp = blockIdx.x, c = blockIdx.y;
    const int i0 = sp * R, i1 = min(a.nblk, i0 + R);
    const float* s0 = a.part0 + (int64_t)c * a.nblk;
    const float* s1 = a.part1 + (int64_t)c * a.nblk;
    constexpr int st = SPLIT_T;
    double d0 = 0.0, d1 = 0.0;
    int i = i0 + threadIdx.x;
    for (; i + 3 * st < i1; i += 4 * st) {
        const float x0 = s0[i], x1 = s0[i + st], x2 = s0[i + 2 * st], x3 = s0[i + 3 * st];
        const float y0 = s1[i], y1 = s1[i + st], y2 = s1[i + 2 * st], y3 = s1[i + 3 * st];
        d0 += (double)x0 + (double)x1 + (double)x2 + (double)x3;
        d1 += (double)y0 + (double)y1 + (double)y2 + (double)y3;
    }
    for (; i < i1; i += st) {
        d0 += (double)s0[i];
        d1 += (double)s1[i];
    }
    d0 = block_sum_d(d0, red);
    d1 = block_sum_d(d1, red);
    if (threadIdx.x == 0) {
        float* o = const_cast<float*>(s0) + i0;
        put_d(o, d0);
        put_d(o + 2, d1);
    }
}

__global__ __launch_bounds__(64) void bn_bwd_merge_kernel(BnBwdArgs a, int R, int S) {
    const int c = blockIdx.x;
    if (threadIdx.x) return;
    const float* s0 = a.part0 + (int64_t)c * a.nblk;
    double d0 = 0.0, d1 = 0.0;
    for (int sp = 0; sp < S; ++sp) {
        d0 += get_d(s0 + sp * R);
        d1 += get_d(s0 + sp * R + 2);
    }
    const float4 f = a.cf_fwd[c];
    const float g = a.gamma ? a.gamma[c] : 1.f;
    if (a.dbeta) a.dbeta[c] = (float)d0;
    if (a.dgamma) a.dgamma[c] = (float)d1;
    if (a.zero) a.zero[c] = 0.f;
    a.cf[c] = make_float4(g * f.w, (float)(d0 / a.count), (float)(d1 / a.count) * f.w, f.z);
}

}  // namespace

// split when a channel has more than two splits' worth of partials (cnn_small L1-L6 forward, the
// Winograd data gradients' backward partials); the few-thousand-partial cases keep one block per channel
static int bn_splits(int nblk) { return nblk > 2 * SPLIT_R ? ceil_div(nblk, SPLIT_R) : 1; }

int launch_bn_fwd_finalize(BnFwdArgs a, hipStream_t s) {
    const int S = a.train && !PCX_AB_BN_NO_SPLIT ? bn_splits(a.nblk) : 1;
    if (S > 1) {
        const int R = ceil_div(a.nblk, S);
        bn_fwd_split_kernel<<<dim3(S, a.C), SPLIT_T, 0, s>>>(a, R);
        PCX_LAUNCH_CHECK("bn_fwd_split_kernel");
        bn_fwd_merge_kernel<<<a.C, 64, 0, s>>>(a, R, S);
        PCX_LAUNCH_CHECK("bn_fwd_merge_kernel");
        return PCX_OK;
    }
    bn_fwd_finalize_kernel<<<a.C, a.train ? 1024 : 64, 0, s>>>(a);
    PCX_LAUNCH_CHECK("bn_fwd_finalize_kernel");
    return PCX_OK;
}

int launch_bn_bwd_finalize(BnBwdArgs a, hipStream_t s) {
    const int S = !PCX_AB_BN_NO_SPLIT ? bn_splits(a.nblk) : 1;
    if (S > 1) {
        const int R = ceil_div(a.nblk, S);
        bn_bwd_split_kernel<<<dim3(S, a.C), SPLIT_T, 0, s>>>(a, R);
        PCX_LAUNCH_CHECK("bn_bwd_split_kernel");
        bn_bwd_merge_kernel<<<a.C, 64, 0, s>>>(a, R, S);
        PCX_LAUNCH_CHECK("bn_bwd_merge_kernel");
        return PCX_OK;
    }
    bn_bwd_finalize_kernel<<<a.C, 1024, 0, s>>>(a);
    PCX_LAUNCH_CHECK("bn_bwd_finalize_kernel");
    return PCX_OK;
}

}  // namespace pcx
