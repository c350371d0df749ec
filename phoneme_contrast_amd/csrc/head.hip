// Embedding head of PhonemeNet / PhonemeNetDeep (reference src/models/phoneme_cnn.py):
//   x = Dropout2d(ReLU(BN(y)))                       (fused: never materialised)
//   a = sigmoid(conv1x1(x)), x' = x * a              SpatialAttention, :129-143
//   pooled = mean_{h,w} x'                           AdaptiveAvgPool2d(1), :74,116-117
//   e = normalize(BN1d(Linear(pooled)))             :75-77,119-124
// and the backward of all of it.  These are small (per-sample) kernels; the trunk convs dominate.
#include "kernels.h"

namespace pcx {
namespace {

__device__ __forceinline__ float xval(float y, float4 cf, float d) { return d * fmaxf(fmaf(y, cf.x, cf.y), 0.f); }

// one block per sample
__global__ __launch_bounds__(256) void head_pool_fwd_kernel(HeadPoolArgs a) {
    extern __shared__ __attribute__((aligned(16))) float sm[];
    float* att = sm;                // [P]
    float* swa = sm + a.P;          // [C]
    float* sdr = swa + a.C;         // [C]
    float4* scf = reinterpret_cast<float4*>(sdr + a.C + ((4 - ((a.P + 2 * a.C) & 3)) & 3));
    const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const float* yb = a.y + (int64_t)b * a.C * a.P;
    for (int c = tid; c < a.C; c += blockDim.x) {
        scf[c] = a.cf[c];
        sdr[c] = a.drop ? a.drop[(int64_t)b * a.C + c] : 1.f;
        swa[c] = a.wa ? a.wa[c] : 0.f;
    }
    __syncthreads();
    const float ba = a.wa ? a.ba[0] : 0.f;
    for (int p = tid; p < a.P; p += blockDim.x) {
        float v = 1.f;
        if (a.wa) {
            float l = ba;
            for (int c = 0; c < a.C; ++c) l = fmaf(swa[c], xval(yb[(int64_t)c * a.P + p], scf[c], sdr[c]), l);
            v = 1.f / (1.f + expf(-l));
            a.att[(int64_t)b * a.P + p] = v;
        }
        att[p] = v;
    }
    __syncthreads();
    const float invp = 1.f / (float)a.P;
    const int nw = blockDim.x / 64;
    if (a.P <= 64) {  // short planes (3 x 13): 4 channels per step, their loads issued together
        const float at = lane < a.P ? att[lane] : 0.f;
        for (int c0 = wave; c0 < a.C; c0 += 4 * nw) {
            float v[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int c = c0 + j * nw;
                v[j] = (c < a.C && lane < a.P) ? yb[(int64_t)c * a.P + lane] : 0.f;
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int c = c0 + j * nw;
                if (c >= a.C) break;
                const float s = wave_sum(lane < a.P ? xval(v[j], scf[c], sdr[c]) * at : 0.f);
                if (lane == 0) a.pooled[(int64_t)b * a.C + c] = s * invp;
            }
        }
        return;
    }
    for (int c = wave; c < a.C; c += nw) {
        const float* yc = yb + (int64_t)c * a.P;
        float4 cf = scf[c];
        float d = sdr[c];
        float s = 0.f;
        for (int p = lane; p < a.P; p += 64) s = fmaf(xval(yc[p], cf, d), att[p], s);
        s = wave_sum(s);
        if (lane == 0) a.pooled[(int64_t)b * a.C + c] = s * invp;
    }
}

__global__ __launch_bounds__(256) void head_pool_bwd_kernel(HeadPoolArgs a) {
    extern __shared__ __attribute__((aligned(16))) float sm[];
    float* att = sm;                // [P]
    float* dl = sm + a.P;           // [P]
    float* swa = dl + a.P;          // [C]
    float* sdr = swa + a.C;         // [C]
    float* sdp = sdr + a.C;         // [C]
    float4* scf = reinterpret_cast<float4*>(sdp + a.C + ((4 - ((2 * a.P + 3 * a.C) & 3)) & 3));
    __shared__ float red[4];
    const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const float* yb = a.y + (int64_t)b * a.C * a.P;
    const float invp = 1.f / (float)a.P;
    for (int c = tid; c < a.C; c += blockDim.x) {
        scf[c] = a.cf[c];
        sdr[c] = a.drop ? a.drop[(int64_t)b * a.C + c] : 1.f;
        swa[c] = a.wa ? a.wa[c] : 0.f;
        sdp[c] = a.dpooled[(int64_t)b * a.C + c] * invp;
    }
    __syncthreads();
    float dls = 0.f;
    for (int p = tid; p < a.P; p += blockDim.x) {
        float at = 1.f, d = 0.f;
        if (a.wa) {
            at = a.att[(int64_t)b * a.P + p];
            float s = 0.f;
            for (int c = 0; c < a.C; ++c) s = fmaf(sdp[c], xval(yb[(int64_t)c * a.P + p], scf[c], sdr[c]), s);
            d = s * at * (1.f - at);
        }
        att[p] = at;
        dl[p] = d;
        dls += d;
    }
    dls = wave_sum(dls);
    if (lane == 0) red[wave] = dls;
    __syncthreads();
    if (tid == 0 && a.wa) a.p_dba[b] = red[0] + red[1] + red[2] + red[3];
    const int nw = blockDim.x / 64;
    if (a.P <= 64) {  // short planes: 4 channels per step, loads issued together
        const bool on = lane < a.P;
        const float atl = on ? att[lane] : 0.f, dll = on ? dl[lane] : 0.f;
        for (int c0 = wave; c0 < a.C; c0 += 4 * nw) {
            float yv[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int c = c0 + j * nw;
                yv[j] = (c < a.C && on) ? yb[(int64_t)c * a.P + lane] : 0.f;
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int c = c0 + j * nw;
                if (c >= a.C) break;
                const float4 cf = scf[c];
                const float dr = sdr[c], g = sdp[c], wac = swa[c];
                const float y = yv[j], z = fmaf(y, cf.x, cf.y);
                const float dx = fmaf(g, atl, dll * wac);
                const float dz = (on && z > 0.f) ? dx * dr : 0.f;
                if (on) a.dz[((int64_t)b * a.C + c) * a.P + lane] = dz;
                const float sdz = wave_sum(dz);
                const float sdx = wave_sum(on ? dz * ((y - cf.z) * cf.w) : 0.f);
                const float sdw = wave_sum(on ? dll * (dr * fmaxf(z, 0.f)) : 0.f);
                if (lane == 0) {
                    a.p_dz[(int64_t)c * a.B + b] = sdz;
                    a.p_dzx[(int64_t)c * a.B + b] = sdx;
                    if (a.wa) a.p_dwa[(int64_t)c * a.B + b] = sdw;
                }
            }
        }
        return;
    }
    for (int c = wave; c < a.C; c += nw) {
        const float* yc = yb + (int64_t)c * a.P;
        float* dzc = a.dz + ((int64_t)b * a.C + c) * a.P;
        const float4 cf = scf[c];
        const float dr = sdr[c], g = sdp[c], wac = swa[c];
        float sdz = 0.f, sdx = 0.f, sdw = 0.f;
        for (int p = lane; p < a.P; p += 64) {
            float y = yc[p];
            float z = fmaf(y, cf.x, cf.y);
            float dx = fmaf(g, att[p], dl[p] * wac);
            float dz = z > 0.f ? dx * dr : 0.f;
            dzc[p] = dz;
            sdz += dz;
            sdx = fmaf(dz, (y - cf.z) * cf.w, sdx);
            sdw = fmaf(dl[p], dr * fmaxf(z, 0.f), sdw);
        }
        sdz = wave_sum(sdz);
        sdx = wave_sum(sdx);
        sdw = wave_sum(sdw);
        if (lane == 0) {
            a.p_dz[(int64_t)c * a.B + b] = sdz;
            a.p_dzx[(int64_t)c * a.B + b] = sdx;
            if (a.wa) a.p_dwa[(int64_t)c * a.B + b] = sdw;
        }
    }
}

// Register-resident form for the PhonemeNet head (C = 128, P <= 512, P % 4 == 0; the cnn_small
// trunk ends at 128 x 10 x 50): one block of 8 waves holds a whole sample in registers -- wave w
// owns channels 16w .. 16w + 15, lane l the pixel quads 4l + 256k (k < 2) -- so y is read from HBM
// once (16-byte loads) instead of once for the attention logits and again for the pool / dz; the
// cross-channel logit sums and the attention map go through LDS.  Other shapes (the residual
// network's 512 x 3 x 13) take the per-sample kernels above.
constexpr int HR_C = 128, HR_CPW = 16, HR_KP = 2, HR_PMAX = 512;

bool head_reg_fits(const HeadPoolArgs& a) { return a.C == HR_C && a.P % 4 == 0 && a.P <= HR_PMAX; }

__global__ __launch_bounds__(512) void head_pool_fwd_reg_kernel(HeadPoolArgs a) {
    __shared__ __attribute__((aligned(16))) float part[8][HR_PMAX];  // per-wave partial logits
    __shared__ __attribute__((aligned(16))) float att[HR_PMAX];
    const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // (uniform: coefficient loads are scalar)
    const int c0 = wave * HR_CPW, P = a.P;
    const float* yb = a.y + ((int64_t)b * HR_C + c0) * P;
    float4 xv[HR_CPW][HR_KP];
    float4 lg[HR_KP];
#pragma unroll
    for (int k = 0; k < HR_KP; ++k) lg[k] = make_float4(0.f, 0.f, 0.f, 0.f);
    // every y load of the sample first (clamped in bounds, zeroed after): one memory round trip per
    // sample -- computing each channel right after its load had the compiler wait for every load
#pragma unroll
    for (int c = 0; c < HR_CPW; ++c)
#pragma unroll
        for (int k = 0; k < HR_KP; ++k) {
            const int p = 4 * lane + 256 * k;
            xv[c][k] = ld4(yb + (int64_t)c * P + (p < P ? p : 0));
        }
#pragma unroll
    for (int c = 0; c < HR_CPW; ++c) {
        const float4 cf = a.cf[c0 + c];
        const float d = a.drop ? a.drop[(int64_t)b * HR_C + c0 + c] : 1.f;
        const float wa = a.wa ? a.wa[c0 + c] : 0.f;
#pragma unroll
        for (int k = 0; k < HR_KP; ++k) {
            const int p = 4 * lane + 256 * k;
            const float4 y = xv[c][k];
            const float4 x = p < P ? make_float4(xval(y.x, cf, d), xval(y.y, cf, d), xval(y.z, cf, d), xval(y.w, cf, d))
                                   : make_float4(0.f, 0.f, 0.f, 0.f);
            xv[c][k] = x;
            lg[k].x = fmaf(wa, x.x, lg[k].x);
            lg[k].y = fmaf(wa, x.y, lg[k].y);
            lg[k].z = fmaf(wa, x.z, lg[k].z);
            lg[k].w = fmaf(wa, x.w, lg[k].w);
        }
    }
    if (a.wa) {
#pragma unroll
        for (int k = 0; k < HR_KP; ++k) {
            const int p = 4 * lane + 256 * k;
            if (p < P) st4(&part[wave][p], lg[k]);
        }
        __syncthreads();
        const float ba = a.ba[0];
        for (int p = tid; p < P; p += 512) {
            float l = ba;
#pragma unroll
            for (int w = 0; w < 8; ++w) l += part[w][p];
            const float v = 1.f / (1.f + expf(-l));
            att[p] = v;
            a.att[(int64_t)b * P + p] = v;
        }
    } else {
        for (int p = tid; p < P; p += 512) att[p] = 1.f;
    }
    __syncthreads();
    const float invp = 1.f / (float)P;
#pragma unroll
    for (int c = 0; c < HR_CPW; ++c) {
        float sum = 0.f;
#pragma unroll
        for (int k = 0; k < HR_KP; ++k) {
            const int p = 4 * lane + 256 * k;
            if (p < P) {
                const float4 at = *reinterpret_cast<const float4*>(&att[p]);
                sum = fmaf(xv[c][k].x, at.x, sum);
                sum = fmaf(xv[c][k].y, at.y, sum);
                sum = fmaf(xv[c][k].z, at.z, sum);
                sum = fmaf(xv[c][k].w, at.w, sum);
            }
        }
        sum = wave_sum(sum);
        if (lane == 0) a.pooled[(int64_t)b * HR_C + c0 + c] = sum * invp;
    }
}

__global__ __launch_bounds__(512) void head_pool_bwd_reg_kernel(HeadPoolArgs a) {
    __shared__ __attribute__((aligned(16))) float part[8][HR_PMAX];
    __shared__ __attribute__((aligned(16))) float att[HR_PMAX];
    __shared__ __attribute__((aligned(16))) float dl[HR_PMAX];
    __shared__ float red[8];
    const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int c0 = wave * HR_CPW, P = a.P;
    const float invp = 1.f / (float)P;
    const float* yb = a.y + ((int64_t)b * HR_C + c0) * P;
    float4 yv[HR_CPW][HR_KP];
#pragma unroll
    for (int c = 0; c < HR_CPW; ++c)
#pragma unroll
        for (int k = 0; k < HR_KP; ++k) {
            const int p = 4 * lane + 256 * k;
            yv[c][k] = ld4(yb + (int64_t)c * P + (p < P ? p : 0));  // (lanes past P: never used)
        }
    if (a.wa) {  // dl[p] = att (1 - att) sum_c dpooled[c] / P x[c][p]
        float4 sp[HR_KP];
#pragma unroll
        for (int k = 0; k < HR_KP; ++k) sp[k] = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int c = 0; c < HR_CPW; ++c) {
            const float4 cf = a.cf[c0 + c];
            const float d = a.drop ? a.drop[(int64_t)b * HR_C + c0 + c] : 1.f;
            const float g = a.dpooled[(int64_t)b * HR_C + c0 + c] * invp;
#pragma unroll
            for (int k = 0; k < HR_KP; ++k) {
                sp[k].x = fmaf(g, xval(yv[c][k].x, cf, d), sp[k].x);
                sp[k].y = fmaf(g, xval(yv[c][k].y, cf, d), sp[k].y);
                sp[k].z = fmaf(g, xval(yv[c][k].z, cf, d), sp[k].z);
                sp[k].w = fmaf(g, xval(yv[c][k].w, cf, d), sp[k].w);
            }
        }
#pragma unroll
        for (int k = 0; k < HR_KP; ++k) {
            const int p = 4 * lane + 256 * k;
            if (p < P) st4(&part[wave][p], sp[k]);
        }
        __syncthreads();
        float dls = 0.f;
        for (int p = tid; p < P; p += 512) {
            float sum = 0.f;
#pragma unroll
            for (int w = 0; w < 8; ++w) sum += part[w][p];
            const float at = a.att[(int64_t)b * P + p];
            const float d = sum * at * (1.f - at);
            att[p] = at;
            dl[p] = d;
            dls += d;
        }
        dls = wave_sum(dls);
        if (lane == 0) red[wave] = dls;
        __syncthreads();
        if (tid == 0) {
            float t = 0.f;
            for (int w = 0; w < 8; ++w) t += red[w];
            a.p_dba[b] = t;
        }
    } else {
        for (int p = tid; p < P; p += 512) {
            att[p] = 1.f;
            dl[p] = 0.f;
        }
        __syncthreads();
    }
#pragma unroll
    for (int c = 0; c < HR_CPW; ++c) {
        const float4 cf = a.cf[c0 + c];
        const float dr = a.drop ? a.drop[(int64_t)b * HR_C + c0 + c] : 1.f;
        const float g = a.dpooled[(int64_t)b * HR_C + c0 + c] * invp;
        const float wac = a.wa ? a.wa[c0 + c] : 0.f;
        float* dzc = a.dz + ((int64_t)b * HR_C + c0 + c) * P;
        float sdz = 0.f, sdx = 0.f, sdw = 0.f;
#pragma unroll
        for (int k = 0; k < HR_KP; ++k) {
            const int p = 4 * lane + 256 * k;
            if (p < P) {
                const float4 at = *reinterpret_cast<const float4*>(&att[p]);
                const float4 dv = *reinterpret_cast<const float4*>(&dl[p]);
                const float yy[4] = {yv[c][k].x, yv[c][k].y, yv[c][k].z, yv[c][k].w};
                const float aa[4] = {at.x, at.y, at.z, at.w}, ll[4] = {dv.x, dv.y, dv.z, dv.w};
                float dz[4];
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const float z = fmaf(yy[e], cf.x, cf.y);
                    const float dx = fmaf(g, aa[e], ll[e] * wac);
                    dz[e] = z > 0.f ? dx * dr : 0.f;
                    sdz += dz[e];
                    sdx = fmaf(dz[e], (yy[e] - cf.z) * cf.w, sdx);
                    sdw = fmaf(ll[e], dr * fmaxf(z, 0.f), sdw);
                }
                st4(dzc + p, make_float4(dz[0], dz[1], dz[2], dz[3]));
            }
        }
        sdz = wave_sum(sdz);
        sdx = wave_sum(sdx);
        sdw = wave_sum(sdw);
        if (lane == 0) {
            a.p_dz[(int64_t)(c0 + c) * a.B + b] = sdz;
            a.p_dzx[(int64_t)(c0 + c) * a.B + b] = sdx;
            if (a.wa) a.p_dwa[(int64_t)(c0 + c) * a.B + b] = sdw;
        }
    }
}

// --------------------------------------------------------------- projection
constexpr int PR = 16;  // rows per block

// h = pooled @ W^T + bias ; one thread per output feature, 16 rows per block
__global__ __launch_bounds__(256) void proj_fwd_kernel(ProjArgs a) {
    extern __shared__ __attribute__((aligned(16))) float sp[];  // [PR][K]
    const int b0 = blockIdx.x * PR, tid = threadIdx.x;
    const int nr = min(PR, a.B - b0);
    for (int e = tid; e < nr * a.K; e += blockDim.x) sp[e] = a.pooled[(int64_t)b0 * a.K + e];
    __syncthreads();
    for (int d = tid; d < a.D; d += blockDim.x) {
        float acc[PR];
        const float bi = a.bias[d];
#pragma unroll
        for (int r = 0; r < PR; ++r) acc[r] = bi;
        for (int k = 0; k < a.K; ++k) {
            const float w = a.wt[(int64_t)k * a.D + d];
#pragma unroll
            for (int r = 0; r < PR; ++r) acc[r] = fmaf(sp[r * a.K + k], w, acc[r]);
        }
        for (int r = 0; r < nr; ++r) a.h[(int64_t)(b0 + r) * a.D + d] = acc[r];
    }
}

__device__ __forceinline__ double bsum(double v, double* red) {
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

// BatchNorm1d statistics over the batch, one block per feature (exact two-pass, float64)
__global__ __launch_bounds__(256) void bn1d_fwd_kernel(ProjArgs a) {
    __shared__ double red[256];
    const int d = blockIdx.x;
    const float g = a.gamma[d], be = a.beta[d];
    if (!a.train) {
        if (threadIdx.x == 0) {
            float invstd = 1.f / sqrtf(a.rvar[d] + a.eps);
            a.cf[d] = make_float4(g * invstd, be - a.rmean[d] * g * invstd, a.rmean[d], invstd);
        }
        return;
    }
    double s = 0.0;
    for (int b = threadIdx.x; b < a.B; b += blockDim.x) s += (double)a.h[(int64_t)b * a.D + d];
    const double mean = bsum(s, red) / a.B;
    double q = 0.0;
    for (int b = threadIdx.x; b < a.B; b += blockDim.x) {
        double t = (double)a.h[(int64_t)b * a.D + d] - mean;
        q += t * t;
    }
    q = bsum(q, red);
    if (threadIdx.x == 0) {
        double var = q / a.B;
        double invstd = 1.0 / sqrt(var + (double)a.eps);
        a.cf[d] = make_float4((float)(g * invstd), (float)(be - mean * g * invstd), (float)mean, (float)invstd);
        double unb = a.B > 1 ? q / (a.B - 1) : q;
        a.rmean[d] = (float)((1.0 - a.momentum) * a.rmean[d] + a.momentum * mean);
        a.rvar[d] = (float)((1.0 - a.momentum) * a.rvar[d] + a.momentum * unb);
        if (d == 0 && a.nbt) a.nbt[0] += 1;
    }
}

// e = z / max(||z||, 1e-12), z = h*s + t ; one wave per row
__global__ __launch_bounds__(256) void normalize_fwd_kernel(ProjArgs a) {
    const int lane = threadIdx.x & 63;
    const int64_t b = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (b >= a.B) return;
    float z[4];
    float ss = 0.f;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        int d = lane + 64 * k;
        z[k] = 0.f;
        if (d < a.D) {
            float4 cf = a.cf[d];
            z[k] = fmaf(a.h[b * a.D + d], cf.x, cf.y);
            ss = fmaf(z[k], z[k], ss);
        }
    }
    const float n = sqrtf(wave_sum(ss));
    const float inv = 1.f / fmaxf(n, 1e-12f);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        int d = lane + 64 * k;
        if (d < a.D) a.emb[b * a.D + d] = z[k] * inv;
    }
    if (lane == 0) a.norm[b] = n;
}

__global__ __launch_bounds__(256) void normalize_bwd_kernel(ProjArgs a) {
    const int lane = threadIdx.x & 63;
    const int64_t b = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (b >= a.B) return;
    float e[4], g[4];
    float dot = 0.f;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        int d = lane + 64 * k;
        e[k] = g[k] = 0.f;
        if (d < a.D) {
            e[k] = a.emb[b * a.D + d];
            g[k] = a.demb[b * a.D + d];
            dot = fmaf(e[k], g[k], dot);
        }
    }
    dot = wave_sum(dot);
    const float n = a.norm[b];
    const bool live = n > 1e-12f;
    const float inv = 1.f / fmaxf(n, 1e-12f);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        int d = lane + 64 * k;
        if (d < a.D) a.dzp[b * a.D + d] = live ? (g[k] - e[k] * dot) * inv : g[k] * inv;
    }
}

__global__ __launch_bounds__(256) void bn1d_bwd_kernel(ProjArgs a) {
    __shared__ double red[256];
    const int d = blockIdx.x;
    const float4 cf = a.cf[d];
    double s0 = 0.0, s1 = 0.0;
    for (int b = threadIdx.x; b < a.B; b += blockDim.x) {
        double g = a.dzp[(int64_t)b * a.D + d];
        s0 += g;
        s1 += g * ((double)a.h[(int64_t)b * a.D + d] - cf.z) * cf.w;
    }
    s0 = bsum(s0, red);
    s1 = bsum(s1, red);
    if (threadIdx.x == 0) {
        a.dbeta[d] = (float)s0;
        a.dgamma[d] = (float)s1;
        a.cfb[d] = make_float4(a.gamma[d] * cf.w, (float)(s0 / a.B), (float)(s1 / a.B) * cf.w, cf.z);
    }
}

// dh = BN1d backward ; dpooled = dh @ W
__global__ __launch_bounds__(256) void proj_bwd_data_kernel(ProjArgs a) {
    extern __shared__ __attribute__((aligned(16))) float sd[];  // [PR][D]
    const int b0 = blockIdx.x * PR, tid = threadIdx.x;
    const int nr = min(PR, a.B - b0);
    for (int e = tid; e < PR * a.D; e += blockDim.x) {
        int r = e / a.D, d = e - r * a.D;
        float v = 0.f;
        if (r < nr) {
            int64_t o = (int64_t)(b0 + r) * a.D + d;
            float4 c = a.cfb[d];
            v = c.x * (a.dzp[o] - c.y - (a.h[o] - c.w) * c.z);
            a.dh[o] = v;
        }
        sd[e] = v;
    }
    __syncthreads();
    for (int k = tid; k < a.K; k += blockDim.x) {
        float acc[PR];
#pragma unroll
        for (int r = 0; r < PR; ++r) acc[r] = 0.f;
        int d = 0;
        if ((a.D & 3) == 0)  // (16-byte LDS reads of the rows' dh, as proj_fwd_kernel)
            for (; d < a.D; d += 4) {
                const float w0 = a.w[(int64_t)d * a.K + k], w1 = a.w[(int64_t)(d + 1) * a.K + k];
                const float w2 = a.w[(int64_t)(d + 2) * a.K + k], w3 = a.w[(int64_t)(d + 3) * a.K + k];
#pragma unroll
                for (int r = 0; r < PR; ++r) {
                    const float4 x = *reinterpret_cast<const float4*>(&sd[r * a.D + d]);
                    acc[r] = fmaf(x.w, w3, fmaf(x.z, w2, fmaf(x.y, w1, fmaf(x.x, w0, acc[r]))));
                }
            }
        for (; d < a.D; ++d) {
            const float w = a.w[(int64_t)d * a.K + k];
#pragma unroll
            for (int r = 0; r < PR; ++r) acc[r] = fmaf(sd[r * a.D + d], w, acc[r]);
        }
        for (int r = 0; r < nr; ++r) a.dpooled[(int64_t)(b0 + r) * a.K + k] = acc[r];
    }
}

// dW[d][k] = sum_b dh[b][d] pooled[b][k] ; db[d] = sum_b dh[b][d].  Block = (16 features,
// slice of rows); 64-row tiles of dh and pooled staged in LDS; thread (half, k) accumulates 8
// features for one k.  Per-slice partials, summed in fixed order by launch_sum_slices.
__global__ __launch_bounds__(256) void proj_bwd_weight_part_kernel(ProjArgs a, int bps) {
    __shared__ float sdh[64][17];
    __shared__ float spo[64][128];
    const int d0 = blockIdx.x * 16, slice = blockIdx.y, tid = threadIdx.x;
    const int half = tid >> 7, kl = tid & 127;
    const int b0 = slice * bps, b1 = min(a.B, b0 + bps);
    const int nd = min(16, a.D - d0);
    float* pw = a.part + (int64_t)slice * a.D * a.K;
    float* pb = a.part + (int64_t)gridDim.y * a.D * a.K + (int64_t)slice * a.D;
    for (int kb = 0; kb < a.K; kb += 128) {
        float acc[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] = 0.f;
        float sdb = 0.f;
        for (int bb = b0; bb < b1; bb += 64) {
            const int nb = min(64, b1 - bb);
            __syncthreads();
            for (int e = tid; e < 64 * 16; e += 256) {
                const int r = e >> 4, j = e & 15;
                sdh[r][j] = (r < nb && j < nd) ? a.dh[(int64_t)(bb + r) * a.D + d0 + j] : 0.f;
            }
            for (int e = tid; e < 64 * 128; e += 256) {
                const int r = e >> 7, k = e & 127;
                spo[r][k] = (r < nb && kb + k < a.K) ? a.pooled[(int64_t)(bb + r) * a.K + kb + k] : 0.f;
            }
            __syncthreads();
            for (int r = 0; r < nb; ++r) {
                const float pv = spo[r][kl];
#pragma unroll
                for (int j = 0; j < 8; ++j) acc[j] = fmaf(sdh[r][half * 8 + j], pv, acc[j]);
            }
            if (kb == 0 && tid < 16)
                for (int r = 0; r < nb; ++r) sdb += sdh[r][tid];
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int d = half * 8 + j;
            if (d < nd && kb + kl < a.K) pw[(int64_t)(d0 + d) * a.K + kb + kl] = acc[j];
        }
        if (kb == 0 && tid < nd) pb[d0 + tid] = sdb;
    }
}

__global__ void transpose_kernel(const float* __restrict__ in, float* __restrict__ out, int rows, int cols) {
    int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= rows * cols) return;
    int r = e / cols, c = e - r * cols;
    out[(int64_t)c * rows + r] = in[e];
}

__global__ __launch_bounds__(256) void row_sum_kernel(const float* __restrict__ part, int64_t cols,
                                                      float* __restrict__ out) {
    __shared__ double red[256];
    const float* p = part + (int64_t)blockIdx.x * cols;
    double s = 0.0;
    for (int64_t c = threadIdx.x; c < cols; c += blockDim.x) s += (double)p[c];
    s = bsum(s, red);
    if (threadIdx.x == 0) out[blockIdx.x] = (float)s;
}

size_t pool_smem(const HeadPoolArgs& a, bool bwd) {
    size_t f = bwd ? (2 * (size_t)a.P + 3 * a.C) : ((size_t)a.P + 2 * a.C);
    f = (f + 3) / 4 * 4;
    return (f + 4 * (size_t)a.C) * sizeof(float);
}

}  // namespace

int launch_head_pool_fwd(HeadPoolArgs a, hipStream_t s) {
    if (head_reg_fits(a)) {
        head_pool_fwd_reg_kernel<<<a.B, 512, 0, s>>>(a);
        PCX_LAUNCH_CHECK("head_pool_fwd_reg_kernel");
        return PCX_OK;
    }
    size_t sm = pool_smem(a, false);
    PCX_CHECK_ARG(sm <= 160 * 1024, "head: spatial size %d too large", a.P);
    (void)hipFuncSetAttribute((const void*)head_pool_fwd_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sm);
    head_pool_fwd_kernel<<<a.B, 256, sm, s>>>(a);
    PCX_LAUNCH_CHECK("head_pool_fwd_kernel");
    return PCX_OK;
}

int launch_head_pool_bwd(HeadPoolArgs a, hipStream_t s) {
    if (head_reg_fits(a)) {
        head_pool_bwd_reg_kernel<<<a.B, 512, 0, s>>>(a);
        PCX_LAUNCH_CHECK("head_pool_bwd_reg_kernel");
        return PCX_OK;
    }
    size_t sm = pool_smem(a, true);
    PCX_CHECK_ARG(sm <= 160 * 1024, "head: spatial size %d too large", a.P);
    (void)hipFuncSetAttribute((const void*)head_pool_bwd_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sm);
    head_pool_bwd_kernel<<<a.B, 256, sm, s>>>(a);
    PCX_LAUNCH_CHECK("head_pool_bwd_kernel");
    return PCX_OK;
}

int launch_proj_fwd(ProjArgs a, hipStream_t s) {
    PCX_CHECK_ARG(a.D <= 256, "projection: embedding_dim %d > 256 unsupported", a.D);
    size_t sm = (size_t)PR * a.K * sizeof(float);
    (void)hipFuncSetAttribute((const void*)proj_fwd_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sm);
    proj_fwd_kernel<<<ceil_div(a.B, PR), 256, sm, s>>>(a);
    PCX_LAUNCH_CHECK("proj_fwd_kernel");
    bn1d_fwd_kernel<<<a.D, 256, 0, s>>>(a);
    PCX_LAUNCH_CHECK("bn1d_fwd_kernel");
    normalize_fwd_kernel<<<ceil_div(a.B, 4), 256, 0, s>>>(a);
    PCX_LAUNCH_CHECK("normalize_fwd_kernel");
    return PCX_OK;
}

#define RC_(x)                  \
    do {                        \
        int _rc = (x);          \
        if (_rc) return _rc;    \
    } while (0)

int proj_wg_nslice(int B) { return std::max(1, std::min(64, B / 64)); }
size_t proj_part_floats(int B, int D, int K) { return (size_t)proj_wg_nslice(B) * D * (K + 1); }

int launch_proj_bwd(ProjArgs a, hipStream_t s) {
    normalize_bwd_kernel<<<ceil_div(a.B, 4), 256, 0, s>>>(a);
    PCX_LAUNCH_CHECK("normalize_bwd_kernel");
    bn1d_bwd_kernel<<<a.D, 256, 0, s>>>(a);
    PCX_LAUNCH_CHECK("bn1d_bwd_kernel");
    size_t sm = (size_t)PR * a.D * sizeof(float);
    (void)hipFuncSetAttribute((const void*)proj_bwd_data_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sm);
    proj_bwd_data_kernel<<<ceil_div(a.B, PR), 256, sm, s>>>(a);
    PCX_LAUNCH_CHECK("proj_bwd_data_kernel");
    PCX_CHECK_ARG(a.part, "proj_bwd: no partial buffer");
    const int ns = proj_wg_nslice(a.B), bps = ceil_div(a.B, ns);
    proj_bwd_weight_part_kernel<<<dim3((unsigned)ceil_div(a.D, 16), (unsigned)ns), 256, 0, s>>>(a, bps);
    PCX_LAUNCH_CHECK("proj_bwd_weight_part_kernel");
    RC_(launch_sum_slices(a.part, ns, (int64_t)a.D * a.K, a.dw, s));
    RC_(launch_sum_slices(a.part + (int64_t)ns * a.D * a.K, ns, a.D, a.db, s));
    return PCX_OK;
}

int launch_transpose(const float* in, float* out, int rows, int cols, hipStream_t s) {
    transpose_kernel<<<ceil_div((int64_t)rows * cols, 256), 256, 0, s>>>(in, out, rows, cols);
    PCX_LAUNCH_CHECK("transpose_kernel");
    return PCX_OK;
}

int launch_row_sum(const float* part, int rows, int64_t cols, float* out, hipStream_t s) {
    row_sum_kernel<<<rows, 256, 0, s>>>(part, cols, out);
    PCX_LAUNCH_CHECK("row_sum_kernel");
    return PCX_OK;
}

}  // namespace pcx
