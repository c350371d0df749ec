// Weight gradient of the 3x3 convs (reference autograd of nn.Conv2d at phoneme_cnn.py:39-61):
//   dW[n][c][tap] = sum_{b,h,w} dy[b,n,h,w] * x[b,c,h+dh,w+dw]
// with dy = BN-backward(dz, y) and x = the forward conv's input recomputed from the previous raw
// conv output by the same prologue (BN+ReLU[+MaxPool2+Dropout2d]).  Neither dy nor x is ever
// written to HBM.
//
// GEMM view: M = cout, N = cin, K = pixels (B*H*W, up to 33 M), 9 taps.  A block owns an
// NB x CB (cout x cin) output block for all 9 taps and walks a slice of pixel chunks (R rows x
// CW columns of one sample, staged once into LDS with zero halo).  Each of its 4 waves owns
// PW distinct MT x MT tiles x 9 taps in registers (MT = 32: v_mfma_f32_32x32x2_f32, 144 acc
// VGPRs; MT = 16: v_mfma_f32_16x16x4_f32 for the 32-channel layers) and runs the FULL K of
// every chunk, so the staging cost is shared by 4 x 9 x PW tiles.  Per-slice partials are summed
// by a second, deterministic pass.
#include "kernels.h"

namespace pcx {
namespace {

constexpr int U = 8;  // staging loads in flight per thread

__device__ __forceinline__ int fdiv(int n, int d, float inv) {
    int q = (int)((float)n * inv);
    int r = n - q * d;
    if (r < 0) --q;
    else if (r >= d) ++q;
    return q;
}

template <int PRO>
__device__ __forceinline__ float x_val(const WgradArgs& a, int c, int b, int hh, int w) {
    if (PRO == PRO_RAW) {
        return a.src[(((int64_t)b * a.cin + c) * a.H + hh) * a.W + w];
    } else if (PRO == PRO_BNRELU) {
        const float4 cf = a.cf_x[c];
        return fmaxf(fmaf(a.src[(((int64_t)b * a.cin + c) * a.H + hh) * a.W + w], cf.x, cf.y), 0.f);
    } else {  // PRO_BNRELU_POOL
        const float4 cf = a.cf_x[c];
        const float* p = a.src + (((int64_t)b * a.cin + c) * a.srcH + 2 * hh) * a.srcW + 2 * w;
        float m = fmaxf(fmaxf(fmaf(p[0], cf.x, cf.y), fmaf(p[1], cf.x, cf.y)),
                        fmaxf(fmaf(p[a.srcW], cf.x, cf.y), fmaf(p[a.srcW + 1], cf.x, cf.y)));
        m = fmaxf(m, 0.f);
        return a.drop ? m * a.drop[(int64_t)b * a.cin + c] : m;
    }
}

template <int MT>
struct Mfma;
template <>
struct Mfma<32> {
    using Acc = f32x16;
    static constexpr int KS = 2, NREG = 16;
    static __device__ __forceinline__ Acc op(float a, float b, Acc c) {
        return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
    }
    static __device__ __forceinline__ int row(int r, int lane) { return acc_row(r, lane >> 5); }
    static __device__ __forceinline__ int col(int lane) { return lane & 31; }
};
template <>
struct Mfma<16> {
    using Acc = f32x4;
    static constexpr int KS = 4, NREG = 4;
    static __device__ __forceinline__ Acc op(float a, float b, Acc c) {
        return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
    }
    static __device__ __forceinline__ int row(int r, int lane) { return (lane >> 4) * 4 + r; }
    static __device__ __forceinline__ int col(int lane) { return lane & 15; }
};

template <int MT, int PW, int PRO>
__global__ __launch_bounds__(256) void wgrad3x3_kernel(WgradArgs a) {
    using M = Mfma<MT>;
    using Acc = typename M::Acc;
    constexpr int KS = M::KS;
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int NB = a.NPM * MT, CB = a.NPC * MT;
    const int P = a.R * a.CW, PS = P + 1;
    const int XS = a.CW + 2, XR = (a.R + 2) * XS, XP = XR + 1;
    float* dyt = smem;
    float* xt = smem + NB * PS;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int ncb = a.cin / CB;
    const int ngroups = (a.cout / NB) * ncb;
    // XCD-aware (slice, group) mapping: the groups of one slice read the same dy / x rows, so
    // give them consecutive dispatch slots of the same XCD (blocks f and f+8 share an XCD).
    const int f = blockIdx.x;
    const int kk = f >> 3;
    const int group = kk % ngroups;
    const int slice = (kk / ngroups) * 8 + (f & 7);
    if (slice >= a.nslice) return;
    const int n0 = (group / ncb) * NB, c0 = (group % ncb) * CB;
    const int li = (MT == 32) ? (lane & 31) : (lane & 15);
    const int kg = (MT == 32) ? (lane >> 5) : (lane >> 4);

    int mi[PW], ci[PW];
#pragma unroll
    for (int k = 0; k < PW; ++k) {
        int p = wave * PW + k;
        mi[k] = p / a.NPC;
        ci[k] = p - mi[k] * a.NPC;
    }
    Acc acc[PW][9];
#pragma unroll
    for (int k = 0; k < PW; ++k)
#pragma unroll
        for (int t = 0; t < 9; ++t) acc[k][t] = Acc{0.f};

    const float invP = 1.f / P, invCW = 1.f / a.CW, invXR = 1.f / XR, invXS = 1.f / XS;
    const int ndy = NB * P, nx = CB * XR;
    const int ch0 = slice * a.per_slice;
    const int ch1 = min(a.nchunks, ch0 + a.per_slice);
    for (int chunk = ch0; chunk < ch1; ++chunk) {
        const int seg = chunk % a.nseg;
        const int rb = (chunk / a.nseg) % a.nrb;
        const int b = chunk / (a.nseg * a.nrb);
        const int h0 = rb * a.R, w0 = seg * a.CW;
        __syncthreads();
        // ---- dy tile [NB][P]: BN backward of (dz, y); loads issued U at a time, clamped
        for (int e0 = tid; e0 < ndy; e0 += 256 * U) {
            float v[U];
            int dst[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int e = e0 + u * 256;
                const bool in = e < ndy;
                const int ee = in ? e : 0;
                const int n = fdiv(ee, P, invP);
                const int pos = ee - n * P;
                const int r = fdiv(pos, a.CW, invCW);
                const int hh = h0 + r, w = w0 + pos - r * a.CW;
                const bool ok = in && hh < a.H && w < a.W;
                const int64_t o = (((int64_t)b * a.cout + n0 + n) * a.H + min(hh, a.H - 1)) * a.W + min(w, a.W - 1);
                const float dz = a.dz[o], y = a.y[o];
                const float4 cf = a.cf_dy[n0 + n];
                v[u] = ok ? cf.x * (dz - cf.y - (y - cf.w) * cf.z) : 0.f;
                dst[u] = in ? n * PS + pos : -1;
                // the first cin-group also materialises dy for the data-gradient conv (which then
                // reads one tensor instead of recomputing the BN backward from two)
                if (a.dy_out && c0 == 0 && ok) a.dy_out[o] = v[u];
            }
#pragma unroll
            for (int u = 0; u < U; ++u)
                if (dst[u] >= 0) dyt[dst[u]] = v[u];
        }
        // ---- x tile [CB][R+2][XS]: forward prologue, zero outside the sample
        for (int e0 = tid; e0 < nx; e0 += 256 * U) {
            float v[U];
            int dst[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int e = e0 + u * 256;
                const bool in = e < nx;
                const int ee = in ? e : 0;
                const int c = fdiv(ee, XR, invXR);
                const int rem = ee - c * XR;
                const int rr = fdiv(rem, XS, invXS);
                const int hh = h0 - 1 + rr, w = w0 - 1 + rem - rr * XS;
                const bool ok = in && hh >= 0 && hh < a.H && w >= 0 && w < a.W;
                const float xv = x_val<PRO>(a, c0 + c, b, min(max(hh, 0), a.H - 1), min(max(w, 0), a.W - 1));
                v[u] = ok ? xv : 0.f;
                dst[u] = in ? c * XP + rem : -1;
            }
#pragma unroll
            for (int u = 0; u < U; ++u)
                if (dst[u] >= 0) xt[dst[u]] = v[u];
        }
        __syncthreads();
        // ---- K loop over the chunk's positions: KS per MFMA, all 9 taps per A value
        int r = 0, w = 0;
        for (int p0 = 0; p0 < P; p0 += KS) {
#pragma unroll
            for (int k = 0; k < PW; ++k) {
                const float av = dyt[(mi[k] * MT + li) * PS + p0 + kg];
                const float* xb = xt + (ci[k] * MT + li) * XP + r * XS + w + kg;
#pragma unroll
                for (int t = 0; t < 9; ++t) acc[k][t] = M::op(av, xb[(t / 3) * XS + (t % 3)], acc[k][t]);
            }
            w += KS;
            if (w >= a.CW) { w = 0; ++r; }
        }
    }
    float* out = a.part + (int64_t)slice * a.cout * a.cin * 9;
#pragma unroll
    for (int k = 0; k < PW; ++k)
#pragma unroll
        for (int t = 0; t < 9; ++t)
#pragma unroll
            for (int q = 0; q < M::NREG; ++q) {
                const int n = n0 + mi[k] * MT + M::row(q, lane);
                const int c = c0 + ci[k] * MT + M::col(lane);
                out[((int64_t)n * a.cin + c) * 9 + t] = acc[k][t][q];
            }
}

}  // namespace

void wgrad3x3_geometry(int B, int H, int W, int cin, int cout, WgradArgs* a) {
    int MT, NPM, NPC;
    if (cout >= 64 && cin >= 64) {
        MT = 32; NPM = 2; NPC = 2;
    } else {
        MT = 16;
        NPM = std::min(cout, 64) / 16;
        NPC = std::min(cin, 32) / 16;
    }
    a->MT = MT; a->NPM = NPM; a->NPC = NPC;
    const int NB = NPM * MT, CB = NPC * MT;
    const int KS = MT == 32 ? 2 : 4;
    // chunk shape: minimise staged elements (incl. halo) plus padded MFMA work within ~76 KB of
    // LDS (measured: whole-row chunks with taller halos were slower — staging latency dominates)
    const size_t lds_cap = 76 * 1024;
    int bestR = 1, bestCW = KS;
    double best = 1e300;
    const int wmax = (W + 3) / 4 * 4;
    for (int cw = 4; cw <= std::max(4, std::min(wmax, 128)); cw += 4) {
        for (int R = 1; R <= std::min(H, 16); ++R) {
            int P = R * cw;
            size_t lds = ((size_t)NB * (P + 1) + (size_t)CB * ((R + 2) * (cw + 2) + 1)) * 4;
            if (lds > lds_cap || P > 512) continue;
            double nch = (double)((W + cw - 1) / cw) * ((H + R - 1) / R);
            double staged = nch * ((double)NB * P + (double)CB * (R + 2) * (cw + 2));
            double compute = nch * P * 0.5 * NB * CB / 64.0;  // position-MACs incl. padding waste
            double cost = staged * 4.0 + compute;
            if (cost < best) { best = cost; bestR = R; bestCW = cw; }
        }
    }
    a->R = bestR;
    a->CW = bestCW;
    (void)KS;
    a->nseg = ceil_div(W, a->CW);
    a->nrb = ceil_div(H, a->R);
    a->nchunks = B * a->nrb * a->nseg;
    const int ngroups = (cout / NB) * (cin / CB);
    int want = std::max(8, 1024 / ngroups);
    want = std::min(want, a->nchunks);
    a->per_slice = ceil_div(a->nchunks, want);
    a->nslice = ceil_div(a->nchunks, a->per_slice);
}

int launch_wgrad3x3(int pro, WgradArgs a, hipStream_t s) {
    const int NB = a.NPM * a.MT, CB = a.NPC * a.MT;
    PCX_CHECK_ARG(a.cout % NB == 0 && a.cin % CB == 0, "wgrad3x3: channels (%d,%d) vs block %dx%d",
                  a.cout, a.cin, NB, CB);
    PCX_CHECK_ARG(a.CW % 4 == 0, "wgrad3x3: chunk width must be a multiple of 4");
    const int pw = a.NPM * a.NPC / 4;
    PCX_CHECK_ARG(pw * 4 == a.NPM * a.NPC && pw >= 1 && pw <= 2, "wgrad3x3: bad tile split");
    const int P = a.R * a.CW;
    size_t smem = ((size_t)NB * (P + 1) + (size_t)CB * ((a.R + 2) * (a.CW + 2) + 1)) * sizeof(float);
    PCX_CHECK_ARG(smem <= 160 * 1024, "wgrad3x3: LDS %zu too large", smem);
    dim3 grid((unsigned)(((a.nslice + 7) / 8) * 8 * ((a.cout / NB) * (a.cin / CB))));
#define PCX_WG(MT_, PW_, P_)                                                                     \
    if (a.MT == MT_ && pw == PW_ && pro == P_) {                                                \
        (void)hipFuncSetAttribute((const void*)wgrad3x3_kernel<MT_, PW_, P_>,                   \
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);       \
        wgrad3x3_kernel<MT_, PW_, P_><<<grid, 256, smem, s>>>(a);                               \
        PCX_LAUNCH_CHECK("wgrad3x3_kernel");                                                    \
        return PCX_OK;                                                                          \
    }
#define PCX_WG_ALL(P_) PCX_WG(32, 1, P_) PCX_WG(16, 1, P_) PCX_WG(16, 2, P_)
    PCX_WG_ALL(PRO_RAW)
    PCX_WG_ALL(PRO_BNRELU)
    PCX_WG_ALL(PRO_BNRELU_POOL)
#undef PCX_WG_ALL
#undef PCX_WG
    set_error("wgrad3x3: unsupported configuration (MT %d, PW %d, prologue %d)", a.MT, pw, pro);
    return PCX_EINVAL;
}

}  // namespace pcx
