// Weight gradient of the 3x3 convs, software-pipelined (the MI355X default).
//
//   dW[n][c][tap] = sum_{b,h,w} dy[b,n,h,w] * x[b,c,h+dh,w+dw]
//   dy = a*(dz - mb - (y - mean)*mgi)   (BN backward; reference autograd of phoneme_cnn.py:37-62)
//   x  = relu(y_prev*s + t) (PRO_BNRELU) or a materialised block input (PRO_RAW)
//
// Same GEMM decomposition as wgrad.hip (M = cout, N = cin, K = pixels; a block owns an NB x CB
// output block for all 9 taps and each wave owns PW MT x MT tiles over the full K of a chunk),
// but LDS is double-buffered and the staging of chunk k+1 is spread over the MFMA loop of chunk
// k: every few k-steps each thread issues the global loads of one staging unit (U elements) and,
// one spacing later, transforms and stores that unit into the other buffer.  Load latency hides
// behind the MFMAs instead of stalling the block between chunks.  The first cin group also writes
// dy to HBM (once per element) for the data-gradient conv that follows.  Per-slice partials are
// summed in a fixed order (deterministic).
#include "kernels.h"

namespace pcx {
namespace {

constexpr int U = 8;           // elements per thread per staging unit
constexpr int ZERO = -0x40000; // element outside the sample: stored as 0

__device__ __forceinline__ int fdiv(int n, int d, float inv) {  // n / d for 0 <= n < 2^22
    int q = (int)((float)n * inv);
    int r = n - q * d;
    if (r < 0) --q;
    else if (r >= d) ++q;
    return q;
}

template <int MT>
struct Mf;
template <>
struct Mf<32> {
    using Acc = f32x16;
    static constexpr int KS = 2, NREG = 16;
    static __device__ __forceinline__ Acc op(float a, float b, Acc c) {
        return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
    }
    static __device__ __forceinline__ int row(int r, int lane) { return acc_row(r, lane >> 5); }
    static __device__ __forceinline__ int col(int lane) { return lane & 31; }
};
template <>
struct Mf<16> {
    using Acc = f32x4;
    static constexpr int KS = 4, NREG = 4;
    static __device__ __forceinline__ Acc op(float a, float b, Acc c) {
        return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
    }
    static __device__ __forceinline__ int row(int r, int lane) { return (lane >> 4) * 4 + r; }
    static __device__ __forceinline__ int col(int lane) { return lane & 15; }
};

// LDS image of one chunk (one buffer): dy [NB][PS] | x [CB][XP], XP = (R+2)*(CW+2) + 1
struct Geo {
    int P, PS, XS, XR, XP, xoff, ndy, nx, NU, BUF;
    float invP, invCW, invXR, invXS;
};

struct Unit {
    float va[U], vb[U];
    int dst[U];   // LDS offset within the buffer, -1 = no element
    int code[U];  // >= 0: dy channel n; ZERO: store 0; otherwise x channel -(code+1)
    int o[U];     // dy: offset inside the sample's [cout][H][W] block (for dy_out)
};

__device__ __forceinline__ void load_unit(const WgradArgs& a, const Geo& g, Unit& un, int u, int b, int h0, int w0,
                                          int n0, int c0, int tid) {
    const int64_t HW = (int64_t)a.H * a.W;
#pragma unroll
    for (int i = 0; i < U; ++i) {
        const int e = tid + 256 * (u * U + i);
        un.dst[i] = -1;
        un.code[i] = ZERO;
        un.o[i] = 0;
        if (e < g.ndy) {
            const int n = fdiv(e, g.P, g.invP);
            const int pos = e - n * g.P;
            const int r = fdiv(pos, a.CW, g.invCW);
            const int hh = h0 + r, w = w0 + pos - r * a.CW;
            const bool ok = hh < a.H && w < a.W;
            const int o = (n0 + n) * (int)HW + min(hh, a.H - 1) * a.W + min(w, a.W - 1);
            const int64_t go = (int64_t)b * a.cout * HW + o;
            un.va[i] = a.dz[go];
            un.vb[i] = a.y[go];
            un.o[i] = o;
            un.dst[i] = n * g.PS + pos;
            un.code[i] = ok ? n : ZERO;
        } else if (e - g.ndy < g.nx) {
            const int ex = e - g.ndy;
            const int c = fdiv(ex, g.XR, g.invXR);
            const int rem = ex - c * g.XR;
            const int rr = fdiv(rem, g.XS, g.invXS);
            const int hh = h0 - 1 + rr, w = w0 - 1 + rem - rr * g.XS;
            const bool ok = hh >= 0 && hh < a.H && w >= 0 && w < a.W;
            un.va[i] = a.src[(((int64_t)b * a.cin + c0 + c) * a.H + min(max(hh, 0), a.H - 1)) * a.W +
                             min(max(w, 0), a.W - 1)];
            un.vb[i] = 0.f;
            un.dst[i] = g.xoff + c * g.XP + rem;
            un.code[i] = ok ? -(c + 1) : ZERO;
        } else {
            un.va[i] = 0.f;
            un.vb[i] = 0.f;
        }
    }
}

template <int PRO>
__device__ __forceinline__ void store_unit(const WgradArgs& a, const Unit& un, float* buf, const float4* cfd,
                                           const float4* cfx, float* dy_out) {
#pragma unroll
    for (int i = 0; i < U; ++i) {
        if (un.dst[i] < 0) continue;
        const int code = un.code[i];
        float v = 0.f;
        if (code >= 0) {
            const float4 k = cfd[code];
            v = k.x * (un.va[i] - k.y - (un.vb[i] - k.w) * k.z);
            if (dy_out) dy_out[un.o[i]] = v;
        } else if (code != ZERO) {
            v = un.va[i];
            if (PRO == PRO_BNRELU) {
                const float4 k = cfx[-code - 1];
                v = fmaxf(fmaf(v, k.x, k.y), 0.f);
            }
        }
        buf[un.dst[i]] = v;
    }
}

template <int MT, int PW, int PRO>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void wgrad_pipe_kernel(WgradArgs a) {
    using M = Mf<MT>;
    using Acc = typename M::Acc;
    constexpr int KS = M::KS;
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int NB = a.NPM * MT, CB = a.NPC * MT;
    Geo g;
    g.P = a.R * a.CW;
    g.PS = g.P + 1;
    g.XS = a.CW + 2;
    g.XR = (a.R + 2) * g.XS;
    g.XP = g.XR + 1;
    g.xoff = NB * g.PS;
    g.ndy = NB * g.P;
    g.nx = CB * g.XR;
    g.NU = (g.ndy + g.nx + 256 * U - 1) / (256 * U);
    g.BUF = NB * g.PS + CB * g.XP;
    g.invP = 1.f / g.P;
    g.invCW = 1.f / a.CW;
    g.invXR = 1.f / g.XR;
    g.invXS = 1.f / g.XS;
    float4* cfd = reinterpret_cast<float4*>(smem);  // [NB]
    float4* cfx = cfd + NB;                          // [CB]
    float* buf0 = smem + 4 * (NB + CB);

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int ncb = a.cin / CB;
    const int ngroups = (a.cout / NB) * ncb;
    const int f = blockIdx.x;
    const int kk = f >> 3;
    const int group = kk % ngroups;
    const int slice = (kk / ngroups) * 8 + (f & 7);
    if (slice >= a.nslice) return;
    const int n0 = (group / ncb) * NB, c0 = (group % ncb) * CB;
    const int li = (MT == 32) ? (lane & 31) : (lane & 15);
    const int kg = (MT == 32) ? (lane >> 5) : (lane >> 4);
    const int64_t HW = (int64_t)a.H * a.W;

    for (int i = tid; i < NB; i += 256) cfd[i] = a.cf_dy[n0 + i];
    if (PRO == PRO_BNRELU)
        for (int i = tid; i < CB; i += 256) cfx[i] = a.cf_x[c0 + i];
    __syncthreads();

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

    const int ch0 = slice * a.per_slice;
    const int ch1 = min(a.nchunks, ch0 + a.per_slice);
    auto geo = [&](int chunk, int& b, int& h0, int& w0) {
        const int seg = chunk % a.nseg;
        const int rb = (chunk / a.nseg) % a.nrb;
        b = chunk / (a.nseg * a.nrb);
        h0 = rb * a.R;
        w0 = seg * a.CW;
    };
    const bool write_dy = a.dy_out != nullptr && c0 == 0;
    Unit un;
    if (ch0 < ch1) {  // prologue: stage the first chunk synchronously
        int b, h0, w0;
        geo(ch0, b, h0, w0);
        float* dyo = write_dy ? a.dy_out + (int64_t)b * a.cout * HW : nullptr;
        for (int u = 0; u < g.NU; ++u) {
            load_unit(a, g, un, u, b, h0, w0, n0, c0, tid);
            store_unit<PRO>(a, un, buf0, cfd, cfx, dyo);
        }
    }
    __syncthreads();
    const int NK = g.P / KS;
    const int S = max(1, NK / (g.NU + 1));  // k-steps between staging actions
    for (int chunk = ch0; chunk < ch1; ++chunk) {
        const int cur = (chunk - ch0) & 1;
        const float* dyt = buf0 + cur * g.BUF;
        const float* xt = dyt + g.xoff;
        float* nxt = buf0 + (cur ^ 1) * g.BUF;
        const bool has_next = chunk + 1 < ch1;
        int nb = 0, nh0 = 0, nw0 = 0;
        if (has_next) geo(chunk + 1, nb, nh0, nw0);
        float* dyo = write_dy ? a.dy_out + (int64_t)nb * a.cout * HW : nullptr;
        int u_next = 0;
        bool pending = false;
        int r = 0, w = 0;
        for (int ks = 0; ks < NK; ++ks) {
            if (has_next && (ks % S) == 0) {
                if (pending) {
                    store_unit<PRO>(a, un, nxt, cfd, cfx, dyo);
                    pending = false;
                }
                if (u_next < g.NU) {
                    load_unit(a, g, un, u_next, nb, nh0, nw0, n0, c0, tid);
                    ++u_next;
                    pending = true;
                }
            }
            const int p0 = ks * KS;
#pragma unroll
            for (int k = 0; k < PW; ++k) {
                const float av = dyt[(mi[k] * MT + li) * g.PS + p0 + kg];
                const float* xb = xt + (ci[k] * MT + li) * g.XP + r * g.XS + w + kg;
#pragma unroll
                for (int t = 0; t < 9; ++t) acc[k][t] = M::op(av, xb[(t / 3) * g.XS + (t % 3)], acc[k][t]);
            }
            w += KS;
            if (w >= a.CW) { w = 0; ++r; }
        }
        if (has_next) {
            if (pending) store_unit<PRO>(a, un, nxt, cfd, cfx, dyo);
            for (; u_next < g.NU; ++u_next) {
                load_unit(a, g, un, u_next, nb, nh0, nw0, n0, c0, tid);
                store_unit<PRO>(a, un, nxt, cfd, cfx, dyo);
            }
        }
        __syncthreads();
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

size_t pipe_lds(int NB, int CB, int R, int CW) {
    const size_t buf = (size_t)NB * (R * CW + 1) + (size_t)CB * ((R + 2) * (CW + 2) + 1);
    return (2 * buf + 4 * (size_t)(NB + CB)) * 4;
}

}  // namespace

void wgrad_pipe_geometry(int B, int H, int W, int cin, int cout, WgradArgs* a) {
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
    // chunk shape: minimise staged elements (incl. halo) plus padded MFMA work; the double
    // buffer takes at most ~76 KB so two blocks share a CU (PCX_WG_LDS_KB overrides)
    size_t cap = 76 * 1024;
    if (const char* e = getenv("PCX_WG_LDS_KB")) cap = (size_t)atoi(e) * 1024;
    int bestR = 1, bestCW = 4;
    double best = 1e300;
    const int wmax = (W + 3) / 4 * 4;
    for (int cw = 4; cw <= std::max(4, std::min(wmax, 128)); cw += 4) {
        for (int R = 1; R <= std::min(H, 16); ++R) {
            const int P = R * cw;
            if (pipe_lds(NB, CB, R, cw) > cap || P > 512) continue;
            const double nch = (double)((W + cw - 1) / cw) * ((H + R - 1) / R);
            const double staged = nch * ((double)NB * P + (double)CB * (R + 2) * (cw + 2));
            const double compute = nch * P * 0.5 * NB * CB / 64.0;
            const double cost = staged * 4.0 + compute + nch * 2000.0;  // + per-chunk barrier
            if (cost < best) { best = cost; bestR = R; bestCW = cw; }
        }
    }
    a->R = bestR;
    a->CW = bestCW;
    a->nseg = ceil_div(W, a->CW);
    a->nrb = ceil_div(H, a->R);
    a->nchunks = B * a->nrb * a->nseg;
    const int ngroups = (cout / NB) * (cin / CB);
    int want = std::max(8, 1024 / ngroups);
    want = std::min(want, a->nchunks);
    a->per_slice = ceil_div(a->nchunks, want);
    a->nslice = ceil_div(a->nchunks, a->per_slice);
}

int launch_wgrad_pipe(int pro, WgradArgs a, hipStream_t s) {
    const int NB = a.NPM * a.MT, CB = a.NPC * a.MT;
    PCX_CHECK_ARG(a.cout % NB == 0 && a.cin % CB == 0, "wgrad_pipe: channels (%d,%d) vs block %dx%d", a.cout,
                  a.cin, NB, CB);
    PCX_CHECK_ARG(a.CW % 4 == 0, "wgrad_pipe: chunk width must be a multiple of 4");
    PCX_CHECK_ARG((int64_t)a.cout * a.H * a.W < ((int64_t)1 << 31), "wgrad_pipe: sample block too large");
    const int pw = a.NPM * a.NPC / 4;
    PCX_CHECK_ARG(pw * 4 == a.NPM * a.NPC && pw >= 1 && pw <= 2, "wgrad_pipe: bad tile split");
    const size_t smem = pipe_lds(NB, CB, a.R, a.CW);
    PCX_CHECK_ARG(smem <= 160 * 1024, "wgrad_pipe: LDS %zu too large", smem);
    dim3 grid((unsigned)(((a.nslice + 7) / 8) * 8 * ((a.cout / NB) * (a.cin / CB))));
#define PCX_WGP(MT_, PW_, P_)                                                                    \
    if (a.MT == MT_ && pw == PW_ && pro == P_) {                                                \
        (void)hipFuncSetAttribute((const void*)wgrad_pipe_kernel<MT_, PW_, P_>,                 \
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);       \
        wgrad_pipe_kernel<MT_, PW_, P_><<<grid, 256, smem, s>>>(a);                             \
        PCX_LAUNCH_CHECK("wgrad_pipe_kernel");                                                  \
        return PCX_OK;                                                                          \
    }
#define PCX_WGP_ALL(P_) PCX_WGP(32, 1, P_) PCX_WGP(16, 1, P_) PCX_WGP(16, 2, P_)
    PCX_WGP_ALL(PRO_RAW)
    PCX_WGP_ALL(PRO_BNRELU)
#undef PCX_WGP_ALL
#undef PCX_WGP
    set_error("wgrad_pipe: unsupported configuration (MT %d, PW %d, prologue %d)", a.MT, pw, pro);
    return PCX_EINVAL;
}

}  // namespace pcx
