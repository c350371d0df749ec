// Weight gradient of the 3x3 convs with a sliding row window (the MI355X default).
//
//   dW[n][c][tap] = sum_{b,h,w} dy[b,n,h,w] * x[b,c,h+dh,w+dw]
//   dy = a*(dz - mb - (y - mean)*mgi)   (BN backward; reference autograd of phoneme_cnn.py:37-62)
//   x  = relu(y_prev*s + t) (PRO_BNRELU) or a materialised block input (PRO_RAW)
//
// The weight gradient is HBM-bound when pixel chunks carry a halo: with R-row chunks every x row
// is fetched (R+2)/R times and narrow chunks waste most of each 128-B line (rocprofv3 FETCH_SIZE
// measured 5-15x the algorithmic bytes).  Here a block walks a column strip (CW columns) of one
// sample top to bottom, one image row per step: LDS keeps a ring of 4 x rows (rows r-1, r, r+1
// for the MFMAs and r+2 arriving) and 2 dy rows (r computing, r+1 arriving), so each x element
// is fetched once per strip (plus a 2-column halo) and dz/y exactly once.  The staging of step
// r+1 is interleaved with the MFMAs of step r (software pipeline, U elements per thread per
// unit), the BN backward / x prologue / zero padding are applied on the way into LDS, and the
// first cin group writes dy to HBM for the data-gradient conv that follows.
//
// GEMM view: M = cout (NB per block), N = cin (CB per block), K = pixels, 9 taps; each wave owns
// PW MT x MT tiles (MT = 32: v_mfma_f32_32x32x2_f32, MT = 16: v_mfma_f32_16x16x4_f32) for all 9
// taps.  Per-slice partials are summed in a fixed order by launch_sum_slices (deterministic).
#include "kernels.h"

namespace pcx {
namespace {

constexpr int U = 8;            // elements per thread per staging unit
constexpr int ZERO = -0x40000;  // element outside the sample: stored as 0

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

// LDS: dy rows [2][NB][DS] (DS = CW+1) | x rows [4][CB][XSP] (XSP = CW+3, image column jj holds
// sample column w0 - 1 + jj for jj < CW + 2)
struct Geo {
    int CW, DS, XS, XSP, ndy, nx, NU, dyslot, xslot, xbase;
    float invCW, invXS;
};

struct Unit {
    float va[U], vb[U];
    int dst[U];   // LDS offset, -1 = nothing to store
    int code[U];  // >= 0: dy channel; ZERO: store 0; otherwise x channel -(code+1)
    int o[U];     // dy: offset inside the sample's [cout][H][W] block (dy_out)
};

// one unit of the staging of (dy row rdy into dy slot ds) and (x row rx into x slot xs_);
// rdy < 0: no dy row; rx outside [0, H): the x row is written as zeros
__device__ __forceinline__ void load_unit(const WgradArgs& a, const Geo& g, Unit& un, int u, int b, int w0, int rdy,
                                          int ds, int rx, int xs_, int n0, int c0, int tid) {
    const int64_t HW = (int64_t)a.H * a.W;
#pragma unroll
    for (int i = 0; i < U; ++i) {
        const int e = tid + 256 * (u * U + i);
        un.dst[i] = -1;
        un.code[i] = ZERO;
        un.o[i] = 0;
        un.va[i] = 0.f;
        un.vb[i] = 0.f;
        if (e < g.ndy) {
            if (rdy >= 0) {
                const int n = fdiv(e, g.CW, g.invCW);
                const int j = e - n * g.CW;
                const int w = w0 + j;
                const int o = (n0 + n) * (int)HW + rdy * a.W + min(w, a.W - 1);
                const int64_t go = (int64_t)b * a.cout * HW + o;
                un.va[i] = a.dz[go];
                un.vb[i] = a.y[go];
                un.o[i] = o;
                un.dst[i] = ds * g.dyslot + n * g.DS + j;
                un.code[i] = w < a.W ? n : ZERO;
            }
        } else if (e - g.ndy < g.nx) {
            const int ex = e - g.ndy;
            const int c = fdiv(ex, g.XS, g.invXS);
            const int jj = ex - c * g.XS;
            const int w = w0 - 1 + jj;
            const bool ok = rx >= 0 && rx < a.H && w >= 0 && w < a.W;
            if (ok)
                un.va[i] = a.src[(((int64_t)b * a.cin + c0 + c) * a.H + rx) * a.W + w];
            un.dst[i] = g.xbase + xs_ * g.xslot + c * g.XSP + jj;
            un.code[i] = ok ? -(c + 1) : ZERO;
        }
    }
}

template <int PRO>
__device__ __forceinline__ void store_unit(const Unit& un, float* lds, const float4* cfd, const float4* cfx,
                                           float* dy_out) {
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
        lds[un.dst[i]] = v;
    }
}

template <int MT, int PW, int PRO>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void wgrad_win_kernel(WgradArgs a) {
    using M = Mf<MT>;
    using Acc = typename M::Acc;
    constexpr int KS = M::KS;
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int NB = a.NPM * MT, CB = a.NPC * MT;
    Geo g;
    g.CW = a.CW;
    g.DS = a.CW + 1;
    g.XS = a.CW + 2;
    g.XSP = a.CW + 3;
    g.ndy = NB * a.CW;
    g.nx = CB * g.XS;
    g.NU = (g.ndy + g.nx + 256 * U - 1) / (256 * U);
    g.dyslot = NB * g.DS;
    g.xslot = CB * g.XSP;
    g.xbase = 2 * g.dyslot;
    g.invCW = 1.f / a.CW;
    g.invXS = 1.f / g.XS;
    float4* cfd = reinterpret_cast<float4*>(smem);  // [NB]
    float4* cfx = cfd + NB;                          // [CB]
    float* lds = smem + 4 * (NB + CB);

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int ncb = a.cin / CB;
    const int ngroups = (a.cout / NB) * ncb;
    // XCD-aware (slice, group) mapping: the groups of one slice read the same rows, so they get
    // consecutive dispatch slots of one XCD (blocks f and f + 8 share an XCD)
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
        const int p = wave * PW + k;
        mi[k] = p / a.NPC;
        ci[k] = p - mi[k] * a.NPC;
    }
    Acc acc[PW][9];
#pragma unroll
    for (int k = 0; k < PW; ++k)
#pragma unroll
        for (int t = 0; t < 9; ++t) acc[k][t] = Acc{0.f};

    const bool write_dy = a.dy_out != nullptr && c0 == 0;
    const int NK = a.CW / KS;
    const int S = max(1, NK / (g.NU + 1));  // k-steps between staging actions
    const int t0 = slice * a.per_slice, t1 = min(a.nchunks, t0 + a.per_slice);
    Unit un;
    for (int task = t0; task < t1; ++task) {
        const int b = task / a.nseg;
        const int w0 = (task - b * a.nseg) * a.CW;
        float* dyo = write_dy ? a.dy_out + (int64_t)b * a.cout * HW : nullptr;
        // ---- prologue: x rows -1, 0, 1 -> slots 0, 1, 2 and dy row 0 -> dy slot 0
        for (int u = 0; u < g.NU; ++u) {
            load_unit(a, g, un, u, b, w0, 0, 0, -1, 0, n0, c0, tid);
            store_unit<PRO>(un, lds, cfd, cfx, dyo);
        }
        for (int q = 0; q <= 1; ++q)
            for (int u = 0; u < g.NU; ++u) {
                load_unit(a, g, un, u, b, w0, -1, 0, q, q + 1, n0, c0, tid);
                store_unit<PRO>(un, lds, cfd, cfx, dyo);
            }
        __syncthreads();
        for (int r = 0; r < a.H; ++r) {
            const bool pre = r + 1 < a.H;  // stage dy row r+1 and x row r+2 (zeros at r+2 == H)
            const float* dyt = lds + (r & 1) * g.dyslot;
            const float* xr0 = lds + g.xbase + (r & 3) * g.xslot;
            const float* xr1 = lds + g.xbase + ((r + 1) & 3) * g.xslot;
            const float* xr2 = lds + g.xbase + ((r + 2) & 3) * g.xslot;
            int u_next = 0;
            bool pending = false;
            for (int ks = 0; ks < NK; ++ks) {
                if (pre && (ks % S) == 0) {
                    if (pending) {
                        store_unit<PRO>(un, lds, cfd, cfx, dyo);
                        pending = false;
                    }
                    if (u_next < g.NU) {
                        load_unit(a, g, un, u_next, b, w0, r + 1, (r + 1) & 1, r + 2, (r + 3) & 3, n0, c0, tid);
                        ++u_next;
                        pending = true;
                    }
                }
                const int p0 = ks * KS;
#pragma unroll
                for (int k = 0; k < PW; ++k) {
                    const float av = dyt[(mi[k] * MT + li) * g.DS + p0 + kg];
                    const int xo = (ci[k] * MT + li) * g.XSP + p0 + kg;
#pragma unroll
                    for (int t = 0; t < 9; ++t) {
                        const float* xr = (t / 3 == 0) ? xr0 : (t / 3 == 1) ? xr1 : xr2;
                        acc[k][t] = M::op(av, xr[xo + (t % 3)], acc[k][t]);
                    }
                }
            }
            if (pre) {
                if (pending) store_unit<PRO>(un, lds, cfd, cfx, dyo);
                for (; u_next < g.NU; ++u_next) {
                    load_unit(a, g, un, u_next, b, w0, r + 1, (r + 1) & 1, r + 2, (r + 3) & 3, n0, c0, tid);
                    store_unit<PRO>(un, lds, cfd, cfx, dyo);
                }
            }
            __syncthreads();
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

size_t win_lds(int NB, int CB, int CW) {
    return ((size_t)2 * NB * (CW + 1) + (size_t)4 * CB * (CW + 3) + 4 * (size_t)(NB + CB)) * 4;
}

}  // namespace

void wgrad_win_geometry(int B, int H, int W, int cin, int cout, WgradArgs* a) {
    int MT, NPM, NPC;
    if (cout >= 64 && cin >= 64) {
        MT = 32; NPM = 2; NPC = 2;
    } else {
        MT = 16;
        NPM = std::min(cout, 64) / 16;
        NPC = std::min(cin, 32) / 16;
    }
    a->MT = MT; a->NPM = NPM; a->NPC = NPC;
    const int NB = NPM * MT, CB = NPC * MT, KS = MT == 32 ? 2 : 4;
    const int pw = NPM * NPC / 4;
    // strip width: per row step, MFMA cycles vs HBM line traffic (128-B lines, ~4.9 B/cycle per
    // block at 2 blocks/CU) + barrier; LDS <= 78 KB so two blocks share a CU
    const size_t cap = 78 * 1024;
    double best = 1e300;
    int bCW = KS;
    for (int cw = KS; cw <= std::max(KS, std::min(128, (W + KS - 1) / KS * KS)); cw += KS) {
        if (win_lds(NB, CB, cw) > cap) continue;
        const int nseg = (W + cw - 1) / cw;
        const double mfma = (double)pw * 9 * cw * (MT == 32 ? 32.0 : 8.0);
        const double lines_dy = cw * 4.0 / 128.0 + 1.0, lines_x = (cw + 2) * 4.0 / 128.0 + 1.0;
        const double mem = 128.0 * (2.0 * NB * lines_dy + CB * lines_x) / 4.9;
        const double step = std::max(mfma, mem) + 400.0;
        const double cost = nseg * (H * step + 3.0 * step);  // + prologue per strip
        if (cost < best) { best = cost; bCW = cw; }
    }
    a->CW = bCW;
    a->R = 1;
    a->nseg = ceil_div(W, bCW);
    a->nrb = 1;
    a->nchunks = B * a->nseg;  // tasks = (sample, strip)
    const int ngroups = (cout / NB) * (cin / CB);
    int want = std::max(8, 512 / ngroups);
    want = std::min(want, a->nchunks);
    a->per_slice = ceil_div(a->nchunks, want);
    a->nslice = ceil_div(a->nchunks, a->per_slice);
}

int launch_wgrad_win(int pro, WgradArgs a, hipStream_t s) {
    const int NB = a.NPM * a.MT, CB = a.NPC * a.MT;
    PCX_CHECK_ARG(a.cout % NB == 0 && a.cin % CB == 0, "wgrad_win: channels (%d,%d) vs block %dx%d", a.cout, a.cin,
                  NB, CB);
    PCX_CHECK_ARG(a.CW % (a.MT == 32 ? 2 : 4) == 0, "wgrad_win: strip width %d", a.CW);
    PCX_CHECK_ARG((int64_t)a.cout * a.H * a.W < ((int64_t)1 << 31), "wgrad_win: sample block too large");
    const int pw = a.NPM * a.NPC / 4;
    PCX_CHECK_ARG(pw * 4 == a.NPM * a.NPC && pw >= 1 && pw <= 2, "wgrad_win: bad tile split");
    const size_t smem = win_lds(NB, CB, a.CW);
    PCX_CHECK_ARG(smem <= 160 * 1024, "wgrad_win: LDS %zu too large", smem);
    dim3 grid((unsigned)(((a.nslice + 7) / 8) * 8 * ((a.cout / NB) * (a.cin / CB))));
#define PCX_WGW(MT_, PW_, P_)                                                                    \
    if (a.MT == MT_ && pw == PW_ && pro == P_) {                                                \
        (void)hipFuncSetAttribute((const void*)wgrad_win_kernel<MT_, PW_, P_>,                  \
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);       \
        wgrad_win_kernel<MT_, PW_, P_><<<grid, 256, smem, s>>>(a);                              \
        PCX_LAUNCH_CHECK("wgrad_win_kernel");                                                   \
        return PCX_OK;                                                                          \
    }
#define PCX_WGW_ALL(P_) PCX_WGW(32, 1, P_) PCX_WGW(16, 1, P_) PCX_WGW(16, 2, P_)
    PCX_WGW_ALL(PRO_RAW)
    PCX_WGW_ALL(PRO_BNRELU)
#undef PCX_WGW_ALL
#undef PCX_WGW
    set_error("wgrad_win: unsupported configuration (MT %d, PW %d, prologue %d)", a.MT, pw, pro);
    return PCX_EINVAL;
}

}  // namespace pcx
