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
};

struct Unit {
    float va[U], vb[U];
    int dst[U];   // LDS offset, -1 = nothing to store
    int code[U];  // >= 0: dy channel; ZERO: store 0; otherwise x channel -(code+1)
    int o[U];     // dy: offset inside the sample's [cout][H][W] block (dy_out)
};

// Staging cursor: element e = tid + 256*k of the flattened [dy row: NB x CW | x row: CB x XS]
// image, advanced incrementally (no divisions in the pipelined loop).
struct Cursor {
    int e, n, j, c, jj;
};

struct Steps {
    int e0, n0, j0, c0, jj0;  // this thread's first dy element and first x element
    int dn, dj, dc, djj;      // advance per 256 elements
};

__device__ __forceinline__ Steps make_steps(const Geo& g, int tid) {
    Steps st;
    st.e0 = tid;
    st.n0 = tid / g.CW;
    st.j0 = tid - st.n0 * g.CW;
    const int k = g.ndy > tid ? (g.ndy - tid + 255) / 256 : 0;  // first element index >= ndy
    const int ex = tid + 256 * k - g.ndy;
    st.c0 = ex / g.XS;
    st.jj0 = ex - st.c0 * g.XS;
    st.dn = 256 / g.CW;
    st.dj = 256 - st.dn * g.CW;
    st.dc = 256 / g.XS;
    st.djj = 256 - st.dc * g.XS;
    return st;
}

__device__ __forceinline__ void reset(Cursor& cu, const Steps& st) {
    cu.e = st.e0;
    cu.n = st.n0;
    cu.j = st.j0;
    cu.c = st.c0;
    cu.jj = st.jj0;
}

// one unit (U elements) of the staging of (dy row rdy into dy slot ds) and (x row rx into x slot
// xs_); rdy < 0: no dy row; rx outside [0, H): the x row is written as zeros
__device__ __forceinline__ void load_unit(const WgradArgs& a, const Geo& g, const Steps& st, Cursor& cu, Unit& un,
                                          const float* dzb, const float* yb, const float* xb, int w0, int rdy,
                                          int ds, int rx, int xs_, int n0) {
    const int HW = a.H * a.W;
    const int wlim = a.W - 1 - w0;  // last valid strip column
    const bool rxok = rx >= 0 && rx < a.H;
#pragma unroll
    for (int i = 0; i < U; ++i) {
        un.dst[i] = -1;
        un.code[i] = ZERO;
        un.o[i] = 0;
        un.va[i] = 0.f;
        un.vb[i] = 0.f;
        if (cu.e < g.ndy) {
            if (rdy >= 0) {
                const int o = (n0 + cu.n) * HW + rdy * a.W + w0 + min(cu.j, wlim);
                un.va[i] = dzb[o];
                un.vb[i] = yb[o];
                un.o[i] = o;
                un.dst[i] = ds * g.dyslot + cu.n * g.DS + cu.j;
                un.code[i] = cu.j <= wlim ? cu.n : ZERO;
            }
            cu.n += st.dn;
            cu.j += st.dj;
            if (cu.j >= g.CW) { cu.j -= g.CW; ++cu.n; }
        } else if (cu.e - g.ndy < g.nx) {
            const int w = w0 - 1 + cu.jj;
            const bool ok = rxok && w >= 0 && w < a.W;
            if (ok) un.va[i] = xb[(cu.c * a.H + rx) * a.W + w];
            un.dst[i] = g.xbase + xs_ * g.xslot + cu.c * g.XSP + cu.jj;
            un.code[i] = ok ? -(cu.c + 1) : ZERO;
            cu.c += st.dc;
            cu.jj += st.djj;
            if (cu.jj >= g.XS) { cu.jj -= g.XS; ++cu.c; }
        }
        cu.e += 256;
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
    // LDS row strides chosen bank-conflict free for the MFMA operand reads (ds_read_b32 serves
    // lanes 0-31 and 32-63 as groups of 32 banks): MT = 32 reads 32 channels (li) per group ->
    // odd stride; MT = 16 reads 16 channels x 2 pixels (kg) per group -> stride = 2 * odd
    g.CW = a.CW;
    g.DS = MT == 32 ? a.CW + 1 : a.CW + 2;
    g.XS = a.CW + 2;
    g.XSP = MT == 32 ? a.CW + 3 : a.CW + 2;
    g.ndy = NB * a.CW;
    g.nx = CB * g.XS;
    g.NU = (g.ndy + g.nx + 256 * U - 1) / (256 * U);
    g.dyslot = NB * g.DS;
    g.xslot = CB * g.XSP;
    g.xbase = 2 * g.dyslot;
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
    const Steps st = make_steps(g, tid);
    Cursor cu;
    const int NK = a.CW / KS;
    const int S = max(1, NK / (g.NU + 1));  // k-steps between staging actions
    const int t0 = slice * a.per_slice, t1 = min(a.nchunks, t0 + a.per_slice);
    Unit un;
    for (int task = t0; task < t1; ++task) {
        const int b = task / a.nseg;
        const int w0 = (task - b * a.nseg) * a.CW;
        float* dyo = write_dy ? a.dy_out + (int64_t)b * a.cout * HW : nullptr;
        const float* dzb = a.dz + (int64_t)b * a.cout * HW;
        const float* yb = a.y + (int64_t)b * a.cout * HW;
        const float* xb = a.src + ((int64_t)b * a.cin + c0) * HW;
        // ---- prologue: x rows -1, 0, 1 -> slots 0, 1, 2 and dy row 0 -> dy slot 0
        for (int q = -1; q <= 1; ++q) {
            reset(cu, st);
            for (int u = 0; u < g.NU; ++u) {
                load_unit(a, g, st, cu, un, dzb, yb, xb, w0, q == -1 ? 0 : -1, 0, q, q + 1, n0);
                store_unit<PRO>(un, lds, cfd, cfx, dyo);
            }
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
            reset(cu, st);
            for (int ks = 0; ks < NK; ++ks) {
                if (pre && (ks % S) == 0) {
                    if (pending) {
                        store_unit<PRO>(un, lds, cfd, cfx, dyo);
                        pending = false;
                    }
                    if (u_next < g.NU) {
                        load_unit(a, g, st, cu, un, dzb, yb, xb, w0, r + 1, (r + 1) & 1, r + 2, (r + 3) & 3, n0);
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
                    load_unit(a, g, st, cu, un, dzb, yb, xb, w0, r + 1, (r + 1) & 1, r + 2, (r + 3) & 3, n0);
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

size_t win_lds(int MT, int NB, int CB, int CW) {
    const int ds = MT == 32 ? CW + 1 : CW + 2, xsp = MT == 32 ? CW + 3 : CW + 2;
    return ((size_t)2 * NB * ds + (size_t)4 * CB * xsp + 4 * (size_t)(NB + CB)) * 4;
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
        if (win_lds(MT, NB, CB, cw) > cap) continue;
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
    const size_t smem = win_lds(a.MT, NB, CB, a.CW);
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
