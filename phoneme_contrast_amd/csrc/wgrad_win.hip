// Weight gradient of the 3x3 convs with a sliding row window (the MI355X default).
//
//   dW[n][c][tap] = sum_{b,h,w} dy[b,n,h,w] * x[b,c,h+dh,w+dw]
//   dy = a*(dz - mb - (y - mean)*mgi)   (BN backward; reference autograd of phoneme_cnn.py:37-62)
//   x  = relu(y_prev*s + t) (PRO_BNRELU) or a materialised block input (PRO_RAW)
//
// A block walks a column strip (CW columns) of one sample top to bottom, one image row per step.
// LDS keeps a ring of 4 x rows (rows r-1, r, r+1 for the MFMAs, r+2 arriving) and 2 dy rows, so
// each x element is fetched once per strip (plus a VEC-column halo each side) and dz / y exactly
// once.  Per row step:
//   1. the whole of dz / y row r+1 and x row r+2 is requested into registers (VEC-wide loads,
//      unconditional on clamped addresses: a predicated load becomes a divergent branch and the
//      waitcnt pass then drains vmcnt in front of every later load);
//   2. the MFMAs of row r run, LDS operands software-pipelined one k-step ahead;
//   3. the BN backward (dy), the x prologue and the zero padding are applied and the rows stored
//      to LDS (values first, then stores: global stores share vmcnt with the loads); the first
//      cin group also writes dy to HBM for the data-gradient conv that follows;  one barrier.
// Taps that read the zero rows above the first / below the last image row are skipped.
//
// GEMM view: M = cout (NB per block), N = cin (CB per block), K = pixels, 9 taps; each wave owns
// PW 16 x 16 tiles (v_mfma_f32_16x16x4_f32) for all 9 taps.  Per-slice partials are summed in a
// fixed order by launch_sum_slices (deterministic).
#include "wgrad_stage.h"

namespace pcx {
namespace {

constexpr int MT = 16, KS = 4;  // v_mfma_f32_16x16x4_f32: 16 x 16 tile, 4 pixels per k-step

__device__ __forceinline__ f32x4 mfma16(float a, float b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}


// MFMAs of one image row: tap rows dh with bit (dh+1) of ROWS set (rows -1 / H are zero: skipped).
// Software-pipelined by hand: the LDS operands of k-step k+1 are requested before the MFMAs of
// k-step k (sched_barrier keeps the scheduler from sinking them next to their use, which exposes
// the LDS latency in front of every MFMA).
template <int PW, int ROWS>
__device__ __forceinline__ void row_mfma(f32x4 (&acc)[PW][9], const float* dyt, const float* xr0, const float* xr1,
                                         const float* xr2, const int (&ao)[PW], const int (&xo)[PW], int kend) {
    if (kend <= 0) return;
    auto load = [&](int ks, float (&av)[PW], float (&bv)[PW][9]) {
        const int p0 = ks * KS;
#pragma unroll
        for (int k = 0; k < PW; ++k) {
            av[k] = dyt[ao[k] + p0];
#pragma unroll
            for (int t = 0; t < 9; ++t) {
                if (!((ROWS >> (t / 3)) & 1)) continue;
                const float* xr = (t / 3 == 0) ? xr0 : (t / 3 == 1) ? xr1 : xr2;
                bv[k][t] = xr[xo[k] + p0 + (t % 3)];
            }
        }
    };
    auto mma = [&](const float (&av)[PW], const float (&bv)[PW][9]) {
#pragma unroll
        for (int k = 0; k < PW; ++k)
#pragma unroll
            for (int t = 0; t < 9; ++t)
                if ((ROWS >> (t / 3)) & 1) acc[k][t] = mfma16(av[k], bv[k][t], acc[k][t]);
    };
    float a0[PW], b0[PW][9], a1[PW], b1[PW][9];
    load(0, a0, b0);
    int ks = 0;
    for (; ks + 2 <= kend; ks += 2) {
        load(min(ks + 1, kend - 1), a1, b1);
        __builtin_amdgcn_sched_barrier(0);
        mma(a0, b0);
        __builtin_amdgcn_sched_barrier(0);
        load(min(ks + 2, kend - 1), a0, b0);
        __builtin_amdgcn_sched_barrier(0);
        mma(a1, b1);
        __builtin_amdgcn_sched_barrier(0);
    }
    if (ks < kend) mma(a0, b0);
}

template <int PW, int PRO, int VEC, int VX, int NQDY, int NQX>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void wgrad_win_kernel(WgradArgs a) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int NB = a.NPM * MT, CB = a.NPC * MT;
    Geo g;
    g.CW = a.CW;
    g.QD = a.CW / VEC;
    g.QX = a.CW / VX + 2;
    g.DS = pad2odd(a.CW);
    g.XSP = pad2odd(a.CW + 2 * VX);
    g.nqd = NB * g.QD;
    g.nqx = CB * g.QX;
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
    const int li = lane & 15, kg = lane >> 4;
    const int64_t HW = (int64_t)a.H * a.W;

    for (int i = tid; i < NB; i += 256) cfd[i] = a.cf_dy[n0 + i];
    if (PRO == PRO_BNRELU)
        for (int i = tid; i < CB; i += 256) cfx[i] = a.cf_x[c0 + i];
    __syncthreads();

    int mi[PW], ci[PW], ao[PW], xo[PW];
#pragma unroll
    for (int k = 0; k < PW; ++k) {
        const int p = wave * PW + k;
        mi[k] = p / a.NPC;
        ci[k] = p - mi[k] * a.NPC;
        ao[k] = (mi[k] * MT + li) * g.DS + kg;
        xo[k] = (ci[k] * MT + li) * g.XSP + kg + (VX - 1);  // image column of sample column w0 - 1
    }
    f32x4 acc[PW][9];
#pragma unroll
    for (int k = 0; k < PW; ++k)
#pragma unroll
        for (int t = 0; t < 9; ++t) acc[k][t] = f32x4{0.f};

    Walk wk;
    wk.n0 = tid / g.QD;
    wk.q0 = tid - wk.n0 * g.QD;
    wk.dn = 256 / g.QD;
    wk.dq = 256 - wk.dn * g.QD;
    wk.c0 = tid / g.QX;
    wk.qx0 = tid - wk.c0 * g.QX;
    wk.dc = 256 / g.QX;
    wk.dqx = 256 - wk.dc * g.QX;

    const bool write_dy = a.dy_out != nullptr && c0 == 0;
    const int NK = a.CW / KS;
    const int t0 = slice * a.per_slice, t1 = min(a.nchunks, t0 + a.per_slice);
    RowStage<PRO, VEC, VX, NQDY, NQX> st;
    for (int task = t0; task < t1; ++task) {
        const int b = task / a.nseg;
        const int w0 = (task - b * a.nseg) * a.CW;
        // k-steps that touch valid columns (the strip tail past the sample edge is all zeros)
        const int kend = min(NK, (a.W - w0 + KS - 1) / KS);
        float* dyo = write_dy ? a.dy_out + ((int64_t)b * a.cout + n0) * HW : nullptr;
        const float* dzb = a.dz + ((int64_t)b * a.cout + n0) * HW;
        const float* yb = a.y + ((int64_t)b * a.cout + n0) * HW;
        const float* xb = a.src + ((int64_t)b * a.cin + c0) * HW;
        // ---- task prologue: x rows 0, 1 -> slots 1, 2 (row -1 is never read), dy row 0 -> slot 0
        st.load_dy(a, g, wk, dzb, yb, w0, 0, NB);
        st.load_x(a, g, wk, xb, w0, 0, CB);
        st.store_dy(a, g, wk, tid, lds, cfd, dyo, w0, 0, 0, NB);
        st.store_x(a, g, wk, tid, lds, cfx, w0, 1, CB);
        if (a.H > 1) {
            st.load_x(a, g, wk, xb, w0, 1, CB);
            st.store_x(a, g, wk, tid, lds, cfx, w0, 2, CB);
        }
        __syncthreads();
        for (int r = 0; r < a.H; ++r) {
            const bool pre = r + 1 < a.H;
            const bool prex = r + 2 < a.H;  // row H is never read (bottom-row taps are skipped)
            if (pre) st.load_dy(a, g, wk, dzb, yb, w0, r + 1, NB);
            if (prex) st.load_x(a, g, wk, xb, w0, r + 2, CB);
            const float* dyt = lds + (r & 1) * g.dyslot;
            const float* xr0 = lds + g.xbase + (r & 3) * g.xslot;
            const float* xr1 = lds + g.xbase + ((r + 1) & 3) * g.xslot;
            const float* xr2 = lds + g.xbase + ((r + 2) & 3) * g.xslot;
            const bool top = r == 0, bot = r + 1 == a.H;
            if (!top && !bot) row_mfma<PW, 7>(acc, dyt, xr0, xr1, xr2, ao, xo, kend);
            else if (top && !bot) row_mfma<PW, 6>(acc, dyt, xr0, xr1, xr2, ao, xo, kend);
            else if (!top && bot) row_mfma<PW, 3>(acc, dyt, xr0, xr1, xr2, ao, xo, kend);
            else row_mfma<PW, 2>(acc, dyt, xr0, xr1, xr2, ao, xo, kend);
            if (pre) st.store_dy(a, g, wk, tid, lds, cfd, dyo, w0, r + 1, (r + 1) & 1, NB);
            if (prex) st.store_x(a, g, wk, tid, lds, cfx, w0, (r + 3) & 3, CB);
            __syncthreads();
        }
    }
    float* out = a.part + (int64_t)slice * a.cout * a.cin * 9;
#pragma unroll
    for (int k = 0; k < PW; ++k)
#pragma unroll
        for (int t = 0; t < 9; ++t)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int n = n0 + mi[k] * MT + (lane >> 4) * 4 + q;
                const int c = c0 + ci[k] * MT + (lane & 15);
                out[((int64_t)n * a.cin + c) * 9 + t] = acc[k][t][q];
            }
}


// register prefetch capacity, in elements per thread per image, by PW (tiles per wave)
constexpr int NPRE[3] = {0, 16, 12};


}  // namespace

void wgrad_win_geometry(int B, int H, int W, int cin, int cout, WgradArgs* a) {
    // block = NB cout x CB cin of 16x16 tiles (4 or 8 tiles: 36 / 72 accumulator VGPRs per lane,
    // leaving room for the row prefetch)
    int NPM, NPC;
    if (cin >= 64 && cout >= 32) {
        NPM = 2; NPC = 4;
    } else {
        NPM = std::min(cout, 64) / 16;
        NPC = std::min(cin, 32) / 16;
    }
    a->MT = MT; a->NPM = NPM; a->NPC = NPC;
    const int NB = NPM * MT, CB = NPC * MT, vec = win_vec(W);
    const int pw = NPM * NPC / 4;
    const int npre = NPRE[pw];
    // strip width: the next row is prefetched into registers (<= npre elements per thread and
    // image), LDS <= 78 KB so two blocks share a CU.  Cost per row step = MFMA cycles of the
    // valid k-steps + a fixed barrier / staging overhead.
    const size_t cap = 80 * 1024;  // two blocks per CU
    double best = 1e300;
    int bCW = KS, bVX = vec;
    for (int vx = vec; vx >= std::max(1, vec / 2); vx >>= 1)
    for (int cw = KS; cw <= std::max(KS, (W + KS - 1) / KS * KS); cw += KS) {
        if (cw % vec) continue;
        if (win_lds(NB, CB, cw, vx) > cap) continue;
        if (NB * cw > 256 * npre || CB * (cw + 2 * vx) > 256 * npre) continue;
        const int nseg = (W + cw - 1) / cw;
        double mf = 0.0;
        for (int sgm = 0; sgm < nseg; ++sgm) {
            const int valid = std::min(cw, W - sgm * cw);
            mf += (double)pw * 9 * ((valid + KS - 1) / KS) * 32.0;
        }
        // narrower x loads cost more instructions per staged element
        const double cost = (H * (mf + nseg * 1200.0) + nseg * 2500.0) * (vx < vec ? 1.03 : 1.0);
        if (cost < best) { best = cost; bCW = cw; bVX = vx; }
    }
    a->CW = bCW;
    a->VX = bVX;
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
    const int NB = a.NPM * a.MT, CB = a.NPC * a.MT, vec = win_vec(a.W), vx = a.VX;
    PCX_CHECK_ARG(vx >= 1 && vx <= vec && vec % vx == 0, "wgrad_win: x vector width %d", vx);
    PCX_CHECK_ARG(a.cout % NB == 0 && a.cin % CB == 0, "wgrad_win: channels (%d,%d) vs block %dx%d", a.cout, a.cin,
                  NB, CB);
    PCX_CHECK_ARG(a.CW % KS == 0 && a.CW % vec == 0, "wgrad_win: strip width %d", a.CW);
    PCX_CHECK_ARG((int64_t)a.cout * a.H * a.W < ((int64_t)1 << 31), "wgrad_win: sample block too large");
    const int pw = a.NPM * a.NPC / 4;
    PCX_CHECK_ARG(a.MT == MT && pw * 4 == a.NPM * a.NPC && pw >= 1 && pw <= 2, "wgrad_win: bad tile split");
    PCX_CHECK_ARG(NB * a.CW <= 256 * NPRE[pw] && CB * (a.CW + 2 * vx) <= 256 * NPRE[pw],
                  "wgrad_win: strip %d exceeds the prefetch", a.CW);
    const size_t smem = win_lds(NB, CB, a.CW, vx);
    PCX_CHECK_ARG(smem <= 160 * 1024, "wgrad_win: LDS %zu too large", smem);
    dim3 grid((unsigned)(((a.nslice + 7) / 8) * 8 * ((a.cout / NB) * (a.cin / CB))));
#define PCX_WGW(PW_, P_, V_, VX_)                                                                      \
    if (pw == PW_ && pro == P_ && vec == V_ && vx == VX_) {                                            \
        constexpr int nq = NPRE[PW_] / V_, nqx = NPRE[PW_] / VX_;                                      \
        (void)hipFuncSetAttribute((const void*)wgrad_win_kernel<PW_, P_, V_, VX_, nq, nqx>,            \
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);              \
        wgrad_win_kernel<PW_, P_, V_, VX_, nq, nqx><<<grid, 256, smem, s>>>(a);                        \
        PCX_LAUNCH_CHECK("wgrad_win_kernel");                                                          \
        return PCX_OK;                                                                                 \
    }
#define PCX_WGW_V(PW_, P_) PCX_WGW(PW_, P_, 4, 4) PCX_WGW(PW_, P_, 4, 2) PCX_WGW(PW_, P_, 2, 2) PCX_WGW(PW_, P_, 2, 1) \
    PCX_WGW(PW_, P_, 1, 1)
#define PCX_WGW_ALL(P_) PCX_WGW_V(1, P_) PCX_WGW_V(2, P_)
    PCX_WGW_ALL(PRO_RAW)
    PCX_WGW_ALL(PRO_BNRELU)
#undef PCX_WGW_ALL
#undef PCX_WGW_V
#undef PCX_WGW
    set_error("wgrad_win: unsupported configuration (PW %d, prologue %d, vec %d)", pw, pro, vec);
    return PCX_EINVAL;
}

}  // namespace pcx
