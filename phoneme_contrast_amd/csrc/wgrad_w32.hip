// Weight gradient of the 3x3 convs on 32 x 32 tiles (v_mfma_f32_32x32x2_f32), sliding row window.
//
//   dW[n][c][tap] = sum_{b,h,w} dy[b,n,h,w] * x[b,c,h+dh,w+dw]      (reference: autograd of the
//   conv layers of PhonemeNet, phoneme_cnn.py:35-65; dy = BN backward of (dz, y), x = the block
//   input after BN + ReLU, or the materialised pooled input)
//
// Used for the narrow rows (W < 50) of the residual network's stride-1 convs, where the 8-column
// stream granule of wgrad_s.hip wastes more than it saves.  Row staging of wgrad_stage.h (a block
// walks a column strip of one sample top to bottom, x rows in a 4-slot LDS ring, dy rows in 2
// slots, the next rows prefetched into registers while the MFMAs of the current row run, one
// barrier per row).  Each wave owns a 32 (cout) x 32 (cin) tile for all 9 taps (144 accumulator
// VGPRs): one k-step (2 pixels) costs 1 A + 9 B LDS reads for 9 MFMAs of 64 cycles.  A block
// holds TM x TN tiles; when that is fewer than 4,
// KW = 4 / (TM TN) waves share a tile and split its k-steps (their partials are separate slices,
// summed with the task slices by launch_sum_slices in a fixed order: deterministic).
#include "wgrad_stage.h"

namespace pcx {
namespace {

// register prefetch per thread and image (dz, y, x) beside 144 accumulators (scalar loads at odd
// widths need more address registers)
constexpr int npre32(int vec) { return vec == 1 ? 8 : 12; }

// MFMAs of one image row for k-steps kb, kb + KW, ... < kend.  Taps that read the zero rows above
// the first / below the last image row are skipped under uniform branches (one inlined body: four
// specialised copies made the allocator keep four sets of 144 accumulators and spill).
template <int KW>
__device__ __forceinline__ void row_mfma32(f32x16 (&acc)[9], const float* dyt, const float* xr0, const float* xr1,
                                           const float* xr2, int ao, int xo, int kb, int kend, bool up, bool dn) {
    if (kb >= kend) return;
    auto load = [&](int ks, float& av, float (&bv)[9]) {
        const int p0 = 2 * ks;
        av = dyt[ao + p0];
#pragma unroll
        for (int t = 0; t < 9; ++t) {
            const float* xr = (t / 3 == 0) ? xr0 : (t / 3 == 1) ? xr1 : xr2;
            bv[t] = xr[xo + p0 + (t % 3)];  // rows -1 / H: stale ring data, never multiplied
        }
    };
    auto mma = [&](float av, const float (&bv)[9]) {
        if (up) {
#pragma unroll
            for (int t = 0; t < 3; ++t) acc[t] = mfma32(av, bv[t], acc[t]);
        }
#pragma unroll
        for (int t = 3; t < 6; ++t) acc[t] = mfma32(av, bv[t], acc[t]);
        if (dn) {
#pragma unroll
            for (int t = 6; t < 9; ++t) acc[t] = mfma32(av, bv[t], acc[t]);
        }
    };
    float a0, b0[9], a1, b1[9];
    load(kb, a0, b0);
    int ks = kb;
    for (; ks + KW < kend; ks += 2 * KW) {
        load(ks + KW, a1, b1);
        __builtin_amdgcn_sched_barrier(0);
        mma(a0, b0);
        __builtin_amdgcn_sched_barrier(0);
        load(min(ks + 2 * KW, kend - 1), a0, b0);
        __builtin_amdgcn_sched_barrier(0);
        mma(a1, b1);
        __builtin_amdgcn_sched_barrier(0);
    }
    if (ks < kend) mma(a0, b0);
}

template <int PRO, int VEC, int VX, int NQDY, int NQX, int TM, int TN>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void wgrad_w32_kernel(WgradArgs a) {
    constexpr int KW = 4 / (TM * TN);
    constexpr int NB = 32 * TM, CB = 32 * TN;
    extern __shared__ __attribute__((aligned(16))) float smem[];
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

    const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, l32 = lane & 31;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int ncb = a.cin / CB;
    const int ngroups = (a.cout / NB) * ncb;
    // XCD-aware (slice, group) mapping: the groups of one slice read the same rows
    const int f = blockIdx.x;
    const int kk = f >> 3;
    const int group = kk % ngroups;
    const int slice = (kk / ngroups) * 8 + (f & 7);
    if (slice >= a.ntslice) return;
    const int n0 = (group / ncb) * NB, c0 = (group % ncb) * CB;
    const int tw = wave / KW, kw = wave - tw * KW;  // tile of this wave, its k-step phase
    const int mi = tw / TN, ci = tw - mi * TN;
    const int64_t HW = (int64_t)a.H * a.W;

    for (int i = tid; i < NB; i += 256) cfd[i] = a.cf_dy[n0 + i];
    if (PRO == PRO_BNRELU)
        for (int i = tid; i < CB; i += 256) cfx[i] = a.cf_x[c0 + i];
    __syncthreads();

    // A: dy[n = mi*32 + l32][pixel 2 ks + h]; B: x[c = ci*32 + l32][pixel 2 ks + h + dw]
    const int ao = (mi * 32 + l32) * g.DS + h;
    const int xo = (ci * 32 + l32) * g.XSP + h + (VX - 1);  // image column of sample column w0 - 1
    f32x16 acc[9];
#pragma unroll
    for (int t = 0; t < 9; ++t) acc[t] = f32x16{0.f};

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
    const int t0 = slice * a.per_slice, t1 = min(a.nchunks, t0 + a.per_slice);
    RowStage<PRO, VEC, VX, NQDY, NQX> st;
    for (int task = t0; task < t1; ++task) {
        const int b = task / a.nseg;
        const int w0 = (task - b * a.nseg) * a.CW;
        // k-steps touching valid columns (an odd tail pixel pairs with a zero column)
        const int kend = min(a.CW / 2, (a.W - w0 + 1) / 2);
        float* dyo = write_dy ? a.dy_out + ((int64_t)b * a.cout + n0) * HW : nullptr;
        const float* dzb = a.dz + ((int64_t)b * a.cout + n0) * HW;
        const float* yb = a.y + ((int64_t)b * a.cout + n0) * HW;
        const float* xb = a.src + ((int64_t)b * a.cin + c0) * HW;
        // task prologue: x rows 0, 1 -> slots 1, 2 (row -1 is never read), dy row 0 -> slot 0
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
            row_mfma32<KW>(acc, dyt, xr0, xr1, xr2, ao, xo, kw, kend, r > 0, r + 1 < a.H);
            if (pre) st.store_dy(a, g, wk, tid, lds, cfd, dyo, w0, r + 1, (r + 1) & 1, NB);
            if (prex) st.store_x(a, g, wk, tid, lds, cfx, w0, (r + 3) & 3, CB);
            __syncthreads();
        }
    }
    float* out = a.part + ((int64_t)slice * KW + kw) * a.cout * a.cin * 9;
    const int c = c0 + ci * 32 + l32;
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
        for (int rr = 0; rr < 16; ++rr) {
            const int n = n0 + mi * 32 + acc_row(rr, h);
            out[((int64_t)n * a.cin + c) * 9 + t] = acc[t][rr];
        }
}

struct W32Cfg {
    int TM, TN, CW, VX;
};

bool w32_fits(int TM, int TN, int CW, int VX, int W) {
    const int NB = 32 * TM, CB = 32 * TN, vec = win_vec(W);
    return CW % vec == 0 && CW % 2 == 0 && VX <= vec && vec % VX == 0 &&
           win_lds(NB, CB, CW, VX) <= 80 * 1024 && NB * CW <= 256 * npre32(vec) && CB * (CW + 2 * VX) <= 256 * npre32(vec);
}

}  // namespace

bool wgrad_w32_geometry(int B, int H, int W, int cin, int cout, WgradArgs* a) {
    // 32-channel inputs stay on the 16x16 kernel: with one 32x32 tile per block the K split over
    // waves and its extra partial slices cost more than the LDS reads saved (measured on MI355X,
    // cnn_small L2: 7.13 + 0.64 ms reduce vs 6.79 + 0.16; L3 even)
    if (cin % 64 || cout % 32) return false;
    const int vec = win_vec(W);
    W32Cfg best{0, 0, 0, 0};
    double bcost = 1e300;
    // modelled cycles per sample: MFMAs (64 cycles each, per wave) + per row step a barrier /
    // staging cost that grows with the staged elements per thread
    const int tiles[4][2] = {{2, 2}, {2, 1}, {1, 2}, {1, 1}};
    for (auto& tt : tiles) {
        const int TM = tt[0], TN = tt[1], KW = 4 / (TM * TN);
        if (cout % (32 * TM) || cin % (32 * TN)) continue;
        const int ngroups = (cout / (32 * TM)) * (cin / (32 * TN));
        for (int vx = vec; vx >= std::max(1, vec / 2); vx >>= 1)
            for (int cw = 4; cw <= (W + 3) / 4 * 4; cw += 2) {
                if (!w32_fits(TM, TN, cw, vx, W)) continue;
                const int nseg = (W + cw - 1) / cw;
                double mf = 0.0;
                for (int sg = 0; sg < nseg; ++sg) {
                    const int valid = std::min(cw, W - sg * cw);
                    mf += (double)((valid + 1) / 2 + KW - 1) / KW * 9 * 64;
                }
                const double staged = (2.0 * 32 * TM * cw + 32.0 * TN * (cw + 2 * vx)) / 256.0;
                const double row = mf + nseg * (1500.0 + 12.0 * staged * (vx < vec ? 1.1 : 1.0));
                const double cost = ngroups * (H * row + nseg * 2500.0);
                if (cost < bcost) { bcost = cost; best = {TM, TN, cw, vx}; }
            }
    }
    if (!best.TM) return false;
    a->MT = 32;
    a->NPM = best.TM;
    a->NPC = best.TN;
    a->KW = 4 / (best.TM * best.TN);
    a->CW = best.CW;
    a->VX = best.VX;
    a->R = 1;
    a->nrb = 1;
    a->nseg = ceil_div(W, best.CW);
    a->nchunks = B * a->nseg;
    const int ngroups = (cout / (32 * best.TM)) * (cin / (32 * best.TN));
    int want = std::max(8, 512 / ngroups);
    want = std::min(want, a->nchunks);
    a->per_slice = ceil_div(a->nchunks, want);
    a->ntslice = ceil_div(a->nchunks, a->per_slice);
    a->nslice = a->ntslice * a->KW;
    return true;
}

int launch_wgrad_w32(int pro, WgradArgs a, hipStream_t s) {
    const int TM = a.NPM, TN = a.NPC, NB = 32 * TM, CB = 32 * TN, vec = win_vec(a.W), vx = a.VX;
    PCX_CHECK_ARG(a.MT == 32 && TM * TN >= 1 && 4 % (TM * TN) == 0 && a.KW == 4 / (TM * TN),
                  "wgrad_w32: bad tile split %dx%d", TM, TN);
    PCX_CHECK_ARG(a.cout % NB == 0 && a.cin % CB == 0, "wgrad_w32: channels (%d,%d) vs block %dx%d", a.cout, a.cin,
                  NB, CB);
    PCX_CHECK_ARG(w32_fits(TM, TN, a.CW, vx, a.W), "wgrad_w32: strip %d / vx %d does not fit", a.CW, vx);
    PCX_CHECK_ARG((int64_t)a.cout * a.H * a.W < ((int64_t)1 << 31), "wgrad_w32: sample block too large");
    PCX_CHECK_ARG(a.nslice == a.ntslice * a.KW, "wgrad_w32: slice count");
    const size_t smem = win_lds(NB, CB, a.CW, vx);
    dim3 grid((unsigned)(((a.ntslice + 7) / 8) * 8 * ((a.cout / NB) * (a.cin / CB))));
#define PCX_W32(P_, V_, VX_, TM_, TN_)                                                                     \
    if (pro == P_ && vec == V_ && vx == VX_ && TM == TM_ && TN == TN_) {                                   \
        constexpr int nq = npre32(V_) / V_, nqx = npre32(V_) / VX_;                                       \
        (void)hipFuncSetAttribute((const void*)wgrad_w32_kernel<P_, V_, VX_, nq, nqx, TM_, TN_>,          \
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);                  \
        wgrad_w32_kernel<P_, V_, VX_, nq, nqx, TM_, TN_><<<grid, 256, smem, s>>>(a);                       \
        PCX_LAUNCH_CHECK("wgrad_w32_kernel");                                                              \
        return PCX_OK;                                                                                     \
    }
#define PCX_W32_T(P_, V_, VX_) PCX_W32(P_, V_, VX_, 2, 2) PCX_W32(P_, V_, VX_, 2, 1) PCX_W32(P_, V_, VX_, 1, 2) \
    PCX_W32(P_, V_, VX_, 1, 1)
#define PCX_W32_V(P_) PCX_W32_T(P_, 4, 4) PCX_W32_T(P_, 4, 2) PCX_W32_T(P_, 2, 2) PCX_W32_T(P_, 2, 1) \
    PCX_W32_T(P_, 1, 1)
    PCX_W32_V(PRO_RAW)
    PCX_W32_V(PRO_BNRELU)
#undef PCX_W32_V
#undef PCX_W32_T
#undef PCX_W32
    set_error("wgrad_w32: unsupported combination (pro %d vec %d vx %d tiles %dx%d)", pro, vec, vx, TM, TN);
    return PCX_EINVAL;
}

}  // namespace pcx
