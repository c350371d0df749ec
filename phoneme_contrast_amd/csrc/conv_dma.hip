// 3x3 / stride 1 / pad 1 conv (forward and data gradient) with asynchronous LDS-DMA staging.
//
// Same implicit GEMM and epilogues as conv.hip, different operand path (MI355X-first):
//  * the raw input rows of a K-chunk (CK channels x NR staged rows, dense [c][row][W] image) and
//    the weight chunk are copied HBM/L2 -> LDS by global_load_lds (dwordx4 when rows are 16-byte
//    aligned, dword otherwise) into one of two buffers; chunk k+1 is in flight while the MFMAs of
//    chunk k run, so staging latency is hidden and costs no VGPRs;
//  * the prologue (BN+ReLU of the producer; the data gradient reads the dy its weight gradient
//    materialised, raw) is applied when a B operand is read from LDS;
//  * zero padding / sample boundaries without data masks: a tap whose neighbour pixel is outside
//    the sample reads a reserved 16-byte group at the end of the channel plane instead (0 for raw
//    operands, NaN for BN+ReLU ones: relu(NaN * s + t) = fmaxf(NaN, 0) = 0).  The choice is one
//    address select per (tap, pixel group), shared by all k-steps of the tap, in place of a
//    v_cndmask on every operand (which also cost VALU->MFMA hazard nops);
//  * one barrier per chunk; all per-chunk tables live in the single dynamic LDS array (no second
//    __shared__ object, so hipcc does not drain the DMA queue before LDS reads).
#include "conv_epilogue.h"

namespace pcx {
namespace {

typedef __attribute__((address_space(3))) void lds_void;

__device__ __forceinline__ int fdiv(int n, int d, float inv) {  // n / d, 0 <= n < 2^22
    int q = (int)((float)n * inv);
    int r = n - q * d;
    if (r < 0) --q;
    else if (r >= d) ++q;
    return q;
}

__device__ __forceinline__ int xcd_remap(int orig, int nb) {
    int q = nb >> 3, r = nb & 7, x = orig & 7;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (orig >> 3);
}

// global -> LDS DMA of VEC floats per lane; LDS destination = wave-uniform base + lane * VEC.
// Issued through inline asm: the builtin makes the waitcnt pass put a vmcnt(0) in front of every
// later ds_read (it cannot tell the DMA target from the buffer being read), which serialises the
// double buffer.  Completion is ordered explicitly by the vmcnt(0) + barrier at each chunk start.
template <int VEC>
__device__ __forceinline__ void dma(const float* g, unsigned lds_byte_addr) {
    const unsigned m0 = __builtin_amdgcn_readfirstlane(lds_byte_addr);
    if constexpr (VEC == 4)
        asm volatile("s_nop 0\n\tglobal_load_lds_dwordx4 %0, off" :: "v"(g), "{m0}"(m0) : "memory");
    else
        asm volatile("s_nop 0\n\tglobal_load_lds_dword %0, off" :: "v"(g), "{m0}"(m0) : "memory");
}

// Same copy in the saddr form: global address = uniform 64-bit base (SGPRs) + per-lane 32-bit
// byte offset.  The offsets of every copy a lane issues are fixed for a tile (only the channel
// base moves from chunk to chunk), so they are computed once and a copy costs no VALU at all.
template <int VEC>
__device__ __forceinline__ void dma_s(const float* sbase, unsigned voff, unsigned lds_byte_addr) {
    const unsigned m0 = __builtin_amdgcn_readfirstlane(lds_byte_addr);
    if constexpr (VEC == 4)
        asm volatile("s_nop 0\n\tglobal_load_lds_dwordx4 %0, %1" :: "v"(voff), "s"(sbase), "{m0}"(m0) : "memory");
    else
        asm volatile("s_nop 0\n\tglobal_load_lds_dword %0, %1" :: "v"(voff), "s"(sbase), "{m0}"(m0) : "memory");
}

__device__ __forceinline__ const float* uniform_ptr(const float* p) {
    const uint64_t v = (uint64_t)(uintptr_t)p;
    const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)v);
    const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(v >> 32));
    return (const float*)(uintptr_t)(((uint64_t)hi << 32) | lo);
}

// copies per wave and K-chunk with precomputed offsets (more fall back to per-copy addressing)
constexpr int DMA_MAXR = 5, DMA_MAXW = 3;

// floats of the per-block tables in front of the staged image: cf [cin] float4, rinfo [NR] int2,
// rowpos [NR] int, segments [NR] int4
__host__ __device__ constexpr int dma_table_floats(int cin, int NR) {
    return 4 * cin + ((2 * NR + 3) & ~3) + ((NR + 3) & ~3) + 4 * NR;
}

// raw image of one K-chunk: CK channels x NR staged rows x W columns (dense)
// (channel planes of PL floats: NR * W image floats, padding to 16 bytes, the reserved group)
template <int VEC>
__device__ __forceinline__ void issue_raw(const ConvArgs& a, const int2* rinfo, unsigned raw, int c0,
                                          int wave, int lane, int total, int PL, float invPL,
                                          float invW) {
    const int PLD = a.NR * a.W;  // image floats per channel plane
    for (int base = wave * 64 * VEC; base < total; base += 4 * 64 * VEC) {
        const int f = min(base + lane * VEC, total - VEC);
        const int cl = fdiv(f, PL, invPL);
        const int rem = f - cl * PL;
        if (rem >= PLD) continue;  // padding / reserved group: never copied
        const int lr = fdiv(rem, a.W, invW);
        const int w = rem - lr * a.W;
        const int2 ri = rinfo[lr];
        const int b = ri.x < 0 ? 0 : ri.x;
        const float* g = a.src + ((((int64_t)b * a.cin + c0 + cl) * a.H + ri.y) * a.W + w);
        dma<VEC>(g, raw + 4u * base);
    }
}

template <int WM>
__device__ __forceinline__ void issue_wts(const ConvArgs& a, unsigned wts, int c0, int n0, int wave,
                                          int lane, int CK) {
    constexpr int COUT_T = 32 * WM;
    const int total = 9 * CK * COUT_T;
    for (int base = wave * 256; base < total; base += 4 * 256) {
        const int f = min(base + lane * 4, total - 4);
        const int row = f / COUT_T, col = f - row * COUT_T;
        const int tap = row / CK, cc = row - tap * CK;
        dma<4>(a.wpack + ((int64_t)(tap * a.cin + c0 + cc)) * a.cout + n0 + col, wts + 4u * base);
    }
}

// Occupancy: latency hiding here comes from co-resident blocks (4 waves of a block share one
// chunk barrier), so the LDS footprint is sized for DMA_OCC(WM) blocks per CU and the register
// budget for as many waves per SIMD (measured: 4 resident blocks run the same GEMM at 72 % of the
// fp32 MFMA peak where 2 reach 60 %).
constexpr int dma_occ(int wm) { return wm == 2 ? 4 : 3; }

template <int WM, int WN, int VEC, int PRO, int EPI, int CK, bool PRE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(dma_occ(WM)))) void conv3x3_dma_kernel(ConvArgs a) {
    constexpr int COUT_T = 32 * WM;
    constexpr int BP = 4 * WN * 32;
    extern __shared__ __attribute__((aligned(16))) float smem[];
    // channel-plane stride of the staged image: dense rows (NR * W), or with PRE the row segments
    // of each sample placed at the 16-byte phase of their global address (host-computed bound);
    // + padding to 16 bytes + the reserved group at PZ (the value of out-of-sample taps)
    const int PZ = ((PRE ? a.RS : a.NR * a.W) + 3) & ~3;
    const int PL = PZ + 4;
    const int rawf = ((CK * PL + 64 * VEC - 1) / (64 * VEC)) * (64 * VEC);
    const int wtsf = ((9 * CK * COUT_T + 255) / 256) * 256;
    float4* cft = reinterpret_cast<float4*>(smem);                        // [cin]
    int2* rinfo = reinterpret_cast<int2*>(smem + 4 * a.cin);              // [NR] (padded to 4)
    int* rowpos = reinterpret_cast<int*>(smem + 4 * a.cin + ((2 * a.NR + 3) & ~3));  // [NR]
    int4* segt = reinterpret_cast<int4*>(rowpos + ((a.NR + 3) & ~3));    // [NR] {kstart, kend, goff, nseg}
    float* raw0 = smem + dma_table_floats(a.cin, a.NR);
    float* wts0 = raw0 + 2 * rawf;
    // LDS byte addresses of the DMA targets (M0 operand)
    const unsigned lds0 = (unsigned)(uintptr_t)(lds_void*)smem;
    const unsigned raw_lds = lds0 + 4u * (unsigned)(raw0 - smem);
    const unsigned wts_lds = lds0 + 4u * (unsigned)(wts0 - smem);

    const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, l32 = lane & 31;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int ny = a.cout / COUT_T;
    const int flat = xcd_remap(blockIdx.x, gridDim.x);
    const int tile = flat / ny;
    const int n0 = (flat - tile * ny) * COUT_T;
    const int64_t HW = (int64_t)a.H * a.W;
    const int64_t Mtot = (int64_t)a.B * HW;
    const int64_t m0 = (int64_t)tile * BP;
    const int64_t row0 = m0 / a.W - 1;
    const int64_t nrows = (int64_t)a.B * a.H;

    // ---- per-block tables (ordinary loads, all consumed before the first DMA is issued)
    if (PRO != PRO_RAW)
        for (int c = tid; c < a.cin; c += 256) cft[c] = a.cf_in[c];
    for (int lr = tid; lr < a.NR; lr += 256) {
        int64_t gr = row0 + lr;
        bool ok = gr >= 0 && gr < nrows;
        int b = ok ? (int)(gr / a.H) : -1;
        rinfo[lr] = make_int2(b, ok ? (int)(gr - (int64_t)b * a.H) : 0);
    }
    int pixoff[WN], prow[WN];
    bool vup[WN], vdn[WN], vl[WN], vr[WN], valid[WN];
    int pb[WN], pp[WN];
#pragma unroll
    for (int ni = 0; ni < WN; ++ni) {
        int64_t m = m0 + (wave * WN + ni) * 32 + l32;
        valid[ni] = m < Mtot;
        int64_t mm = valid[ni] ? m : Mtot - 1;
        int64_t gr = mm / a.W;
        int w = (int)(mm - gr * a.W);
        int b = (int)(gr / a.H);
        int hr = (int)(gr - (int64_t)b * a.H);
        prow[ni] = (int)(gr - row0);
        pixoff[ni] = w;
        vup[ni] = hr > 0;
        vdn[ni] = hr < a.H - 1;
        vl[ni] = w > 0;
        vr[ni] = w < a.W - 1;
        pb[ni] = b;
        pp[ni] = hr * a.W + w;
    }
    const int bf = row0 < 0 ? 0 : (int)(row0 / a.H);
    if constexpr (PRE) {
        // row segments (maximal runs of rows of one sample, or of invalid rows): a segment starts
        // on a fresh 16-byte group, its first row at the 16-byte phase of its global address, so
        // that every group of the image is one aligned dwordx4 copy of one segment
        __syncthreads();
        if (tid == 0) {
            int pos = 0, nseg = 0, pb_ = -2, ph_ = -2;
            for (int lr = 0; lr < a.NR; ++lr) {
                const int2 ri = rinfo[lr];
                if (lr == 0 || ri.x != pb_ || (ri.x >= 0 && ri.y != ph_ + 1)) {
                    if (nseg) segt[nseg - 1].y = (pos + 3) >> 2;
                    const int ks = (pos + 3) >> 2;
                    const int phase = ri.x >= 0 ? (ri.y * a.W) & 3 : 0;
                    const int goff = ri.x >= 0 ? (ri.x - bf) * a.cin * (int)HW + ri.y * a.W - phase : -1;
                    segt[nseg++] = make_int4(ks, 0, goff, 0);
                    pos = 4 * ks + phase;
                }
                rowpos[lr] = pos;
                pos += a.W;
                pb_ = ri.x;
                ph_ = ri.y;
            }
            segt[nseg - 1].y = (pos + 3) >> 2;
            segt[0].w = nseg;
        }
    }
    __syncthreads();
#pragma unroll
    for (int ni = 0; ni < WN; ++ni) pixoff[ni] += PRE ? rowpos[prow[ni]] : prow[ni] * a.W;

    f32x16 acc[WM][WN];
#pragma unroll
    for (int mi = 0; mi < WM; ++mi)
#pragma unroll
        for (int ni = 0; ni < WN; ++ni) acc[mi][ni] = f32x16{0.f};

    const int rawtotal = CK * PL;
    const float invPL = 1.f / PL, invW = 1.f / a.W;
    const int nchunk = a.cin / CK;
    constexpr int WTOT = 9 * CK * COUT_T;
    // precomputed copy offsets: raw rows relative to (first sample of the block, channel c0),
    // weights relative to (wpack + c0 * cout + n0)
    unsigned roff[PRE ? DMA_MAXR : 1], woff[PRE ? DMA_MAXW : 1];
    bool rskip[PRE ? DMA_MAXR : 1];
    if constexpr (PRE) {
        static_assert(!PRE || VEC == 4, "segment layout copies 16-byte groups");
        const int QP = PL / 4, nseg = segt[0].w;
        const float invQP = 1.f / QP;
#pragma unroll
        for (int j = 0; j < DMA_MAXR; ++j) {
            const int g = min(wave * 64 + j * 256 + lane, rawtotal / 4 - 1);
            const int cl = fdiv(g, QP, invQP);
            const int k = g - cl * QP;
            int4 sg = segt[0];
            for (int t = 1; t < nseg; ++t) {
                const int4 st = segt[t];
                if (k >= st.x) sg = st;
            }
            // gaps and invalid rows copy the channel's first group (in bounds, never read); the
            // reserved group is not copied at all
            const int off = cl * (int)HW + ((sg.z >= 0 && k < sg.y) ? sg.z + 4 * (k - sg.x) : 0);
            roff[j] = 4u * (unsigned)off;
            rskip[j] = k == QP - 1;
        }
#pragma unroll
        for (int j = 0; j < DMA_MAXW; ++j) {
            const int f = min(wave * 256 + j * 1024 + lane * 4, WTOT - 4);
            const int row = f / COUT_T, col = f - row * COUT_T;
            const int tap = row / CK, cc = row - tap * CK;
            woff[j] = 4u * (unsigned)((tap * a.cin + cc) * a.cout + col);
        }
    }
    auto issue = [&](int c0, unsigned nb) {
        if constexpr (PRE) {
            const float* sr = uniform_ptr(a.src + ((int64_t)bf * a.cin + c0) * HW);
            const float* sw = uniform_ptr(a.wpack + (int64_t)c0 * a.cout + n0);
#pragma unroll
            for (int j = 0; j < DMA_MAXR; ++j) {
                const int base = wave * 64 * VEC + j * 256 * VEC;
                if (base < rawtotal && !rskip[j]) dma_s<VEC>(sr, roff[j], raw_lds + nb * 4u * rawf + 4u * base);
            }
#pragma unroll
            for (int j = 0; j < DMA_MAXW; ++j) {
                const int base = wave * 256 + j * 1024;
                if (base < WTOT) dma_s<4>(sw, woff[j], wts_lds + nb * 4u * wtsf + 4u * base);
            }
        } else {
            issue_raw<VEC>(a, rinfo, raw_lds + nb * 4u * rawf, c0, wave, lane, rawtotal, PL, invPL, invW);
            issue_wts<WM>(a, wts_lds + nb * 4u * wtsf, c0, n0, wave, lane, CK);
        }
    };
    // reserved groups of both buffers (ordered before any read by the first chunk barrier; the
    // copies never write them)
    for (int i = tid; i < 2 * CK * 4; i += 256) {
        const int buf = i / (CK * 4), r = i - buf * CK * 4;
        raw0[buf * rawf + (r >> 2) * PL + PZ + (r & 3)] = PRO == PRO_RAW ? 0.f : __builtin_nanf("");
    }
    issue(0, 0u);
    for (int k = 0; k < nchunk; ++k) {
        const int c0 = k * CK;
        float* raw = raw0 + (k & 1) * rawf;
        float* wts = wts0 + (k & 1) * wtsf;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();  // chunk k visible to all waves; chunk k-1 fully consumed
        if (k + 1 < nchunk) issue(c0 + CK, (unsigned)((k + 1) & 1));
        float4 cf[CK / 2];
        if (PRO != PRO_RAW) {
#pragma unroll
            for (int s = 0; s < CK / 2; ++s) cf[s] = cft[c0 + 2 * s + h];
        }
        // (tap, s) steps, software-pipelined by hand: the LDS operands of step i+1 are requested
        // before the MFMAs of step i (sched_barrier keeps the scheduler from sinking the reads
        // next to their use, which exposes the LDS latency in front of the MFMAs)
        constexpr int NST = 9 * (CK / 2);
        float av[2][WM], rv[2][WN];
        auto load = [&](int st, float (&a_)[WM], float (&r_)[WN]) {
            const int tap = st / (CK / 2), s = st % (CK / 2);
            const int dh = tap / 3 - 1, dw = tap % 3 - 1;
            const int toff = dh * a.W + dw;
#pragma unroll
            for (int mi = 0; mi < WM; ++mi) a_[mi] = wts[(tap * CK + 2 * s + h) * COUT_T + mi * 32 + l32];
#pragma unroll
            for (int ni = 0; ni < WN; ++ni) {
                bool ok = true;
                if (dh < 0) ok = ok && vup[ni];
                if (dh > 0) ok = ok && vdn[ni];
                if (dw < 0) ok = ok && vl[ni];
                if (dw > 0) ok = ok && vr[ni];
                r_[ni] = raw[(2 * s + h) * PL + (ok ? pixoff[ni] + toff : PZ)];
            }
        };
        load(0, av[0], rv[0]);
#pragma unroll
        for (int st = 0; st < NST; ++st) {
            const int cur = st & 1;
            if (st + 1 < NST) load(st + 1, av[cur ^ 1], rv[cur ^ 1]);
            __builtin_amdgcn_sched_barrier(0);
            const int s = st % (CK / 2);
            float bv[WN];
#pragma unroll
            for (int ni = 0; ni < WN; ++ni)
                bv[ni] = PRO == PRO_RAW ? rv[cur][ni] : fmaxf(fmaf(rv[cur][ni], cf[s].x, cf[s].y), 0.f);
#pragma unroll
            for (int mi = 0; mi < WM; ++mi)
#pragma unroll
                for (int ni = 0; ni < WN; ++ni) acc[mi][ni] = mfma32(av[cur][mi], bv[ni], acc[mi][ni]);
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    __syncthreads();  // LDS is reused for the cross-wave statistics
    conv_epilogue<WM, WN, EPI>(a, acc, smem, tile, n0, m0, Mtot, HW, wave, tid, valid, pb, pp);
}

// ------------------------------------------------------------------ BN + ReLU + MaxPool2 + Dropout2d
// x[b,c,h,w] = drop[b,c] * max_{2x2} relu(y*s + t)  (reference block tail phoneme_cnn.py:40-43)
// One block per group of PPB channel planes; thread = 4 pooled outputs of one row (8 input columns
// of two rows).  VEC4: source rows 16-byte aligned (Ws % 4 == 0) -> four 16-byte loads per thread;
// otherwise paired / scalar loads.  32-bit index math only.
template <int VEC, int NI>
__global__ __launch_bounds__(256) void bn_relu_pool_kernel(const float* __restrict__ y, const float4* __restrict__ cf,
                                                           const float* __restrict__ drop, float* __restrict__ x,
                                                           int nplanes, int C, int Hs, int Ws, int Hp, int Wp, int ppb,
                                                           float* __restrict__ ysel, uint8_t* __restrict__ parg) {
    const int Wq = (Wp + 3) / 4, nqp = Hp * Wq;
    const int pbase = blockIdx.x * ppb;
    const int tot = min(ppb, nplanes - pbase) * nqp;
    // NI quads per thread per pass, all loads of a pass issued before any arithmetic (the pass keeps
    // NI x 64 bytes per thread in flight instead of 64)
    for (int t0 = threadIdx.x; t0 < tot; t0 += NI * blockDim.x) {
        float u[NI][8], v[NI][8];
        int bcs[NI], hps[NI], qs[NI];
#pragma unroll
        for (int n = 0; n < NI; ++n) {
            const int t = min(t0 + n * (int)blockDim.x, tot - 1);  // (a tail item repeats the last quad: same values)
            const int pl = t / nqp, rem = t - pl * nqp;
            const int hp = rem / Wq, q = rem - hp * Wq;
            const int bc = pbase + pl;
            bcs[n] = bc; hps[n] = hp; qs[n] = q;
            const float* s0 = y + ((int64_t)bc * Hs + 2 * hp) * Ws + 8 * q;
            const float* s1 = s0 + Ws;
            if (VEC == 4 && 8 * q + 8 <= Ws) {
                const float4 a0 = ld4(s0), a1 = ld4(s0 + 4), b0 = ld4(s1), b1 = ld4(s1 + 4);
                u[n][0] = a0.x; u[n][1] = a0.y; u[n][2] = a0.z; u[n][3] = a0.w;
                u[n][4] = a1.x; u[n][5] = a1.y; u[n][6] = a1.z; u[n][7] = a1.w;
                v[n][0] = b0.x; v[n][1] = b0.y; v[n][2] = b0.z; v[n][3] = b0.w;
                v[n][4] = b1.x; v[n][5] = b1.y; v[n][6] = b1.z; v[n][7] = b1.w;
            } else if (VEC >= 2) {
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const bool ok = 8 * q + 2 * j + 1 < Ws;
                    const float2 a0 = ok ? *reinterpret_cast<const float2*>(s0 + 2 * j) : make_float2(0.f, 0.f);
                    const float2 b0 = ok ? *reinterpret_cast<const float2*>(s1 + 2 * j) : make_float2(0.f, 0.f);
                    u[n][2 * j] = a0.x; u[n][2 * j + 1] = a0.y; v[n][2 * j] = b0.x; v[n][2 * j + 1] = b0.y;
                }
            } else {
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    const bool ok = 8 * q + e < 2 * Wp;
                    u[n][e] = ok ? s0[e] : 0.f;
                    v[n][e] = ok ? s1[e] : 0.f;
                }
            }
        }
#pragma unroll
        for (int n = 0; n < NI; ++n) {
            if (t0 + n * (int)blockDim.x >= tot) break;
            const int bc = bcs[n], hp = hps[n], q = qs[n];
            const float4 k = cf[bc % C];
            const float d = drop ? drop[bc] : 1.f;
            float out[4], ya[4];
            unsigned ag = 0;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                // first maximum of relu(BN) in window scan order (torch max_pool2d; the data gradient's rule)
                const float q0 = fmaxf(fmaf(u[n][2 * j], k.x, k.y), 0.f), q1 = fmaxf(fmaf(u[n][2 * j + 1], k.x, k.y), 0.f);
                const float q2 = fmaxf(fmaf(v[n][2 * j], k.x, k.y), 0.f), q3 = fmaxf(fmaf(v[n][2 * j + 1], k.x, k.y), 0.f);
                float best = q0, yy = u[n][2 * j];
                unsigned arg = 0;
                if (q1 > best) { best = q1; arg = 1; yy = u[n][2 * j + 1]; }
                if (q2 > best) { best = q2; arg = 2; yy = v[n][2 * j]; }
                if (q3 > best) { best = q3; arg = 3; yy = v[n][2 * j + 1]; }
                out[j] = d * best;
                ya[j] = yy;
                ag |= arg << (8 * j);
            }
            const int64_t po = ((int64_t)bc * Hp + hp) * Wp + 4 * q;
            float* dst = x + po;
            if ((Wp & 3) == 0) {
                st4(dst, make_float4(out[0], out[1], out[2], out[3]));
                if (ysel) {
                    st4(ysel + po, make_float4(ya[0], ya[1], ya[2], ya[3]));
                    *reinterpret_cast<unsigned*>(parg + po) = ag;
                }
            } else if ((Wp & 1) == 0) {  // 8-byte aligned pairs (the quad's second pair may lie past the row)
#pragma unroll
                for (int j = 0; j < 4; j += 2)
                    if (4 * q + j < Wp) {
                        *reinterpret_cast<float2*>(dst + j) = make_float2(out[j], out[j + 1]);
                        if (ysel) {
                            *reinterpret_cast<float2*>(ysel + po + j) = make_float2(ya[j], ya[j + 1]);
                            *reinterpret_cast<uint16_t*>(parg + po + j) = (uint16_t)(ag >> (8 * j));
                        }
                    }
            } else {
                for (int j = 0; j < 4 && 4 * q + j < Wp; ++j) {
                    dst[j] = out[j];
                    if (ysel) {
                        ysel[po + j] = ya[j];
                        parg[po + j] = (uint8_t)(ag >> (8 * j));
                    }
                }
            }
        }
    }
}

}  // namespace

int conv3x3_dma_ck(int cout, int PL, int NR, int cin) {
    // largest K-chunk whose double-buffered raw image + weights let dma_occ blocks share a CU
    const int cout_t = cout == 32 ? 32 : 64;
    for (int ck = 8; ck >= 2; ck >>= 1) {
        if (cin % ck) continue;
        size_t raw = (size_t)ck * PL + 256;
        size_t wts = (size_t)9 * ck * cout_t + 256;
        size_t bytes = (2 * raw + 2 * wts + (size_t)dma_table_floats(cin, NR)) * 4;
        if (bytes <= (size_t)160 * 1024 / dma_occ(cout == 32 ? 1 : 2)) return ck;
    }
    return 2;
}

int launch_conv3x3_dma(int pro, int epi, ConvArgs a, hipStream_t s) {
    PCX_CHECK_ARG(a.cout == 32 || a.cout % 64 == 0, "conv3x3: cout %d unsupported", a.cout);
    PCX_CHECK_ARG(pro == PRO_RAW || pro == PRO_BNRELU, "conv3x3_dma: prologue %d", pro);
    const int wm = a.cout == 32 ? 1 : 2, wn = a.cout == 32 ? 4 : 2;
    const int bp = 4 * wn * 32, cout_t = 32 * wm;
    const int64_t M = (int64_t)a.B * a.H * a.W;
    const int ntile = ceil_div(M, bp);
    PCX_CHECK_ARG(a.nblk == ntile, "conv3x3: partial buffer sized for %d tiles, need %d", a.nblk, ntile);
    a.NR = (bp - 1 + a.W - 1) / a.W + 1 + 2;
    // Preferred: segment layout (16-byte copies at any W, offsets precomputed per tile).  A tile's
    // rows span at most NR / H + 2 samples plus an invalid run at either end; each segment costs
    // at most 7 floats of alignment gap.
    const int64_t HW = (int64_t)a.H * a.W;
    // (channel planes of the staged image carry one more 16-byte group: the reserved value of
    // out-of-sample taps)
    const int PLseg = ((a.NR * a.W + 8 * (a.NR / a.H + 4)) + 3) & ~3;
    int ck = conv3x3_dma_ck(a.cout, PLseg + 4, a.NR, a.cin);
    bool pre = HW % 4 == 0 && a.cin % ck == 0 && ceil_div(ck * (PLseg + 4), 1024) <= DMA_MAXR &&
               ceil_div(9 * ck * cout_t, 1024) <= DMA_MAXW &&
               (int64_t)((a.NR / a.H + 3) * a.cin) * HW * 4 < ((int64_t)1 << 31);
    int vec = 4, PL = PLseg + 4;
    if (pre) {
        a.RS = PLseg;
    } else {
        vec = (a.W % 4 == 0) ? 4 : 1;
        PL = ((a.NR * a.W + 3) & ~3) + 4;
        ck = conv3x3_dma_ck(a.cout, PL, a.NR, a.cin);
    }
    PCX_CHECK_ARG(a.cin % ck == 0, "conv3x3: cin %d not a multiple of %d", a.cin, ck);
    const int rawf = ((ck * PL + 64 * vec - 1) / (64 * vec)) * (64 * vec);
    const int wtsf = ((9 * ck * cout_t + 255) / 256) * 256;
    size_t smem = ((size_t)dma_table_floats(a.cin, a.NR) + 2 * (size_t)rawf + 2 * (size_t)wtsf) * 4;
    size_t red = ((size_t)4 * cout_t * 3 + 4 * (size_t)cout_t) * 4;  // epilogue partials + cf table
    if (smem < red) smem = red;
    PCX_CHECK_ARG(smem <= 160 * 1024, "conv3x3_dma: W=%d needs %zu B of LDS", a.W, smem);
    dim3 grid((unsigned)(ntile * (a.cout / cout_t)));
#define PCX_DMA_CASE(WM_, WN_, V_, P_, E_, CK_)                                                   \
    if (wm == WM_ && vec == V_ && pro == P_ && epi == E_ && ck == CK_) {                         \
        if constexpr (V_ == 4) if (pre) {                                                        \
            (void)hipFuncSetAttribute((const void*)conv3x3_dma_kernel<WM_, WN_, V_, P_, E_, CK_, true>, \
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);    \
            conv3x3_dma_kernel<WM_, WN_, V_, P_, E_, CK_, true><<<grid, 256, smem, s>>>(a);      \
            PCX_LAUNCH_CHECK("conv3x3_dma_kernel");                                              \
            return PCX_OK;                                                                       \
        }                                                                                        \
        {                                                                                        \
            (void)hipFuncSetAttribute((const void*)conv3x3_dma_kernel<WM_, WN_, V_, P_, E_, CK_, false>, \
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);    \
            conv3x3_dma_kernel<WM_, WN_, V_, P_, E_, CK_, false><<<grid, 256, smem, s>>>(a);     \
        }                                                                                        \
        PCX_LAUNCH_CHECK("conv3x3_dma_kernel");                                                  \
        return PCX_OK;                                                                           \
    }
#define PCX_DMA_CK(WM_, WN_, V_, P_, E_) \
    PCX_DMA_CASE(WM_, WN_, V_, P_, E_, 8) PCX_DMA_CASE(WM_, WN_, V_, P_, E_, 4) PCX_DMA_CASE(WM_, WN_, V_, P_, E_, 2)
#define PCX_DMA_V(WM_, WN_, P_, E_) PCX_DMA_CK(WM_, WN_, 4, P_, E_) PCX_DMA_CK(WM_, WN_, 1, P_, E_)
#define PCX_DMA_ALL(P_, E_) PCX_DMA_V(1, 4, P_, E_) PCX_DMA_V(2, 2, P_, E_)
    PCX_DMA_ALL(PRO_RAW, EPI_FWD)
    PCX_DMA_ALL(PRO_BNRELU, EPI_FWD)
    PCX_DMA_ALL(PRO_RAW, EPI_BWD_RELU)   // data gradient on the dy materialised by the wgrad
    PCX_DMA_ALL(PRO_RAW, EPI_BWD_POOL)
    PCX_DMA_ALL(PRO_RAW, EPI_BWD_STORE)  // cnn_deep's stride-1 3x3 data gradients
#undef PCX_DMA_ALL
#undef PCX_DMA_V
#undef PCX_DMA_CK
#undef PCX_DMA_CASE
    set_error("conv3x3_dma: unsupported combination (pro %d epi %d ck %d vec %d)", pro, epi, ck, vec);
    return PCX_EINVAL;
}

// x = drop[b, c] relu(ysel s_c + t_c) at the pooled resolution: bn_relu_pool_kernel's output value at the window's
// selected element (the same fmaf, the same product with the dropout factor).  Four 16-byte loads per thread in
// flight per step, nontemporal stores (the streaming-copy probe's shape: one load per step ran at 4.7 TB/s).
constexpr int PA_U = 4;
__global__ __launch_bounds__(256) void pool_act_kernel(const float4* __restrict__ ysel, const float4* __restrict__ cf,
                                                       const float* __restrict__ drop, float4* __restrict__ x, int C,
                                                       int q4, int64_t n4) {
    const int64_t stride = (int64_t)gridDim.x * 256;
    for (int64_t i0 = (int64_t)blockIdx.x * 256 + threadIdx.x; i0 < n4; i0 += PA_U * stride) {
        float4 v[PA_U];
#pragma unroll
        for (int u = 0; u < PA_U; ++u) {
            const int64_t i = i0 + u * stride;
            typedef float pa_f4 __attribute__((ext_vector_type(4)));
            const pa_f4 t = i < n4 ? __builtin_nontemporal_load(reinterpret_cast<const pa_f4*>(ysel) + i) : pa_f4{0.f, 0.f, 0.f, 0.f};
            v[u] = make_float4(t.x, t.y, t.z, t.w);
        }
#pragma unroll
        for (int u = 0; u < PA_U; ++u) {
            const int64_t i = i0 + u * stride;
            if (i >= n4) break;
            const int bc = (int)udiv32(i, q4);
            const float4 k = cf[bc % C];
            const float d = drop ? drop[bc] : 1.f;
            float4 o;
            o.x = d * fmaxf(fmaf(v[u].x, k.x, k.y), 0.f);
            o.y = d * fmaxf(fmaf(v[u].y, k.x, k.y), 0.f);
            o.z = d * fmaxf(fmaf(v[u].z, k.x, k.y), 0.f);
            o.w = d * fmaxf(fmaf(v[u].w, k.x, k.y), 0.f);
            typedef float pa_f4 __attribute__((ext_vector_type(4)));
            __builtin_nontemporal_store(pa_f4{o.x, o.y, o.z, o.w}, reinterpret_cast<pa_f4*>(x) + i);
        }
    }
}

int launch_pool_act(const float* ysel, const float4* cf, const float* drop, float* x, int B, int C, int HWp,
                    hipStream_t s) {
    PCX_CHECK_ARG(HWp % 4 == 0 && (int64_t)B * C * HWp < ((int64_t)1 << 31), "pool_act: %d x %d planes of %d pixels",
                  B, C, HWp);
    const int64_t n4 = (int64_t)B * C * (HWp / 4);
    const int blocks = (int)std::min<int64_t>(ceil_div(n4, (int64_t)256 * PA_U), (int64_t)num_cus() * 16);
    pool_act_kernel<<<blocks, 256, 0, s>>>(reinterpret_cast<const float4*>(ysel), cf, drop,
                                           reinterpret_cast<float4*>(x), C, HWp / 4, n4);
    PCX_LAUNCH_CHECK("pool_act_kernel");
    return PCX_OK;
}

int launch_bn_relu_pool(const float* y, const float4* cf, const float* drop, float* x, int B, int C,
                        int Hs, int Ws, hipStream_t s, float* ysel, uint8_t* parg) {
    PCX_CHECK_ARG((ysel == nullptr) == (parg == nullptr), "bn_relu_pool: ysel and parg go together");
    const int Hp = Hs / 2, Wp = Ws / 2;
    PCX_CHECK_ARG((int64_t)B * C < ((int64_t)1 << 31), "bn_relu_pool: too many planes");
    const int nplanes = B * C, nqp = Hp * ((Wp + 3) / 4);
    const int ppb = std::max(1, 1024 / std::max(1, nqp));  // ~1024 quads per block
    const int blocks = ceil_div(nplanes, ppb);
    constexpr int ni = PCX_AB_POOL_NI;
#define PCX_BRP(V_, NI_)                                                                                       \
    bn_relu_pool_kernel<V_, NI_><<<blocks, 256, 0, s>>>(y, cf, drop, x, nplanes, C, Hs, Ws, Hp, Wp, ppb, ysel, parg)
    const int v = Ws % 4 == 0 ? 4 : Ws % 2 == 0 ? 2 : 1;
    if (ni == 1) {
        if (v == 4) PCX_BRP(4, 1); else if (v == 2) PCX_BRP(2, 1); else PCX_BRP(1, 1);
    } else {
        if (v == 4) PCX_BRP(4, 2); else if (v == 2) PCX_BRP(2, 2); else PCX_BRP(1, 2);
    }
#undef PCX_BRP
    PCX_LAUNCH_CHECK("bn_relu_pool_kernel");
    return PCX_OK;
}

}  // namespace pcx
