// Channel-last bf16 convolution engine for PhonemeNetDeep with precision "bf16" (SURVEY 8(f) row 2).
//
// The general bf16 implicit GEMM (convg_bf16.hip) gathers its operands from planar NCHW float32:
// every k of a GEMM row is a different channel plane, so each element is its own 4-byte load and
// the kernel runs at ~10 % of the bf16 MFMA roof.  Here each conv operand is first written once as a
// zero-padded channel-last bf16 image
//
//     xn[b][h + 1][w + 1][c]   (h in [-1, H], w in [-1, W]; the ring is zero = the conv padding)
//
// by to_nhwc_kernel (optionally applying the BN backward dy = a (g - mb - (y - mean) mgi) on the
// way, which replaces the float32 dy pass), and the GEMMs read it in 16-byte runs of 8 channels:
//  * forward (mode 0) / data gradient (mode 1, stride 1; mode 3, one parity class of stride 2):
//    M = output channels, N = pixels, K = taps x channels (tap-major, 32 channels per chunk).  A
//    pixel's operand row for a tap is one contiguous 64-byte run at a tap offset that is the same
//    for every pixel, so the B tile costs two 16-byte loads per thread and no bounds tests (the
//    ring supplies the zeros);
//  * weight gradient (mode 2): M = cout, N = taps x cin, K = pixels.  Both operands are staged
//    pixel-major ([k][channels], 16-byte runs) and read K-contiguous by ds_read_b64_tr_b16.
// Operand rounding (bf16 round-to-nearest-even of the float32 value) and float32 accumulation are
// those of convg_bf16; only the summation order differs.
#include "conv_epilogue.h"
#include "kernels.h"

namespace pcx {
namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));

constexpr int NKB = 32;  // k per chunk

__device__ __forceinline__ bf16x8 ld16(const __bf16* p) { return *reinterpret_cast<const bf16x8*>(p); }

__device__ __forceinline__ f32x16 mfma_bf16(bf16x8 a, bf16x8 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// ------------------------------------------------------------------ NCHW float32 -> padded NHWC bf16
// Block: one sample x 64 channels, row by row, each row transposed through LDS.  The value written is
//   NHWC_COPY   src
//   NHWC_BNBWD  a (src - mb - (y - mean) mgi)                 (BN backward, cf = {a, mb, mgi, mean})
//   NHWC_ACT    drop[b,c] relu(src s + t + res')  res' = res rs + rt | res | 0   (bn_act, cf = {s, t})
// and NHWC_ACT can also store its float32 NCHW result (out32).  Each thread issues its V-wide loads
// of a batch before any LDS write, so a block's reads are all in flight together.
template <int V, int OP>
__global__ __launch_bounds__(256) void to_nhwc_kernel(NhwcArgs a) {
    extern __shared__ float t[];  // [64][W + 1]
    typedef float fv __attribute__((ext_vector_type(V)));
    const int Hp = a.H + 2, Wp = a.W + 2;
    const int b = blockIdx.x;
    const int c0 = blockIdx.y * 64, nc = min(64, a.C - c0), ng = nc >> 3;
    __bf16* dimg = static_cast<__bf16*>(a.dst) + (int64_t)b * Hp * Wp * a.C + c0;
    const bool two = OP == NHWC_BNBWD && a.dst_b != nullptr;
    __bf16* dimg2 = two ? static_cast<__bf16*>(a.dst_b) + (int64_t)b * Hp * Wp * a.C + c0 : nullptr;
    // per-channel coefficients in LDS first: the element loop then waits on nothing but its loads
    __shared__ float4 kc[64], kr[64], kc2[64];
    __shared__ float kd[64];
    if (OP != NHWC_COPY && threadIdx.x < nc) {
        const int c = c0 + threadIdx.x;
        kc[threadIdx.x] = a.cf[c];
        if (two) kc2[threadIdx.x] = a.cf_b[c];
        if (OP == NHWC_ACT || (OP == NHWC_BNBWD && a.mcf)) {
            kr[threadIdx.x] = OP == NHWC_ACT ? (a.rcf ? a.rcf[c] : make_float4(1.f, 0.f, 0.f, 0.f)) : a.mcf[c];
            kd[threadIdx.x] = a.drop ? a.drop[(int64_t)b * a.C + c] : 1.f;
        }
    }
    // the zero ring rows
    for (int i = threadIdx.x; i < 2 * Wp * ng; i += 256) {
        const int r = i / (Wp * ng), j = i - r * (Wp * ng);
        const int wp = j / ng, g = j - wp * ng;
        *reinterpret_cast<bf16x8*>(dimg + ((int64_t)r * (Hp - 1) * Wp + wp) * a.C + 8 * g) = bf16x8{};
        if (two) *reinterpret_cast<bf16x8*>(dimg2 + ((int64_t)r * (Hp - 1) * Wp + wp) * a.C + 8 * g) = bf16x8{};
    }
    // LDS tile [64][TW] with channel c's run of R image rows at c TW + 4 (c >> 3): TW a multiple of 4
    // keeps the V-wide writes aligned, and the 4 (c >> 3) shift puts the 8 channel rows a row-out read
    // touches (lanes g = 0..7 of one pixel, 4 pixels per 32 lanes) on 32 different banks.  R (a.rows,
    // set by the launcher) image rows per step: narrow images (W = 50, 25, 13) fill a step with the same
    // number of loads as a 100-wide row (the R rows of a channel are contiguous in NCHW).
    const int W = a.W, R = a.rows, TW = (R * W + 3) & ~3, nv = W / V;
    float* t2 = t + 64 * TW + 32;  // (two: the second image's tile)
    const int64_t HW = (int64_t)a.H * W;
    const int64_t pbase = ((int64_t)b * a.C + c0) * HW;
    constexpr int U = 4;
    // the block walks its sample's rows: consecutive rows of the same 64 planes (page / line reuse)
    float* rres = t + (two ? 2 : 1) * (64 * TW + 32);  // res_pool (R = 1): the row's residual, transposed like t
    for (int h0 = 0; h0 < a.H; h0 += R) {
        const int h = h0;
        const int Rr = min(R, a.H - h0), nvr = Rr * nv, n = nc * nvr;
        const int64_t base = pbase + (int64_t)h0 * W;
        if (OP == NHWC_ACT && a.res_pool) {  // pooled NHWC row (b, h): 16-byte runs of 4 channels, coalesced
            const float* rrow = a.res + ((int64_t)b * a.H + h) * W * a.C + c0;
            const int nq = W * (nc >> 2);
            for (int k = threadIdx.x; k < nq; k += 256) {
                const int w = k / (nc >> 2), c4 = (k - w * (nc >> 2)) * 4;
                const float4 r4 = *reinterpret_cast<const float4*>(rrow + (int64_t)w * a.C + c4);
                rres[c4 * TW + 4 * (c4 >> 3) + w] = r4.x;
                rres[(c4 + 1) * TW + 4 * ((c4 + 1) >> 3) + w] = r4.y;
                rres[(c4 + 2) * TW + 4 * ((c4 + 2) >> 3) + w] = r4.z;
                rres[(c4 + 3) * TW + 4 * ((c4 + 3) >> 3) + w] = r4.w;
            }
        }
        __syncthreads();  // (coefficients ready; previous row's LDS reads done)
        for (int i0 = 0; i0 < n; i0 += U * 256) {
            fv x[U], y2[U], y3[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {  // (tail items load a valid element and are dropped below)
                const int i = min(i0 + u * 256 + (int)threadIdx.x, n - 1);
                const int c = i / nvr, w0 = (i - c * nvr) * V;
                const int64_t o = base + c * HW + w0;
                x[u] = *reinterpret_cast<const fv*>(a.src + o);
                if (OP == NHWC_BNBWD) y2[u] = *reinterpret_cast<const fv*>(a.y + o);
                if (OP == NHWC_BNBWD && two) y3[u] = *reinterpret_cast<const fv*>(a.y_b + o);
                if (OP == NHWC_ACT) {
                    if (a.res_pool) {  // staged above (transposed)
                        y2[u] = *reinterpret_cast<const fv*>(rres + c * TW + 4 * (c >> 3) + w0);
                    } else {
                        y2[u] = a.res ? *reinterpret_cast<const fv*>(a.res + o) : fv{};
                    }
                }
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int i = i0 + u * 256 + (int)threadIdx.x;
                if (i < n) {
                    const int c = i / nvr, w0 = (i - c * nvr) * V;
                    fv v = x[u];
                    if (OP == NHWC_BNBWD) {
                        const float4 k = kc[c];
                        if (a.mcf) {  // the ReLU / Dropout2d backward of the BN output (bwd_prep_kernel's MASK_BN)
                            const float4 mk = kr[c];
                            const float d = kd[c];
#pragma unroll
                            for (int e = 0; e < V; ++e) v[e] = fmaf(y2[u][e], mk.x, mk.y) > 0.f ? v[e] * d : 0.f;
                        }
                        if (two) {
                            const float4 k2 = kc2[c];
                            fv v2;
#pragma unroll
                            for (int e = 0; e < V; ++e) v2[e] = k2.x * (v[e] - k2.y - (y3[u][e] - k2.w) * k2.z);
                            *reinterpret_cast<fv*>(t2 + c * TW + 4 * (c >> 3) + w0) = v2;
                        }
#pragma unroll
                        for (int e = 0; e < V; ++e) v[e] = k.x * (v[e] - k.y - (y2[u][e] - k.w) * k.z);
                    } else if (OP == NHWC_ACT) {
                        const float4 k = kc[c], rk = kr[c];
                        const float d = kd[c];
#pragma unroll
                        for (int e = 0; e < V; ++e) {
                            float r = fmaf(v[e], k.x, k.y);
                            if (a.res_pool) r += fmaxf(fmaf(y2[u][e], rk.x, rk.y), 0.f);
                            else if (a.res) r += fmaf(y2[u][e], rk.x, rk.y);
                            v[e] = d * fmaxf(r, 0.f);
                        }
                        if (a.out32) *reinterpret_cast<fv*>(a.out32 + base + c * HW + w0) = v;
                        if (a.mask8) {
                            unsigned mb = 0;
#pragma unroll
                            for (int e = 0; e < V; ++e) mb |= (v[e] > 0.f ? 1u : 0u) << (8 * e);
                            uint8_t* mp = a.mask8 + base + c * HW + w0;
                            if (V == 4) *reinterpret_cast<unsigned*>(mp) = mb;
                            else if (V == 2) *reinterpret_cast<uint16_t*>(mp) = (uint16_t)mb;
                            else *mp = (uint8_t)mb;
                        }
                    }
                    *reinterpret_cast<fv*>(t + c * TW + 4 * (c >> 3) + w0) = v;
                }
            }
        }
        __syncthreads();
        for (int i = threadIdx.x; i < Rr * Wp * ng; i += 256) {
            const int hr = i / (Wp * ng), i2 = i - hr * (Wp * ng);
            const int wp = i2 / ng, g = i2 - wp * ng;
            const int px = hr * W + wp - 1;  // the pixel within the step's rows
            bf16x8 o{};
            if (wp > 0 && wp <= W) {
#pragma unroll
                for (int j = 0; j < 8; ++j) o[j] = (__bf16)t[(8 * g + j) * TW + 4 * g + px];
            }
            const int64_t ro = ((int64_t)(h0 + hr + 1) * Wp + wp) * a.C + 8 * g;
            *reinterpret_cast<bf16x8*>(dimg + ro) = o;
            if (two) {
                bf16x8 o2{};
                if (wp > 0 && wp <= W) {
#pragma unroll
                    for (int j = 0; j < 8; ++j) o2[j] = (__bf16)t2[(8 * g + j) * TW + 4 * g + px];
                }
                *reinterpret_cast<bf16x8*>(dimg2 + ro) = o2;
            }
        }
    }
}

// ------------------------------------------------------------------ forward / data gradient
// Operand tiles are copied HBM/L2 -> LDS by global_load_lds_dwordx4 (no VGPR staging, no LDS store
// instructions), double-buffered: the copy of chunk k + 1 runs under the MFMAs of chunk k.  A DMA
// wave-instruction fills 1 KB of LDS contiguously (lane L -> byte 16 L), i.e. 16 rows of 64 bytes
// (32 bf16 of k); each lane picks the global 16-byte run that belongs in its slot, which lets the
// rows be XOR-swizzled instead of padded: logical run q of row r sits in slot q ^ ((r >> 2) & 3),
// so the MFMA operand reads (ds_read_b128, rows l32, run 2 ks + h) are conflict-free.
typedef __attribute__((address_space(3))) void lds_void;

__device__ __forceinline__ void dma16(const __bf16* g, unsigned lds_byte_addr) {
    // inline asm: the builtin would make the waitcnt pass wait for every DMA before each ds_read
    const unsigned m0 = __builtin_amdgcn_readfirstlane(lds_byte_addr);
    asm volatile("s_nop 0\n\tglobal_load_lds_dwordx4 %0, off" :: "v"(g), "{m0}"(m0) : "memory");
}

// rows of KC bf16 (64 / 128 bytes): logical 16-byte run q of row r in slot q ^ f(r); f spreads the
// rows one ds_read_b128 lane group reads over all 64 banks
template <int KC>
__device__ __forceinline__ int swz(int r, int q) {
    return KC == 32 ? r * 64 + 16 * (q ^ ((r >> 2) & 3)) : r * 128 + 16 * (q ^ ((r >> 1) & 7));
}

// Workgroups are dealt to the 8 XCDs round-robin and each XCD has its own L2.  Launch 8 * per
// workgroups and give XCD x the logical blocks [x per, (x + 1) per): the blocks that share operand rows
// (the M tiles of a pixel tile; the N tiles of a weight-gradient K slice) are consecutive in logical
// order, so they run on one XCD at about the same time and read those rows from its L2 instead of HBM.
__host__ __device__ inline int64_t xcd_per(int64_t nblocks) { return (nblocks + 7) / 8; }
__device__ __forceinline__ int64_t xcd_logical(int64_t nblocks) {
    const int64_t bid = blockIdx.x;
    return (bid & 7) * xcd_per(nblocks) + (bid >> 3);
}

// Epilogue of the forward / data-gradient kernels: planar NCHW float32 stores (columns = pixels:
// 128-byte rows per MFMA output row), optionally the producer BN's backward sums (EP, mode 1) or the BN
// forward partials (mode 0).  col[ni]: the flattened pixel of the lane's column (a valid pixel even where
// valid[ni] is false), cnt_w: valid pixels among the wave's 32 WN columns, tn of ntile: the partials' tile.
// bs >= 0 (the halo kernel, modes 0 / 1): every column of the tile is a pixel of sample bs, and col[] holds the
// pixel's index inside that sample -- no per-lane 64-bit division (round 6: ~100 VALU per column).
template <int MODE, int WM, int WN, bool EP, int NWC = 2>
__device__ __forceinline__ void convn_epilogue(const ConvGArgs& a, const f32x16 (&acc)[WM][WN], char* smem, int64_t m0,
                                               int64_t M, const int64_t (&col)[WN], const bool (&valid)[WN], int cnt_w,
                                               int64_t ntile, int64_t tn, int64_t tm, int bs = -1) {
    // (NWC wave columns of 32 WN pixels, two wave rows of 32 WM output rows)
    constexpr int BM = 64 * WM;
    const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, l32 = lane & 31;
    const int wave = tid >> 6, wr = wave / NWC, wc = wave % NWC;
    const int ph = a.par >> 1, pw = a.par & 1;
    const int64_t OHW = (int64_t)a.OH * a.OW, IHW = (int64_t)a.IH * a.IW;
    const int IHc = (a.IH - ph + 1) / 2, IWc = (a.IW - pw + 1) / 2;
    const int64_t CHW = (int64_t)IHc * IWc;
#pragma unroll
    for (int ni = 0; ni < WN; ++ni) {
        if (!valid[ni]) continue;
        const int64_t cl = col[ni];
        int64_t obase, ostride;
        float* dst = a.out;
        if (MODE == 0) {
            const int64_t b = bs >= 0 ? bs : cl / OHW;
            obase = b * a.cout * OHW + (bs >= 0 ? cl : cl - b * OHW);
            ostride = OHW;
        } else if (MODE == 1) {
            const int64_t b = bs >= 0 ? bs : cl / IHW;
            obase = b * a.cin * IHW + (bs >= 0 ? cl : cl - b * IHW);
            ostride = IHW;
        } else {
            const int64_t b = cl / CHW, p = cl - b * CHW;
            if (a.par_out) {  // dense class planes (contiguous 128-byte rows)
                dst = a.par_out;
                obase = b * a.cin * CHW + p;
                ostride = CHW;
            } else {
                const int ihc = (int)(p / IWc), iwc = (int)(p - (int64_t)(p / IWc) * IWc);
                obase = b * a.cin * IHW + (int64_t)(2 * ihc + ph) * a.IW + 2 * iwc + pw;
                ostride = IHW;
            }
        }
#pragma unroll
        for (int mi = 0; mi < WM; ++mi)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int64_t row = m0 + wr * 32 * WM + mi * 32 + acc_row(r, h);
                if (row < M) {
                    float* o = dst + obase + row * ostride;
                    if (MODE != 0 && a.accumulate) *o += acc[mi][ni][r];
                    else *o = acc[mi][ni][r];
                }
            }
    }
    if constexpr (MODE == 1 && EP) {
        // backward partials of the BN + ReLU (+ Dropout2d) that produced this conv's input (replaces
        // the bwd_prep pass over dx): producer values loaded for all of a row block first, per-row
        // sums over the lanes by the transposed butterfly, the two pixel halves added
        __syncthreads();  // operand stages consumed
        float* red = reinterpret_cast<float*>(smem);                   // [NWC (wc)][BM][2]
        float4* cfl = reinterpret_cast<float4*>(red + 2 * NWC * BM);  // [BM]
        if (tid < BM) cfl[tid] = a.ep_cf[min(m0 + tid, M - 1)];
        __syncthreads();
        const int64_t IHWe = (int64_t)a.IH * a.IW;
        int64_t yb[WN], db[WN];
#pragma unroll
        for (int ni = 0; ni < WN; ++ni) {
            const int64_t cc = col[ni], b = bs >= 0 ? bs : cc / IHWe;
            yb[ni] = b * a.cin * IHWe + (bs >= 0 ? cc : cc - b * IHWe);
            db[ni] = b * a.cin;
        }
#pragma unroll
        for (int mi = 0; mi < WM; ++mi) {
            // one pixel column block at a time (16 y and 16 dropout values live, not 2 x 32), summed in
            // the same order as before (ni ascending)
            float sg[16], sx[16];
#pragma unroll
            for (int r = 0; r < 16; ++r) sg[r] = sx[r] = 0.f;
#pragma unroll
            for (int ni = 0; ni < WN; ++ni) {
                float yv[16], dv[16];
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int64_t rc = min(m0 + wr * 32 * WM + mi * 32 + acc_row(r, h), M - 1);
                    yv[r] = a.ep_y[yb[ni] + rc * IHWe];
                    dv[r] = a.ep_drop ? a.ep_drop[db[ni] + rc] : 1.f;
                }
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int rl = wr * 32 * WM + mi * 32 + acc_row(r, h);
                    const float4 k = cfl[rl];
                    const bool rok = m0 + rl < M;
                    const float y = yv[r];
                    const float g = (valid[ni] && rok && fmaf(y, k.x, k.y) > 0.f) ? acc[mi][ni][r] * dv[r] : 0.f;
                    sg[r] += g;
                    sx[r] = fmaf(g, (y - k.z) * k.w, sx[r]);
                }
            }
            const float tg = xsum16(sg, l32), tx = xsum16(sx, l32);
            if (!(l32 & 1)) {
                float* d = red + (wc * BM + wr * 32 * WM + mi * 32 + acc_row(l32 >> 1, h)) * 2;
                d[0] = tg;
                d[1] = tx;
            }
        }
        __syncthreads();
        if (tid < BM && m0 + tid < M) {
            float pg = 0.f, px = 0.f;
#pragma unroll
            for (int w = 0; w < NWC; ++w) {
                pg += red[(w * BM + tid) * 2];
                px += red[(w * BM + tid) * 2 + 1];
            }
            a.ep_pg[(m0 + tid) * ntile + tn] = pg;
            a.ep_px[(m0 + tid) * ntile + tn] = px;
        }
    }
    if (MODE == 0 && a.st_part0 != nullptr) {
        // BN forward partials of the tile (replaces the statistics pass over out): per (wave, channel)
        // Chan statistics of its valid pixels about the channel's first pixel in the wave (K, v_readlane),
        // reduced over the lanes with the transposed butterfly, then the two pixel halves merged
        __syncthreads();  // every wave is done with the operand stages: the LDS holds the exchange
        float* red = reinterpret_cast<float*>(smem);
#pragma unroll
        for (int mi = 0; mi < WM; ++mi) {
            float kv[16], s1[16], s2[16];
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const float k0 = readlane_f(acc[mi][0][r], 0), k1 = readlane_f(acc[mi][0][r], 32);
                kv[r] = h ? k1 : k0;
                s1[r] = 0.f;
                s2[r] = 0.f;
#pragma unroll
                for (int ni = 0; ni < WN; ++ni)
                    if (valid[ni]) {
                        const float d = acc[mi][ni][r] - kv[r];
                        s1[r] += d;
                        s2[r] = fmaf(d, d, s2[r]);
                    }
            }
            const float t1 = xsum16(s1, l32), t2 = xsum16(s2, l32), K = xsel16(kv, l32);
            if (!(l32 & 1)) {
                const float n = (float)cnt_w;
                float* d = red + (wc * BM + wr * 32 * WM + mi * 32 + acc_row(l32 >> 1, h)) * 3;
                d[0] = n;
                d[1] = cnt_w ? K + t1 / n : 0.f;
                d[2] = cnt_w ? fmaxf(t2 - t1 * t1 / n, 0.f) : 0.f;
            }
        }
        __syncthreads();
        if (tid < BM && m0 + tid < M) {
            float n = 0.f, mean = 0.f, m2 = 0.f;
#pragma unroll
            for (int w = 0; w < NWC; ++w) {
                const float* d = red + (w * BM + tid) * 3;
                if (d[0] > 0.f) {
                    const float nt = n + d[0], delta = d[1] - mean;
                    mean += delta * d[0] / nt;
                    m2 += d[2] + delta * delta * n * d[0] / nt;
                    n = nt;
                }
            }
            a.st_part0[(m0 + tid) * ntile + tn] = n * mean;
            a.st_part1[(m0 + tid) * ntile + tn] = m2;
            if (tid == 0 && tm == 0) a.st_partn[tn] = n;
        }
    }
}

// EP (mode 1 only): the producer BN's backward sums in the epilogue (a separate instantiation: its
// registers held every data-gradient launch at 1-2 waves per SIMD)
template <int MODE, int WM, int KC, bool EP = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void convn_kernel(ConvGArgs a) {
    constexpr int WN = 2;
    constexpr int BM = 64 * WM, BN = 64 * WN;
    constexpr int RB = 2 * KC, RPI = 1024 / RB, SPR = RB / 16;  // row bytes, rows per DMA instruction, runs per row
    constexpr int ABYTES = BM * RB, STAGE = (BM + BN) * RB;
    constexpr int NA = BM / RPI / 4, NB = BN / RPI / 4;  // DMA instructions per wave and chunk
    __shared__ __attribute__((aligned(1024))) char smem[2 * STAGE];
    const unsigned lds0 = (unsigned)(uintptr_t)(lds_void*)smem;

    const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, l32 = lane & 31;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), wr = wave >> 1, wc = wave & 1;
    const int s = a.stride, pad = a.pad;
    const int ph = a.par >> 1, pw = a.par & 1;
    const int kh0 = (ph + pad) & 1, kw0 = (pw + pad) & 1;
    const int64_t OHW = (int64_t)a.OH * a.OW, IHW = (int64_t)a.IH * a.IW;
    const int IHc = (a.IH - ph + 1) / 2, IWc = (a.IW - pw + 1) / 2;
    const int64_t CHW = (int64_t)IHc * IWc;
    int CK, Hp, Wp, nth, ntw;
    int64_t M, N;
    if (MODE == 0) {
        CK = a.cin; Hp = a.IH + 2; Wp = a.IW + 2; M = a.cout; N = a.B * OHW; nth = a.KH; ntw = a.KW;
    } else {
        CK = a.cout; Hp = a.OH + 2; Wp = a.OW + 2; M = a.cin;
        if (MODE == 1) { N = a.B * IHW; nth = a.KH; ntw = a.KW; }
        else { N = a.B * CHW; nth = (a.KH - kh0 + 1) / 2; ntw = (a.KW - kw0 + 1) / 2; }
    }
    const int T = nth * ntw, nch = T * (CK / KC);
    const int64_t K = (int64_t)T * CK;  // packed row length (a multiple of 32)
    const int64_t mt = (M + BM - 1) / BM;
    const int64_t lid = xcd_logical(mt * ((N + BN - 1) / BN));
    if (lid >= mt * ((N + BN - 1) / BN)) return;  // (grid padded to a multiple of 8)
    const int64_t tm = lid % mt, tn = lid / mt;
    const int64_t m0 = tm * BM, n0 = tn * BN;

    // DMA roles: wave instruction j covers tile rows RPI (wave + 4 j) ..; lane -> row lr, slot ls
    const int lr = lane / SPR, ls = lane % SPR;
    auto slot_run = [&](int r) { return KC == 32 ? ls ^ ((r >> 2) & 3) : ls ^ ((r >> 1) & 7); };
    const __bf16* asrc[NA];
#pragma unroll
    for (int j = 0; j < NA; ++j) {
        const int r = RPI * (wave + 4 * j) + lr;
        const int64_t row = m0 + r;  // rows past M copy row 0: finite, never stored
        asrc[j] = static_cast<const __bf16*>(a.wpack) + (row < M ? row : 0) * K + 8 * slot_run(r);
    }
    const __bf16* bsrc[NB];
#pragma unroll
    for (int j = 0; j < NB; ++j) {
        const int r = RPI * (wave + 4 * j) + lr;
        int64_t nn = n0 + r;
        if (nn >= N) nn = N - 1;  // tail pixels copy a valid row; their columns are never stored
        int64_t pb;               // image element of the pixel's operand row at tap 0
        if (MODE == 0) {
            const int64_t b = nn / OHW;
            const int rr = (int)(nn - b * OHW), oh = rr / a.OW, ow = rr - oh * a.OW;
            pb = ((b * Hp + oh * s - pad + 1) * Wp + ow * s - pad + 1) * CK;
        } else if (MODE == 1) {
            const int64_t b = nn / IHW;
            const int rr = (int)(nn - b * IHW), ih = rr / a.IW, iw = rr - ih * a.IW;
            pb = ((b * Hp + ih + pad + 1) * Wp + iw + pad + 1) * CK;
        } else {
            const int64_t b = nn / CHW;
            const int rr = (int)(nn - b * CHW), ihc = rr / IWc, iwc = rr - ihc * IWc;
            const int oh0 = (2 * ihc + ph + pad - kh0) >> 1, ow0 = (2 * iwc + pw + pad - kw0) >> 1;
            pb = ((b * Hp + oh0 + 1) * Wp + ow0 + 1) * CK;
        }
        bsrc[j] = static_cast<const __bf16*>(MODE == 0 ? a.xn : a.dyn) + pb + 8 * slot_run(r);
    }
    // K walks channel-major (32 channels x every tap, then the next 32): the taps of a channel
    // group re-read one halo of the image back to back, out of L2
    auto issue = [&](int ch, int stage) {
        const int cc = ch / T, tap = ch - cc * T, c0 = cc * KC;
        const int th = tap / ntw, tw = tap - th * ntw;
        const int toff = (MODE == 0 ? 1 : -1) * (th * Wp + tw) * CK + c0;
        const unsigned base = lds0 + (unsigned)(stage * STAGE);
#pragma unroll
        for (int j = 0; j < NA; ++j) dma16(asrc[j] + (int64_t)ch * KC, base + (unsigned)(RPI * (wave + 4 * j) * RB));
#pragma unroll
        for (int j = 0; j < NB; ++j) dma16(bsrc[j] + toff, base + (unsigned)(ABYTES + RPI * (wave + 4 * j) * RB));
    };

    f32x16 acc[WM][WN];
#pragma unroll
    for (int mi = 0; mi < WM; ++mi)
#pragma unroll
        for (int ni = 0; ni < WN; ++ni) acc[mi][ni] = f32x16{0.f};

    if (nch > 0) issue(0, 0);
    for (int ch = 0; ch < nch; ++ch) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();  // chunk ch in LDS for every wave; the other stage's readers are done
        if (ch + 1 < nch) issue(ch + 1, (ch + 1) & 1);
        const char* st = smem + (ch & 1) * STAGE;
#pragma unroll
        for (int ks = 0; ks < KC / 16; ++ks) {
            bf16x8 av8[WM], bv8[WN];
#pragma unroll
            for (int mi = 0; mi < WM; ++mi)
                av8[mi] = *reinterpret_cast<const bf16x8*>(st + swz<KC>(wr * 32 * WM + mi * 32 + l32, 2 * ks + h));
#pragma unroll
            for (int ni = 0; ni < WN; ++ni)
                bv8[ni] = *reinterpret_cast<const bf16x8*>(st + ABYTES + swz<KC>(wc * 32 * WN + ni * 32 + l32, 2 * ks + h));
#pragma unroll
            for (int mi = 0; mi < WM; ++mi)
#pragma unroll
                for (int ni = 0; ni < WN; ++ni) acc[mi][ni] = mfma_bf16(av8[mi], bv8[ni], acc[mi][ni]);
        }
    }

    // ---- epilogue (shared with the halo-staged kernel)
    int64_t col[WN];
    bool valid[WN];
#pragma unroll
    for (int ni = 0; ni < WN; ++ni) {
        const int64_t c = n0 + wc * 32 * WN + ni * 32 + l32;
        valid[ni] = c < N;
        col[ni] = valid[ni] ? c : N - 1;
    }
    const int64_t nw0 = n0 + wc * 32 * WN;
    const int cnt_w = (int)max((int64_t)0, min((int64_t)(32 * WN), N - nw0));
    convn_epilogue<MODE, WM, WN, EP>(a, acc, smem, m0, M, col, valid, cnt_w, (N + BN - 1) / BN, tn, tm);
}

// ------------------------------------------------------------------ halo-staged forward / data gradient
// (round 5) Stride 1, 3x3, pad 1, modes 0 and 1.  The per-tap kernel above copies every pixel's 64-byte
// operand run once per tap (nine times per channel chunk) and is bound by that L2 -> LDS stream on the
// 64-channel layers.  Here a tile is TR x TW output pixels of one sample (N columns n = r TW + c, up to
// 128), and per 32-channel chunk the (TR + 2) x (TW + 2) pixels of the padded image it touches are copied
// once (the halo); the nine taps read their B operand at shifted halo positions.  The weights come per
// tap row (three BM x 32 tiles); the next row's weights and, spread over the rows, the next chunk's halo
// are copied under the current row's MFMAs (both double-buffered, one barrier per tap row).
struct HaloGeo {
    int TR, TW;     // tile rows / columns
    int nsr, nsc;   // tiles per sample along rows / columns
    int hp;         // halo pixels (TR + 2) (TW + 2) rounded up to 16 (one DMA instruction = 16 pixels)
};

template <int MODE, int WM, bool EP, int NW = 4>
__global__ __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(2))) void convn_halo_kernel(ConvGArgs a, HaloGeo g) {
    // NW waves: two wave rows (32 WM output rows each) x NW / 2 wave columns (64 pixels each)
    constexpr int WN = 2, KC = 32, RB = 64, NWC = NW / 2;
    constexpr int BM = 64 * WM;
    constexpr int ABYTES = BM * RB;
    extern __shared__ __attribute__((aligned(1024))) char smem[];  // [2][3 A tiles] [2][halo]
    const unsigned lds0 = (unsigned)(uintptr_t)(lds_void*)smem;
    const int HB = g.hp * RB;  // halo stage bytes
    const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, l32 = lane & 31;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), wr = wave / NWC, wc = wave % NWC;
    // image of the B operand: mode 0 the input x, mode 1 dy (both padded, channel count CK)
    int CK, H, W, Hp, Wp;
    int64_t M;
    if (MODE == 0) { CK = a.cin; H = a.OH; W = a.OW; M = a.cout; }
    else { CK = a.cout; H = a.IH; W = a.IW; M = a.cin; }
    Hp = H + 2; Wp = W + 2;
    // (32-bit tile decode, host-checked mt * ntile < 2^31: the int64 divisions were ~100 scalar instructions each)
    const int tps = g.nsr * g.nsc;
    const int mt = (int)((M + BM - 1) / BM), ntile = a.B * tps;
    const unsigned nb = (unsigned)(mt * ntile), bid = blockIdx.x;
    const unsigned lid = (bid & 7) * ((nb + 7) >> 3) + (bid >> 3);  // xcd_logical in 32 bits
    if (lid >= nb) return;  // (grid padded to a multiple of 8)
    const int tm = (int)(lid % (unsigned)mt), tn = (int)(lid / (unsigned)mt);
    const int64_t m0 = (int64_t)tm * BM;
    const int b = tn / tps, tl = tn - b * tps;
    const int sr = tl / g.nsc, sc = tl - sr * g.nsc;
    const int oh0 = sr * g.TR, ow0 = sc * g.TW;
    const int HW2 = g.TW + 2;

    // A rows (weights, as the per-tap kernel: logical run q of row r in slot q ^ ((r >> 2) & 3))
    constexpr int RPI = 1024 / RB, NAI = BM / RPI, NA = (NAI + NW - 1) / NW;  // A copy instructions: tile, wave
    const int lr = lane >> 2, ls = lane & 3;
    const __bf16* asrc[NA];
#pragma unroll
    for (int j = 0; j < NA; ++j) {
        const int r = RPI * (wave + NW * j) + lr;
        const int64_t row = m0 + r;
        asrc[j] = static_cast<const __bf16*>(a.wpack) + (row < M && r < BM ? row : 0) * (int64_t)(9 * CK) + 8 * (ls ^ ((r >> 2) & 3));
    }
    // halo copies: instruction j (of g.hp / 16) covers halo pixels 16 j .. 16 j + 15, lane -> pixel
    // 16 j + (lane >> 2), slot (lane & 3) holding run (lane & 3) ^ swz(pixel); wave w issues j = w, w + 4, ..
    const int nhi = g.hp / 16;
    const int nhw = (nhi - wave + NW - 1) / NW;  // this wave's halo instructions per chunk (<= 7)
    const __bf16* img = static_cast<const __bf16*>(MODE == 0 ? a.xn : a.dyn) + (int64_t)b * Hp * Wp * CK;
    unsigned hoff[7];
#pragma unroll
    for (int k = 0; k < 7; ++k) {
        const int j = wave + NW * k;
        int px = 16 * j + (lane >> 2);
        if (px >= (g.TR + 2) * HW2) px = 0;  // the stage's round-up slack: any readable run
        const int i = px / HW2, jj = px - i * HW2;
        const int hr = min(oh0 + i, Hp - 1), hc = min(ow0 + jj, Wp - 1);  // (clamped: feeds masked outputs only)
        const int q = (lane & 3) ^ ((px >> 2) & 3);
        hoff[k] = 2u * (unsigned)((hr * Wp + hc) * CK + 8 * q);
    }
    // A of one tap row (taps 3 th .. 3 th + 2 of chunk cc = iteration it = 3 cc + th): three BM x 32 tiles
    auto issue_a = [&](int it, int stage) {
#pragma unroll
        for (int tw = 0; tw < 3; ++tw) {
            const unsigned base = lds0 + (unsigned)((3 * stage + tw) * ABYTES);
#pragma unroll
            for (int j = 0; j < NA; ++j)
                if (NAI % NW == 0 || wave + NW * j < NAI)
                    dma16(asrc[j] + (int64_t)(3 * it + tw) * KC, base + (unsigned)(RPI * (wave + NW * j) * RB));
        }
    };
    auto issue_h = [&](int cc, int k, int stage) {  // this wave's k-th halo instruction of chunk cc
        const __bf16* sb = img + cc * KC;
        const unsigned m0l = lds0 + (unsigned)(6 * ABYTES + stage * HB + (wave + NW * k) * 1024);
        const unsigned m0u = __builtin_amdgcn_readfirstlane(m0l);
        const uint64_t v = (uint64_t)(uintptr_t)sb;
        const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)v), hi = __builtin_amdgcn_readfirstlane((unsigned)(v >> 32));
        const __bf16* su = (const __bf16*)(uintptr_t)(((uint64_t)hi << 32) | lo);
        asm volatile("s_nop 0\n\tglobal_load_lds_dwordx4 %0, %1" :: "v"(hoff[k]), "s"(su), "{m0}"(m0u) : "memory");
    };
    // the lane's columns: tile pixel n = wc 64 + ni 32 + l32 -> (r, c); halo pixel of tap (th, tw):
    // mode 0 (r + th) HW2 + c + tw, mode 1 (r + 2 - th) HW2 + c + 2 - tw
    int hpb[WN];
    bool valid[WN];
    int64_t col[WN];
    int cnt_w = 0;
#pragma unroll
    for (int ni = 0; ni < WN; ++ni) {
        const int n = wc * 32 * WN + ni * 32 + l32;
        const int r = n / g.TW, c = n - r * g.TW;
        valid[ni] = n < g.TR * g.TW && oh0 + r < H && ow0 + c < W;
        const int rr = valid[ni] ? r : 0, cq = valid[ni] ? c : 0;
        hpb[ni] = MODE == 0 ? rr * HW2 + cq : (rr + 2) * HW2 + cq + 2;
        col[ni] = (int64_t)(oh0 + rr) * W + ow0 + cq;  // (pixel inside sample b: the epilogue's bs)
        cnt_w += __popcll(__ballot(valid[ni]) & 0xffffffffull);
    }

    f32x16 acc[WM][WN];
#pragma unroll
    for (int mi = 0; mi < WM; ++mi)
#pragma unroll
        for (int ni = 0; ni < WN; ++ni) acc[mi][ni] = f32x16{0.f};

    // one barrier per tap row (3 taps, 12 WM MFMAs per wave); the next chunk's halo instructions are
    // spread over the rows (<= 3 of the wave's per row), issued after the next A
    const int ncc = CK / KC, nit = 3 * ncc;
    issue_a(0, 0);
#pragma unroll
    for (int k = 0; k < 7; ++k)
        if (k < nhw) issue_h(0, k, 0);
    int th = 0, cc = 0;
    for (int it = 0; it < nit; ++it) {
        // A(it) must have landed; the halo instructions issued after it in the previous row may fly
        const int hprev = (th >= 1 && cc + 1 < ncc) ? min(3, max(0, nhw - 3 * (th - 1))) : 0;
        if (hprev >= 3) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
        else if (hprev == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
        else if (hprev == 1) asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();  // A(it) (and at th 0 the chunk's halo) in LDS for every wave; the other A stage free
        if (it + 1 < nit) issue_a(it + 1, (it + 1) & 1);
        if (cc + 1 < ncc)
#pragma unroll
            for (int k = 0; k < 3; ++k)
                if (3 * th + k < nhw) issue_h(cc + 1, 3 * th + k, (cc + 1) & 1);
        const char* hs = smem + 6 * ABYTES + (cc & 1) * HB;
#pragma unroll
        for (int tw = 0; tw < 3; ++tw) {
            const char* as = smem + (3 * (it & 1) + tw) * ABYTES;
            const int toff = MODE == 0 ? th * HW2 + tw : -(th * HW2 + tw);
#pragma unroll
            for (int ks = 0; ks < KC / 16; ++ks) {
                bf16x8 av8[WM], bv8[WN];
#pragma unroll
                for (int mi = 0; mi < WM; ++mi)
                    av8[mi] = *reinterpret_cast<const bf16x8*>(as + swz<KC>(wr * 32 * WM + mi * 32 + l32, 2 * ks + h));
#pragma unroll
                for (int ni = 0; ni < WN; ++ni) {
                    const int px = hpb[ni] + toff;
                    bv8[ni] = *reinterpret_cast<const bf16x8*>(hs + px * RB + 16 * ((2 * ks + h) ^ ((px >> 2) & 3)));
                }
#pragma unroll
                for (int mi = 0; mi < WM; ++mi)
#pragma unroll
                    for (int ni = 0; ni < WN; ++ni) acc[mi][ni] = mfma_bf16(av8[mi], bv8[ni], acc[mi][ni]);
            }
        }
        if (++th == 3) { th = 0; ++cc; }
    }
    convn_epilogue<MODE, WM, WN, EP, NWC>(a, acc, smem, m0, M, col, valid, cnt_w, ntile, tn, tm, b);
}

// ------------------------------------------------------------------ weight gradient
// Tiles are staged pixel-major, As[k][cout], Bs[k][(tap, cin)], and the MFMA operands (8
// consecutive k of one row) are read with ds_read_b64_tr_b16: per 16-lane group, 4 k-rows x 16
// columns delivered column-major.  Row strides of 48 / 80 dwords (= 16 mod 64) put the four k-rows
// of a read on disjoint bank quarters: conflict-free.
template <int WM>
__global__ __launch_bounds__(256) void convn_wgrad_kernel(ConvGArgs a) {
    constexpr int WN = 2;
    constexpr int BM = 64 * WM, BN = 64 * WN;
    constexpr int AS = BM + 32, BS = BN + 32;
    __shared__ __attribute__((aligned(16))) __bf16 As[2][NKB][AS];
    __shared__ __attribute__((aligned(16))) __bf16 Bs[2][NKB][BS];

    const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, l32 = lane & 31;
    const int wave = tid >> 6, wr = wave >> 1, wc = wave & 1;
    const int s = a.stride, pad = a.pad;
    const int KK = a.KH * a.KW;
    const int64_t OHW = (int64_t)a.OH * a.OW;
    const int64_t M = a.cout, N = (int64_t)a.cin * KK, K = a.B * OHW;
    const int Hp = a.IH + 2, Wp = a.IW + 2, Hq = a.OH + 2, Wq = a.OW + 2;
    const int64_t mt = (M + BM - 1) / BM, nt = (N + BN - 1) / BN;
    int64_t bid = xcd_logical(mt * nt * a.nslice);
    if (bid >= mt * nt * a.nslice) return;  // (grid padded to a multiple of 8)
    const int64_t tm = bid % mt;
    bid /= mt;
    const int64_t tn = bid % nt;
    const int slice = (int)(bid / nt);
    const int64_t m0 = tm * BM, n0 = tn * BN;
    const int64_t k_begin = (int64_t)slice * a.kslice, k_end = min(K, k_begin + a.kslice);
    const int nch = (int)((k_end - k_begin + NKB - 1) / NKB);

    // staging: pixel rows kk = (tid >> 4) + 16 r, 16-byte column group g = tid & 15
    const int kk0 = tid >> 4, g = tid & 15;
    // B: columns n0 + 8 g .. + 7 = one tap, 8 input channels
    const int64_t nb = n0 + 8 * g;
    const bool bval = nb < N;
    int xtoff;  // (tap-major columns: n = tap * cin + ci)
    {
        const int tap = bval ? (int)(nb / a.cin) : 0, ci = bval ? (int)(nb - (int64_t)tap * a.cin) : 0;
        const int kh = tap / a.KW, kw = tap - kh * a.KW;
        xtoff = (kh * Wp + kw) * a.cin + ci;
    }
    // A: BM = 128: output channels m0 + 8 g of both rows; BM = 64: row r = g >> 3, channels m0 + 8 (g & 7)
    constexpr int NA = WM == 2 ? 2 : 1;
    const int ag = WM == 2 ? g : (g & 7);
    const int arr = WM == 2 ? 0 : (g >> 3);
    const bool aval = m0 + 8 * ag < M;
    const int dytoff = (int)(m0 + 8 * ag);

    const __bf16* xn = static_cast<const __bf16*>(a.xn);
    const __bf16* dyn = static_cast<const __bf16*>(a.dyn);
    struct PixPos { int64_t b; int oh, ow; };
    PixPos pp[2];
#pragma unroll
    for (int r = 0; r < 2; ++r) {
        const int64_t q = k_begin + kk0 + 16 * r;
        pp[r].b = q / OHW;
        const int rr = (int)(q - pp[r].b * OHW);
        pp[r].oh = rr / a.OW;
        pp[r].ow = rr - pp[r].oh * a.OW;
    }
    auto advance = [&](PixPos& p) {  // + 32 pixels
        p.ow += NKB;
        while (p.ow >= a.OW) {
            p.ow -= a.OW;
            if (++p.oh == a.OH) { p.oh = 0; ++p.b; }
        }
    };

    bf16x8 rx[2], rd[NA];
    auto gather = [&](int ch) {
        const int64_t kb = k_begin + (int64_t)ch * NKB + kk0;
#pragma unroll
        for (int r = 0; r < 2; ++r) {
            const bool v = kb + 16 * r < k_end;
            const PixPos& p = pp[r];
            const int64_t xo = ((p.b * Hp + p.oh * s - pad + 1) * Wp + p.ow * s - pad + 1) * a.cin + xtoff;
            rx[r] = (v && bval) ? ld16(xn + xo) : bf16x8{};
        }
        int64_t yo[2];
#pragma unroll
        for (int r = 0; r < 2; ++r) yo[r] = ((pp[r].b * Hq + pp[r].oh + 1) * Wq + pp[r].ow + 1) * a.cout + dytoff;
#pragma unroll
        for (int r = 0; r < NA; ++r) {
            const bool sel = WM == 2 ? r != 0 : arr != 0;  // (a select, not a dynamic index)
            const bool v = kb + (sel ? 16 : 0) < k_end;
            rd[r] = (v && aval) ? ld16(dyn + (sel ? yo[1] : yo[0])) : bf16x8{};
        }
        advance(pp[0]);
        advance(pp[1]);
    };
    auto stash = [&](int buf) {
#pragma unroll
        for (int r = 0; r < 2; ++r) *reinterpret_cast<bf16x8*>(&Bs[buf][kk0 + 16 * r][8 * g]) = rx[r];
#pragma unroll
        for (int r = 0; r < NA; ++r) {
            const int rr = WM == 2 ? r : arr;
            *reinterpret_cast<bf16x8*>(&As[buf][kk0 + 16 * rr][8 * ag]) = rd[r];
        }
    };

    // transposed-read lane roles: group grp = lane >> 4 -> k-block hh, column half cc; within the
    // group lane 4q + p addresses k-row q, columns 4p .. 4p + 3
    const int grp = lane >> 4, hh = grp >> 1, cc = grp & 1, q4 = (lane & 15) >> 2, p4 = lane & 3;
    auto tr_operand = [&](const __bf16* tile, int stride, int col, int krow) {
        typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
        const __bf16* p0 = tile + (krow + q4) * stride + col + 4 * p4;
        const __bf16* p1 = p0 + 4 * stride;
        const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p0));
        const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p1));
        const s16x8 v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
        return __builtin_bit_cast(bf16x8, v);
    };

    f32x16 acc[WM][WN];
#pragma unroll
    for (int mi = 0; mi < WM; ++mi)
#pragma unroll
        for (int ni = 0; ni < WN; ++ni) acc[mi][ni] = f32x16{0.f};

    if (nch > 0) {
        gather(0);
        stash(0);
        if (nch > 1) gather(1);
    }
    __syncthreads();
    for (int ch = 0; ch < nch; ++ch) {  // (stash at the top, as convn_kernel)
        const int buf = ch & 1;
        if (ch + 1 < nch) stash(buf ^ 1);
        if (ch + 2 < nch) gather(ch + 2);
#pragma unroll
        for (int ks = 0; ks < NKB / 16; ++ks) {
            bf16x8 av8[WM], bv8[WN];
#pragma unroll
            for (int mi = 0; mi < WM; ++mi)
                av8[mi] = tr_operand(&As[buf][0][0], AS, wr * 32 * WM + mi * 32 + 16 * cc, 16 * ks + 8 * hh);
#pragma unroll
            for (int ni = 0; ni < WN; ++ni)
                bv8[ni] = tr_operand(&Bs[buf][0][0], BS, wc * 32 * WN + ni * 32 + 16 * cc, 16 * ks + 8 * hh);
#pragma unroll
            for (int mi = 0; mi < WM; ++mi)
#pragma unroll
                for (int ni = 0; ni < WN; ++ni) acc[mi][ni] = mfma_bf16(av8[mi], bv8[ni], acc[mi][ni]);
        }
        __syncthreads();
    }

    // ---- epilogue: slice partial in the reference layout [cout][cin][KH][KW]
#pragma unroll
    for (int ni = 0; ni < WN; ++ni) {
        const int64_t col = n0 + wc * 32 * WN + ni * 32 + l32;
        if (col >= N) continue;
        const int tap = (int)(col / a.cin), c = (int)(col - (int64_t)tap * a.cin);
        const int64_t obase = (int64_t)slice * M * N + (int64_t)c * KK + tap;
#pragma unroll
        for (int mi = 0; mi < WM; ++mi)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int64_t row = m0 + wr * 32 * WM + mi * 32 + acc_row(r, h);
                if (row < M) a.out[obase + row * N] = acc[mi][ni][r];
            }
    }
}

// weight rows of the forward / data-gradient kernel: row m, k = (c / KC) (T KC) + t KC + c % KC over
// the T (class) taps t = th ntw + tw, kernel tap (kh0 + step th, kw0 + step tw), step 2 for mode 3
__global__ __launch_bounds__(256) void convn_pack_kernel(const float* __restrict__ w, __bf16* __restrict__ wp, int mode,
                                                         int cin, int cout, int KH, int KW, int kh0, int kw0, int step,
                                                         int ntw, int T, int KC, int64_t M, int64_t K) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= M * K) return;
    const int64_t m = i / K;
    const int k = (int)(i - m * K);
    const int cc = k / (T * KC), rem = k - cc * T * KC, t = rem / KC, c = cc * KC + rem - t * KC;
    const int kh = kh0 + step * (t / ntw), kw = kw0 + step * (t % ntw);
    const float v = mode == 0 ? w[((m * cin + c) * KH + kh) * KW + kw]            // [cout = m][cin = c]
                              : w[(((int64_t)c * cin + m) * KH + kh) * KW + kw];  // [cout = c][cin = m]
    wp[i] = (__bf16)v;
}

}  // namespace

size_t nhwc_bytes(int B, int C, int H, int W) { return (size_t)B * (H + 2) * (W + 2) * C * 2; }

int launch_to_nhwc(NhwcArgs a, hipStream_t s) {
    PCX_CHECK_ARG(a.C % 8 == 0 && a.B > 0 && a.H > 0 && a.W > 0, "to_nhwc: C %d must be a multiple of 8", a.C);
    PCX_CHECK_ARG(a.op == NHWC_COPY || a.op == NHWC_BNBWD || a.op == NHWC_ACT, "to_nhwc: op %d", a.op);
    PCX_CHECK_ARG(a.op != NHWC_BNBWD || (a.y && a.cf), "to_nhwc: BN backward needs y and cf");
    PCX_CHECK_ARG(a.op != NHWC_ACT || a.cf, "to_nhwc: activation needs cf");
    PCX_CHECK_ARG(!a.res_pool || (a.op == NHWC_ACT && a.res && a.rcf), "to_nhwc: pooled residual needs res and rcf");
    PCX_CHECK_ARG(!a.dst_b || (a.op == NHWC_BNBWD && a.y_b && a.cf_b), "to_nhwc: second image needs y_b and cf_b");
    // image rows per step: up to 128 floats of a channel (narrow images: fewer, fuller steps); one row
    // with the pooled residual (staged per row)
    constexpr bool one_row = PCX_AB_NHWC_ROWS1;  // A/B: a row per step
    a.rows = a.res_pool || one_row ? 1 : std::max(1, std::min(a.H, (a.dst_b ? 124 : 128) / a.W));
    const size_t sm = ((size_t)64 * ((a.rows * a.W + 3) & ~3) + 32) * 4 * (a.dst_b || a.res_pool ? 2 : 1);
    PCX_CHECK_ARG(!a.res_pool || a.C % 4 == 0, "to_nhwc: pooled residual needs C %% 4 == 0");
    PCX_CHECK_ARG(sm <= 64 * 1024, "to_nhwc: row of %d pixels too long", a.W);
    dim3 grid((unsigned)a.B, (unsigned)ceil_div(a.C, 64));
    const int v = a.W % 4 == 0 ? 4 : a.W % 2 == 0 ? 2 : 1;
#define PCX_TN(V_, OP_) \
    if (v == V_ && a.op == OP_) to_nhwc_kernel<V_, OP_><<<grid, 256, sm, s>>>(a);
    PCX_TN(4, NHWC_COPY) PCX_TN(2, NHWC_COPY) PCX_TN(1, NHWC_COPY)
    PCX_TN(4, NHWC_BNBWD) PCX_TN(2, NHWC_BNBWD) PCX_TN(1, NHWC_BNBWD)
    PCX_TN(4, NHWC_ACT) PCX_TN(2, NHWC_ACT) PCX_TN(1, NHWC_ACT)
#undef PCX_TN
    PCX_LAUNCH_CHECK("to_nhwc_kernel");
    return PCX_OK;
}

// K per chunk of the forward / data-gradient kernel: 64 channels (128-byte rows: whole-line requests,
// 14 % faster than 32 on the 256-channel layers) where the channel count allows
static int convn_kc(int ck) { return ck % 64 == 0 ? 64 : 32; }

// halo-staged tiling of an H x W image (stride-1 3x3 pad-1 modes 0 / 1): the fewest TR x TW tiles of at
// most maxpx pixels (ties: the smaller halo); used only when the tiles keep >= 90 % of their MFMA columns
// busy (T = 200, 128 pixels: 20 x 100 -> 16 tiles of 5 x 25, 10 x 50 -> 4, 5 x 25 -> 1; 256 pixels:
// 20 x 100 -> 8 of 10 x 25).  PCX_AB_NO_CONVN_HALO: per-tap copies everywhere.
static bool convn_halo_tiles(int H, int W, int maxpx, HaloGeo* out) {
    constexpr bool off = PCX_AB_NO_CONVN_HALO;
    if (off || H < 1 || W < 1) return false;
    HaloGeo best{};
    int64_t bt = -1, bh = 0;
    for (int nsc = 1; nsc <= W; ++nsc) {
        const int TW = (W + nsc - 1) / nsc;
        if (TW > maxpx) continue;
        if (nsc > 1 && (W + nsc - 2) / (nsc - 1) == TW) continue;  // same width as nsc - 1
        const int TR0 = std::min(H, maxpx / TW);
        const int nsr = (H + TR0 - 1) / TR0, TR = (H + nsr - 1) / nsr;
        const int64_t tiles = (int64_t)nsr * nsc, halo = (int64_t)(TR + 2) * (TW + 2);
        if (bt < 0 || tiles < bt || (tiles == bt && halo < bh)) {
            bt = tiles; bh = halo;
            best.TR = TR; best.TW = TW; best.nsr = nsr; best.nsc = nsc;
            best.hp = (int)((halo + 15) / 16 * 16);
        }
        if (TW < 8) break;
    }
    if (bt < 0 || (double)H * W < 0.9 * (double)bt * maxpx || best.hp > 7 * 16 * (maxpx / 32)) return false;
    if (out) *out = best;
    return true;
}

// 8-wave blocks (256-pixel tiles: two blocks of 8 waves per CU instead of three of 4) for the 64-row
// forward and the plain data gradient; 4 waves elsewhere (the BN-sum epilogue's registers, 128 rows' LDS)
static int convn_halo_waves(const ConvGArgs& a) {
    constexpr int env = PCX_AB_CONVN_NW;
    const int64_t M = a.mode == 0 ? a.cout : a.cin;
    const bool eight = M <= 64 && (a.mode == 0 || !a.ep_pg);
    if (env == 4 || env == 8) return eight ? env : 4;
    return eight ? 8 : 4;
}

// mode 1 here is always the BN-sum context (convn_stat_tiles): 4 waves
static bool convn_halo_ok(const ConvGArgs& a, HaloGeo* g, int nw = 4) {
    if ((a.mode != 0 && a.mode != 1) || a.stride != 1 || a.KH != 3 || a.KW != 3 || a.pad != 1) return false;
    if (a.mode == 0 ? (a.OH != a.IH || a.OW != a.IW) : (a.IH != a.OH || a.IW != a.OW)) return false;
    return convn_halo_tiles(a.mode == 0 ? a.OH : a.IH, a.mode == 0 ? a.OW : a.IW, 32 * nw, g);
}

int64_t convn_stat_tiles(const ConvGArgs& a) {
    HaloGeo g;
    const int nw = a.mode == 0 ? convn_halo_waves(a) : 4;
    if (convn_halo_ok(a, &g, nw)) return (int64_t)a.B * g.nsr * g.nsc;
    return ceil_div((int64_t)a.B * (a.mode == 1 ? (int64_t)a.IH * a.IW : (int64_t)a.OH * a.OW), 128);
}

int64_t convn_tile_bound(int B, int H, int W) {
    HaloGeo g;
    int64_t t = ceil_div((int64_t)B * H * W, 128);
    for (int px : {128, 256})
        if (convn_halo_tiles(H, W, px, &g)) t = std::max(t, (int64_t)B * g.nsr * g.nsc);
    return t;
}

bool convn_fits(const ConvGArgs& a) {
    if (a.KH != a.KW || (a.KH != 1 && a.KH != 3) || a.pad > 1 || a.pad < 0) return false;
    if (a.mode == 2) return a.cin % 8 == 0 && a.cout % 8 == 0;
    return (a.mode == 0 ? a.cin : a.cout) % NKB == 0;
}

// called by launch_convg_bf16 once the weights are packed (modes 0 / 1 / 3)
int launch_convn(const ConvGArgs& a, hipStream_t s) {
    PCX_CHECK_ARG(convn_fits(a), "convn: shape unsupported (k %d, pad %d, channels %d / %d)", a.KH, a.pad, a.cin, a.cout);
    const int64_t IHW = (int64_t)a.IH * a.IW, OHW = (int64_t)a.OH * a.OW;
    if (a.mode == 2) {
        PCX_CHECK_ARG(a.xn && a.dyn && a.kslice % NKB == 0 && a.nslice >= 1, "convn: bad weight-gradient arguments");
        const int64_t M = a.cout, N = (int64_t)a.cin * a.KH * a.KW;
        const int wm = M >= 128 ? 2 : 1;
        const int64_t nblocks = ceil_div(M, 64 * wm) * ceil_div(N, 128) * a.nslice;
        PCX_CHECK_ARG(nblocks < ((int64_t)1 << 31), "convn: grid too large");
        const unsigned grid = (unsigned)(8 * xcd_per(nblocks));
        if (wm == 2) convn_wgrad_kernel<2><<<grid, 256, 0, s>>>(a);
        else convn_wgrad_kernel<1><<<grid, 256, 0, s>>>(a);
        PCX_LAUNCH_CHECK("convn_wgrad_kernel");
        return PCX_OK;
    }
    PCX_CHECK_ARG(a.mode == 0 ? a.xn != nullptr : a.dyn != nullptr, "convn: missing channel-last operand");
    PCX_CHECK_ARG(a.wpack != nullptr, "convn: packed weights required");
    int64_t M, N;
    if (a.mode == 0) { M = a.cout; N = a.B * OHW; }
    else if (a.mode == 1) { M = a.cin; N = a.B * IHW; }
    else {
        M = a.cin;
        N = a.B * (int64_t)((a.IH - (a.par >> 1) + 1) / 2) * ((a.IW - (a.par & 1) + 1) / 2);
    }
    if (N == 0) return PCX_OK;
    int kh0 = 0, kw0 = 0, nth = a.KH, ntw = a.KW, step = 1;
    if (a.mode == 3) {
        kh0 = ((a.par >> 1) + a.pad) & 1;
        kw0 = ((a.par & 1) + a.pad) & 1;
        nth = (a.KH - kh0 + 1) / 2;
        ntw = (a.KW - kw0 + 1) / 2;
        step = 2;
        // a parity class without taps (1x1 stride 2) adds nothing
        if ((nth == 0 || ntw == 0) && a.accumulate) return PCX_OK;
    }
    const int ck = a.mode == 0 ? a.cin : a.cout;
    HaloGeo hg;
    const int hnw = a.mode == 3 ? 4 : convn_halo_waves(a);
    const bool halo = a.mode != 3 && convn_halo_ok(a, &hg, hnw);
    const int kc = halo ? 32 : convn_kc(ck);
    {
        const int64_t K = (int64_t)nth * ntw * ck;
        if (M * K > 0) {
            convn_pack_kernel<<<(unsigned)ceil_div(M * K, 256), 256, 0, s>>>(
                a.w, static_cast<__bf16*>(const_cast<void*>(a.wpack)), a.mode == 0 ? 0 : 1, a.cin, a.cout, a.KH, a.KW,
                kh0, kw0, step, ntw, nth * ntw, kc, M, K);
            PCX_LAUNCH_CHECK("convn_pack_kernel");
        }
    }
    const int wm = M >= 128 ? 2 : 1;
    const bool ep = a.ep_pg != nullptr;
    if (halo) {
        PCX_CHECK_ARG(!a.st_part0 || (a.mode == 0 && a.st_part1 && a.st_partn), "convn: forward statistics need mode 0");
        PCX_CHECK_ARG(!a.ep_pg || (a.mode == 1 && a.ep_px && a.ep_y && a.ep_cf && !a.accumulate),
                      "convn: data-gradient BN sums need mode 1, y, cf and both partial arrays");
        const int64_t nblocks = ceil_div(M, 64 * wm) * (int64_t)a.B * hg.nsr * hg.nsc;
        PCX_CHECK_ARG(nblocks < ((int64_t)1 << 31), "convn: grid too large");
        const size_t smem = (size_t)6 * 64 * wm * 64 + (size_t)2 * hg.hp * 64;
        dim3 grid((unsigned)(8 * xcd_per(nblocks)));
#define PCX_CH(MODE_, WM_, EP_, NW_)                                                                        \
        if (a.mode == MODE_ && wm == WM_ && ep == EP_ && hnw == NW_) {                                      \
            (void)hipFuncSetAttribute((const void*)convn_halo_kernel<MODE_, WM_, EP_, NW_>,                 \
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);               \
            convn_halo_kernel<MODE_, WM_, EP_, NW_><<<grid, 64 * NW_, smem, s>>>(a, hg);                    \
            PCX_LAUNCH_CHECK("convn_halo_kernel");                                                          \
            return PCX_OK;                                                                                  \
        }
        PCX_CH(0, 1, false, 4) PCX_CH(0, 2, false, 4) PCX_CH(1, 1, false, 4) PCX_CH(1, 2, false, 4)
        PCX_CH(1, 1, true, 4) PCX_CH(1, 2, true, 4) PCX_CH(0, 1, false, 8) PCX_CH(1, 1, false, 8)
#undef PCX_CH
    }
    constexpr int wn = 2;  // (128 x 256 tiles measured slower: 2 blocks per CU instead of 4)
    PCX_CHECK_ARG(!a.st_part0 || (a.mode == 0 && a.st_part1 && a.st_partn && convn_stat_tiles(a) == ceil_div(N, 64 * wn)),
                  "convn: forward statistics need mode 0 and all three partial arrays");
    PCX_CHECK_ARG(!a.ep_pg || (a.mode == 1 && a.ep_px && a.ep_y && a.ep_cf && !a.accumulate &&
                               convn_stat_tiles(a) == ceil_div(N, 64 * wn)),
                  "convn: data-gradient BN sums need mode 1 (stride 1, no accumulate), y, cf and both partial arrays");
    const int64_t nblocks = ceil_div(M, 64 * wm) * ceil_div(N, 64 * wn);
    PCX_CHECK_ARG(nblocks < ((int64_t)1 << 31), "convn: grid too large");
    dim3 grid((unsigned)(8 * xcd_per(nblocks)));
#define PCX_CN(MODE_, WM_, KC_, EP_)                                                           \
    if (a.mode == MODE_ && wm == WM_ && kc == KC_ && ep == EP_) {                              \
        convn_kernel<MODE_, WM_, KC_, EP_><<<grid, 256, 0, s>>>(a);                            \
        PCX_LAUNCH_CHECK("convn_kernel");                                                      \
        return PCX_OK;                                                                         \
    }
    PCX_CN(0, 1, 32, false) PCX_CN(0, 2, 32, false) PCX_CN(3, 1, 32, false) PCX_CN(3, 2, 32, false)
    PCX_CN(0, 1, 64, false) PCX_CN(0, 2, 64, false) PCX_CN(3, 1, 64, false) PCX_CN(3, 2, 64, false)
    PCX_CN(1, 1, 32, false) PCX_CN(1, 2, 32, false) PCX_CN(1, 1, 64, false) PCX_CN(1, 2, 64, false)
    PCX_CN(1, 1, 32, true) PCX_CN(1, 2, 32, true) PCX_CN(1, 1, 64, true) PCX_CN(1, 2, 64, true)
#undef PCX_CN
    set_error("convn: mode %d unsupported", a.mode);
    return PCX_EINVAL;
}

}  // namespace pcx
