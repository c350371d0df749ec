// General convolution (any cin/cout, KxK, stride 1 or 2, zero pad) as an implicit GEMM on
// v_mfma_f32_32x32x2_f32, plus the elementwise / per-channel-statistics kernels of the residual
// network (reference src/models/phoneme_cnn.py:146-304, PhonemeNetDeep + ResidualBlock).
//
//  mode 0  forward     y[b,n,oh,ow]   = sum_{c,kh,kw} W[n,c,kh,kw] x[b,c,oh*s-p+kh,ow*s-p+kw]
//                      GEMM  M = cout, N = B*OH*OW, K = cin*KH*KW
//  mode 1  data grad   dx[b,c,ih,iw]  = sum_{n,kh,kw} W[n,c,kh,kw] dy[b,n,(ih+p-kh)/s,(iw+p-kw)/s]
//                      (only taps where the division is exact and in range)
//                      GEMM  M = cin,  N = B*IH*IW, K = cout*KH*KW
//  mode 3  data grad of a stride-2 conv for one parity class (ih % 2, iw % 2) = (ph, pw): only the
//          taps kh = ph + p (mod 2), kw = pw + p (mod 2) reach those pixels, so the class is a dense
//          GEMM  M = cin, N = B*ceil((IH-ph)/2)*ceil((IW-pw)/2), K = cout*(valid taps); the four
//          classes cover dx exactly once with none of mode 1's zero taps (3/4 of its K at stride 2)
//  mode 2  weight grad dW[n,c,kh,kw]  = sum_{b,oh,ow} dy[b,n,oh,ow] x[b,c,oh*s-p+kh,ow*s-p+kw]
//                      GEMM  M = cout, N = cin*KH*KW, K = B*OH*OW split into slices (partials)
//
// Block = 4 waves in 2x2, each wave (32*WM) x (32*WN) of accumulators; K advances in chunks of 16
// staged through double-buffered LDS with the next chunk's global gathers in flight during the
// current chunk's MFMAs (one barrier per chunk).  Operands are gathered straight from the NCHW
// tensors (no im2col buffer).  Every output element is written by exactly one lane (no atomics):
// results are deterministic.
#include "kernels.h"

namespace pcx {
namespace {

constexpr int KC = 16;

// K order (modes 0, 1, 3) is tap-major: k = tap * CK + channel, CK = cin (mode 0) or cout (modes 1,
// 3).  With CK % 16 == 0 (FK) every K-chunk then shares one tap, so a thread's B gathers of a chunk
// are one bounds check and NBv loads at a fixed channel stride -- no per-element index arithmetic.
// Mode 2's N index is (tap, cin) likewise, its per-column decomposition hoisted out of the K loop.
template <int MODE, int KH, int KW, int WM, int WN, bool FK>
__global__ __launch_bounds__(256) void convg_kernel(ConvGArgs a) {
    constexpr int KK = KH * KW;
    constexpr int BM = 64 * WM, BN = 64 * WN;
    constexpr int SA = BM + 4, SB = BN + 4;
    constexpr int NA = BM / 16, NBv = BN / 16;  // staged elements per thread per chunk
    __shared__ float As[2][KC][SA];
    __shared__ float Bs[2][KC][SB];

    const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, l32 = lane & 31;
    const int wave = tid >> 6, wr = wave >> 1, wc = wave & 1;
    const int64_t OHW = (int64_t)a.OH * a.OW, IHW = (int64_t)a.IH * a.IW;
    const int s = a.stride, pad = a.pad;
    const int CK = MODE == 0 ? a.cin : a.cout;

    // parity class (mode 3): pixels (2 ihc + ph, 2 iwc + pw), taps kh0 + 2 i, kw0 + 2 j
    const int ph = a.par >> 1, pw = a.par & 1;
    const int kh0 = (ph + pad) & 1, kw0 = (pw + pad) & 1;
    const int nth = (KH - kh0 + 1) / 2, ntw = (KW - kw0 + 1) / 2, KKp = nth * ntw;
    const int IHc = (a.IH - ph + 1) / 2, IWc = (a.IW - pw + 1) / 2;
    const int64_t CHW = (int64_t)IHc * IWc;
    int64_t M, N, K;
    if (MODE == 0) { M = a.cout; N = a.B * OHW; K = (int64_t)a.cin * KK; }
    else if (MODE == 1) { M = a.cin; N = a.B * IHW; K = (int64_t)a.cout * KK; }
    else if (MODE == 3) { M = a.cin; N = a.B * CHW; K = (int64_t)a.cout * KKp; }
    else { M = a.cout; N = (int64_t)a.cin * KK; K = a.B * OHW; }
    const int64_t mt = (M + BM - 1) / BM, nt = (N + BN - 1) / BN;
    // XCD-aware order (grid padded to a multiple of 8): XCD x runs logical blocks [x per, (x + 1) per),
    // so the M tiles of a pixel tile / the N tiles of a K slice, which read the same rows, share an L2
    const int64_t nlog = mt * nt * (MODE == 2 ? a.nslice : 1), per = (nlog + 7) / 8;
    int64_t bid = (int64_t)(blockIdx.x & 7) * per + (blockIdx.x >> 3);
    if (bid >= nlog) return;
    const int64_t tq = udiv32(bid, mt), tm = bid - tq * mt;
    bid = tq;
    const int64_t tr_ = udiv32(bid, nt), tn = bid - tr_ * nt;
    const int slice = (int)tr_;
    const int64_t m0 = tm * BM, n0 = tn * BN;
    int64_t k_begin = 0, k_end = K;
    if (MODE == 2) {
        k_begin = (int64_t)slice * a.kslice;
        k_end = min(K, k_begin + a.kslice);
    }
    const int nch = (int)((k_end - k_begin + KC - 1) / KC);

    // ---- per-thread staging state
    const int kq = tid & 15;       // k-fast mapping: k offset within the chunk
    const int colq = tid >> 4;     // k-fast mapping: first column
    // column-fast mapping (B of modes 0/1/3): fixed pixel per thread
    const int bcol = tid % BN;
    const int brow = tid / BN;     // first k row; rows advance by 256/BN
    constexpr int BROWS = 256 / BN;
    int64_t xbase = 0;             // mode 0: x + b*cin*IHW ; modes 1, 3: dy + b*cout*OHW
    int ih0 = 0, iw0 = 0;          // mode 0: oh*s-p, ow*s-p ; modes 1, 3: ih+p, iw+p
    bool bvalid = false;
    if (MODE == 0 || MODE == 1 || MODE == 3) {
        const int64_t m = n0 + bcol;
        bvalid = m < N;
        const int64_t mm = bvalid ? m : 0;
        if (MODE == 3) {
            const int64_t b = udiv32(mm, CHW), p = mm - b * CHW;
            const int ihc = (int)udiv32(p, IWc), iwc = (int)(p - (int64_t)ihc * IWc);
            xbase = b * a.cout * OHW;
            ih0 = 2 * ihc + ph + pad;
            iw0 = 2 * iwc + pw + pad;
        } else if (MODE == 0) {
            const int64_t b = udiv32(mm, OHW), p = mm - b * OHW;
            const int oh = (int)udiv32(p, a.OW), ow = (int)(p - (int64_t)oh * a.OW);
            xbase = b * a.cin * IHW;
            ih0 = oh * s - pad;
            iw0 = ow * s - pad;
        } else {
            const int64_t b = udiv32(mm, IHW), p = mm - b * IHW;
            const int ih = (int)udiv32(p, a.IW), iw = (int)(p - (int64_t)ih * a.IW);
            xbase = b * a.cout * OHW;
            ih0 = ih + pad;
            iw0 = iw + pad;
        }
    }
    // mode 2: pixel tracker of k = k_begin + chunk*KC + kq, and the fixed (tap, channel) of each
    // staged B column
    int64_t pb = 0;
    int poh = 0, pow_ = 0;
    int wkh[MODE == 2 ? NBv : 1], wkw[MODE == 2 ? NBv : 1];
    int64_t wco[MODE == 2 ? NBv : 1];
    if (MODE == 2) {
        const int64_t q = k_begin + kq;
        pb = udiv32(q, OHW);
        const int64_t p = q - pb * OHW;
        poh = (int)udiv32(p, a.OW);
        pow_ = (int)(p - (int64_t)poh * a.OW);
#pragma unroll
        for (int i = 0; i < NBv; ++i) {
            const int64_t jj = n0 + colq + 16 * i;
            const int tap = (int)udiv32(jj, a.cin), c = (int)(jj - (int64_t)tap * a.cin);
            const bool jv = jj < N;
            wkh[i] = jv ? tap / KW - pad : -(1 << 28);  // out of range: never loads
            wkw[i] = tap % KW - pad;
            wco[i] = (int64_t)c * IHW;
        }
    }

    float ra[NA], rb[NBv];
    auto gather = [&](int chunk) {
        const int64_t kbase = k_begin + (int64_t)chunk * KC;
        if (MODE == 0 || MODE == 1 || MODE == 3) {
            // A: weights, k = kbase + kq -> (tap, channel)
            const int64_t k = kbase + kq;
            const int tap = (int)udiv32(k, CK), ch = (int)(k - (int64_t)tap * CK);
            const bool kv = k < K;
            if (a.wpack) {  // packed [M][K16] rows: 16 lanes read 64 contiguous bytes
                const float* wp = static_cast<const float*>(a.wpack) + k;
                const int64_t Kp = (K + KC - 1) / KC * KC;
#pragma unroll
                for (int j = 0; j < NA; ++j) {
                    const int64_t m = m0 + colq + 16 * j;
                    ra[j] = m < M ? wp[m * Kp] : 0.f;
                }
            } else
#pragma unroll
            for (int j = 0; j < NA; ++j) {
                const int64_t m = m0 + colq + 16 * j;
                float v = 0.f;
                if (kv && m < M) {
                    if (MODE == 0) v = a.w[(m * a.cin + ch) * KK + tap];
                    else if (MODE == 1) v = a.w[((int64_t)ch * a.cin + m) * KK + tap];
                    else v = a.w[(((int64_t)ch * a.cin + m) * KH + kh0 + 2 * (tap / ntw)) * KW + kw0 + 2 * (tap % ntw)];
                }
                ra[j] = v;
            }
        }
        if (MODE == 0) {
            if (FK) {  // one tap per chunk
                const int tap = (int)udiv32(kbase, CK), c0 = (int)(kbase - (int64_t)tap * CK);
                const int ih = ih0 + tap / KW, iw = iw0 + tap % KW;
                const bool ok = bvalid && ih >= 0 && ih < a.IH && iw >= 0 && iw < a.IW;
                const float* p = a.x + xbase + (int64_t)(c0 + brow) * IHW + (int64_t)ih * a.IW + iw;
#pragma unroll
                for (int i = 0; i < NBv; ++i) rb[i] = ok ? p[(int64_t)i * BROWS * IHW] : 0.f;
            } else {
#pragma unroll
                for (int i = 0; i < NBv; ++i) {
                    const int64_t kb = kbase + brow + BROWS * i;
                    float v = 0.f;
                    if (bvalid && kb < K) {
                        const int tap = (int)udiv32(kb, CK), c = (int)(kb - (int64_t)tap * CK);
                        const int ih = ih0 + tap / KW, iw = iw0 + tap % KW;
                        if (ih >= 0 && ih < a.IH && iw >= 0 && iw < a.IW)
                            v = a.x[xbase + ((int64_t)c * a.IH + ih) * a.IW + iw];
                    }
                    rb[i] = v;
                }
            }
        } else if (MODE == 1) {
            auto src = [&](int tap, int& oh, int& ow) {
                const int th = ih0 - tap / KW, tw = iw0 - tap % KW;
                oh = th;
                ow = tw;
                bool ok = th >= 0 && tw >= 0;
                if (s == 2) {
                    ok = ok && ((th | tw) & 1) == 0;
                    oh = th >> 1;
                    ow = tw >> 1;
                }
                return ok && oh < a.OH && ow < a.OW;
            };
            if (FK) {
                const int tap = (int)udiv32(kbase, CK), c0 = (int)(kbase - (int64_t)tap * CK);
                int oh = 0, ow = 0;
                const bool ok = bvalid && src(tap, oh, ow);
                const float* p = a.dy + xbase + (int64_t)(c0 + brow) * OHW + (int64_t)oh * a.OW + ow;
#pragma unroll
                for (int i = 0; i < NBv; ++i) rb[i] = ok ? p[(int64_t)i * BROWS * OHW] : 0.f;
            } else {
#pragma unroll
                for (int i = 0; i < NBv; ++i) {
                    const int64_t kb = kbase + brow + BROWS * i;
                    float v = 0.f;
                    if (bvalid && kb < K) {
                        const int tap = (int)udiv32(kb, CK), nn = (int)(kb - (int64_t)tap * CK);
                        int oh = 0, ow = 0;
                        if (src(tap, oh, ow)) v = a.dy[xbase + ((int64_t)nn * a.OH + oh) * a.OW + ow];
                    }
                    rb[i] = v;
                }
            }
        } else if (MODE == 3) {
            if (FK) {
                const int tap = (int)udiv32(kbase, CK), c0 = (int)(kbase - (int64_t)tap * CK);
                const int oh = (ih0 - (kh0 + 2 * (tap / ntw))) >> 1, ow = (iw0 - (kw0 + 2 * (tap % ntw))) >> 1;
                const bool ok = bvalid && oh >= 0 && ow >= 0 && oh < a.OH && ow < a.OW;
                const float* p = a.dy + xbase + (int64_t)(c0 + brow) * OHW + (int64_t)oh * a.OW + ow;
#pragma unroll
                for (int i = 0; i < NBv; ++i) rb[i] = ok ? p[(int64_t)i * BROWS * OHW] : 0.f;
            } else {
#pragma unroll
                for (int i = 0; i < NBv; ++i) {
                    const int64_t kb = kbase + brow + BROWS * i;
                    float v = 0.f;
                    if (bvalid && kb < K) {
                        const int tap = (int)udiv32(kb, CK), nn = (int)(kb - (int64_t)tap * CK);
                        const int oh = (ih0 - (kh0 + 2 * (tap / ntw))) >> 1, ow = (iw0 - (kw0 + 2 * (tap % ntw))) >> 1;
                        if (oh >= 0 && ow >= 0 && oh < a.OH && ow < a.OW)
                            v = a.dy[xbase + ((int64_t)nn * a.OH + oh) * a.OW + ow];
                    }
                    rb[i] = v;
                }
            }
        } else {
            const bool kval = (kbase + kq) < k_end;
            const int64_t pofs = (int64_t)poh * a.OW + pow_;
#pragma unroll
            for (int j = 0; j < NA; ++j) {
                const int64_t n = m0 + colq + 16 * j;
                float v = 0.f;
                if (kval && n < M) {
                    const int64_t o = (pb * a.cout + n) * OHW + pofs;
                    if (!FK) {  // mode 2: FK = false selects the BN-fused dy (launch_convg)
                        const float4 k = a.bn_cf[n];
                        v = k.x * (a.bn_g[o] - k.y - (a.bn_y[o] - k.w) * k.z);
                    } else {
                        v = a.dy[o];
                    }
                }
                ra[j] = v;
            }
            const float* xb = a.x + pb * a.cin * IHW;
            const int ihb = poh * s, iwb = pow_ * s;
#pragma unroll
            for (int i = 0; i < NBv; ++i) {
                const int ih = ihb + wkh[i], iw = iwb + wkw[i];
                rb[i] = (kval && ih >= 0 && ih < a.IH && iw >= 0 && iw < a.IW) ? xb[wco[i] + (int64_t)ih * a.IW + iw]
                                                                              : 0.f;
            }
            // advance the pixel tracker by KC
            pow_ += KC;
            while (pow_ >= a.OW) {
                pow_ -= a.OW;
                if (++poh == a.OH) { poh = 0; ++pb; }
            }
        }
    };
    auto stash = [&](int buf) {
#pragma unroll
        for (int j = 0; j < NA; ++j) As[buf][kq][colq + 16 * j] = ra[j];
        if (MODE == 2) {
#pragma unroll
            for (int i = 0; i < NBv; ++i) Bs[buf][kq][colq + 16 * i] = rb[i];
        } else {
#pragma unroll
            for (int i = 0; i < NBv; ++i) Bs[buf][brow + BROWS * i][bcol] = rb[i];
        }
    };

    f32x16 acc[WM][WN];
#pragma unroll
    for (int mi = 0; mi < WM; ++mi)
#pragma unroll
        for (int ni = 0; ni < WN; ++ni) acc[mi][ni] = f32x16{0.f};

    if (nch > 0) {
        gather(0);
        stash(0);
    }
    __syncthreads();
    for (int ch = 0; ch < nch; ++ch) {
        const int buf = ch & 1;
        if (ch + 1 < nch) gather(ch + 1);
#pragma unroll
        for (int ks = 0; ks < KC / 2; ++ks) {
            float av[WM], bv[WN];
#pragma unroll
            for (int mi = 0; mi < WM; ++mi) av[mi] = As[buf][2 * ks + h][wr * 32 * WM + mi * 32 + l32];
#pragma unroll
            for (int ni = 0; ni < WN; ++ni) bv[ni] = Bs[buf][2 * ks + h][wc * 32 * WN + ni * 32 + l32];
#pragma unroll
            for (int mi = 0; mi < WM; ++mi)
#pragma unroll
                for (int ni = 0; ni < WN; ++ni) acc[mi][ni] = mfma32(av[mi], bv[ni], acc[mi][ni]);
        }
        if (ch + 1 < nch) stash(buf ^ 1);
        __syncthreads();
    }

    // ---- epilogue: row = M index, column = N index (32 consecutive columns per lane group)
#pragma unroll
    for (int ni = 0; ni < WN; ++ni) {
        const int64_t col = n0 + wc * 32 * WN + ni * 32 + l32;
        if (col >= N) continue;
        int64_t obase;
        int64_t ostride;  // distance between consecutive rows (M index)
        float* dst = a.out;
        if (MODE == 0) {
            const int64_t b = udiv32(col, OHW);
            obase = b * a.cout * OHW + (col - b * OHW);
            ostride = OHW;
        } else if (MODE == 1) {
            const int64_t b = udiv32(col, IHW);
            obase = b * a.cin * IHW + (col - b * IHW);
            ostride = IHW;
        } else if (MODE == 3) {
            const int64_t b = udiv32(col, CHW), p = col - b * CHW;
            if (a.par_out) {  // dense class planes
                dst = a.par_out;
                obase = b * a.cin * CHW + p;
                ostride = CHW;
            } else {
                const int ihc = (int)udiv32(p, IWc), iwc = (int)(p - (int64_t)ihc * IWc);
                obase = b * a.cin * IHW + (int64_t)(2 * ihc + ph) * a.IW + 2 * iwc + pw;
                ostride = IHW;
            }
        } else {  // column (tap, c) -> the reference weight layout [cout][cin][KH][KW]
            const int tap = (int)udiv32(col, a.cin), c = (int)(col - (int64_t)tap * a.cin);
            obase = (int64_t)slice * M * N + (int64_t)c * KK + tap;
            ostride = N;
        }
#pragma unroll
        for (int mi = 0; mi < WM; ++mi)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int64_t row = m0 + wr * 32 * WM + mi * 32 + acc_row(r, h);
                if (row < M) {
                    float* o = dst + obase + row * ostride;
                    if ((MODE == 1 || MODE == 3) && a.accumulate) *o += acc[mi][ni][r];
                    else *o = acc[mi][ni][r];
                }
            }
    }
}

// ------------------------------------------------------------------ per-channel statistics
__device__ __forceinline__ double block_sum(double v, double* red) {
    const int tid = threadIdx.x;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    __syncthreads();
    if ((tid & 63) == 0) red[tid >> 6] = v;
    __syncthreads();
    return red[0] + red[1] + red[2] + red[3];
}

// Walk of the elements e = tid + 256 j of the planes (b, c) for b in [b0, b1): every lane busy
// whatever the plane size (the deep net's planes go down to 3 x 13 pixels), no per-element division.
struct PlaneWalk {
    int b, p, db, dp;
    __device__ __forceinline__ PlaneWalk(int b0, int P) {
        b = b0 + (int)threadIdx.x / P;
        p = (int)threadIdx.x % P;
        db = 256 / P;
        dp = 256 % P;
    }
    __device__ __forceinline__ void next(int P) {
        b += db;
        p += dp;
        if (p >= P) { p -= P; ++b; }
    }
};

// Forward BN partials of y [B][C][P]: block (c, slice) -> (sum, M2 about the block mean, count).
// Elements are walked in units of V (16-byte loads when P % 4 == 0), U units in flight per thread;
// a unit's shifted values are summed in float32, the running sums are float64 about a shift (the
// slice's first element) — consumed by launch_bn_fwd_finalize.
template <int V, int U>
__global__ __launch_bounds__(256) void chan_stats_kernel(const float* __restrict__ y, int B, int C, int64_t P64,
                                                         int bps, float* part0, float* part1, float* partn) {
    typedef float fv __attribute__((ext_vector_type(V)));
    __shared__ double red[4];
    const int c = blockIdx.x, sl = blockIdx.y, nsl = gridDim.y;
    const int b0 = sl * bps, b1 = min(B, b0 + bps);
    const int P = (int)P64, PV = P / V;
    const float K = b0 < B ? y[((int64_t)b0 * C + c) * P] : 0.f;
    double s1 = 0.0, s2 = 0.0;
    PlaneWalk w(b0, PV);
    while (w.b < b1) {
        fv v[U];
        bool ok[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            ok[u] = w.b < b1;
            v[u] = ok[u] ? *reinterpret_cast<const fv*>(y + ((int64_t)w.b * C + c) * P + (int64_t)w.p * V) : fv{};
            w.next(PV);
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (ok[u]) {
                float t1 = 0.f, t2 = 0.f;
#pragma unroll
                for (int e = 0; e < V; ++e) {
                    const float d = v[u][e] - K;
                    t1 += d;
                    t2 = fmaf(d, d, t2);
                }
                s1 += (double)t1;
                s2 += (double)t2;
            }
    }
    s1 = block_sum(s1, red);
    s2 = block_sum(s2, red);
    if (threadIdx.x == 0) {
        const double n = (double)(b1 > b0 ? b1 - b0 : 0) * (double)P;
        part0[(int64_t)c * nsl + sl] = (float)(n * (double)K + s1);
        part1[(int64_t)c * nsl + sl] = n > 0 ? (float)fmax(s2 - s1 * s1 / n, 0.0) : 0.f;
        if (c == 0) partn[sl] = (float)n;
    }
}

// n / d for 0 <= n < 2^22 with inv = 1 / d (float): one correction step makes it exact
__device__ __forceinline__ int wdiv_f(int n, int d, float inv) {
    int q = (int)((float)n * inv);
    const int r = n - q * d;
    q += r >= d ? 1 : 0;
    q -= r < 0 ? 1 : 0;
    return q;
}

// Backward BN partials: g = d (+ d2) masked, written to g; sums of g and g*xhat_k for up to two
// BNs (the main-path BN and the shortcut BN of a residual block share the same upstream g).
// Units of V elements (16-byte accesses when P % 4 == 0), U units in flight per thread.
template <int V, int U>
__global__ __launch_bounds__(256) void bwd_prep_kernel(BwdPrepArgs a) {
    typedef float fv __attribute__((ext_vector_type(V)));
    __shared__ double red[4];
    const int c = blockIdx.x, sl = blockIdx.y, nsl = gridDim.y;
    const int b0 = sl * a.bps, b1 = min(a.B, b0 + a.bps);
    const int P = (int)a.P, PV = P / V;
    const float4 mc = a.mask_cf ? a.mask_cf[c] : make_float4(1.f, 0.f, 0.f, 1.f);
    const float4 c1 = a.cf1 ? a.cf1[c] : make_float4(0.f, 0.f, 0.f, 0.f);
    const float4 c2 = a.cf2 ? a.cf2[c] : make_float4(0.f, 0.f, 0.f, 0.f);
    const float a_invW = a.dpar ? 1.f / (float)a.W : 0.f;
    double sg = 0.0, sx1 = 0.0, sx2 = 0.0;
    PlaneWalk w(b0, PV);
    while (w.b < b1) {
        int64_t o[U], bc[U];
        bool ok[U];
        fv g[U], m[U], y1v[U], y2v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            ok[u] = w.b < b1;
            bc[u] = (int64_t)(ok[u] ? w.b : b0) * a.C + c;
            o[u] = bc[u] * P + (ok[u] ? (int64_t)w.p * V : 0);
            w.next(PV);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (a.dpar) {  // class-planar d: the V elements from their parity classes
                const int p0 = (int)(o[u] - bc[u] * P), W = a.W;
                bool done = false;
                if constexpr (V == 4) {
                    if ((W & 3) == 0) {  // one row, columns w0 .. w0 + 3 (w0 % 4 == 0): two 8-byte loads
                        const int h = wdiv_f(p0, W, a_invW), w0 = p0 - h * W;
                        const int r = h & 1, IWc = W >> 1, IHc = (a.H - r + 1) >> 1;
                        const int64_t so = bc[u] * IHc * IWc + (int64_t)(h >> 1) * IWc + (w0 >> 1);
                        const float2 e = *reinterpret_cast<const float2*>(a.dpar + a.dpo[2 * r] + so);
                        const float2 od = *reinterpret_cast<const float2*>(a.dpar + a.dpo[2 * r + 1] + so);
                        g[u] = fv{e.x, od.x, e.y, od.y};
                        done = true;
                    } else if ((W & 1) == 0) {  // two column pairs (w, w + 1), w even: one division each
                        const int IWc = W >> 1;
#pragma unroll
                        for (int k2 = 0; k2 < 2; ++k2) {
                            const int pp = p0 + 2 * k2, h = wdiv_f(pp, W, a_invW), w = pp - h * W;
                            const int r = h & 1, IHc = (a.H - r + 1) >> 1;
                            const int64_t so = bc[u] * IHc * IWc + (int64_t)(h >> 1) * IWc + (w >> 1);
                            g[u][2 * k2] = a.dpar[a.dpo[2 * r] + so];
                            g[u][2 * k2 + 1] = a.dpar[a.dpo[2 * r + 1] + so];
                        }
                        done = true;
                    }
                }
                if (!done) {
#pragma unroll
                    for (int e = 0; e < V; ++e) {
                        const int pp = p0 + e, h = wdiv_f(pp, W, a_invW), w = pp - h * W;
                        const int q = 2 * (h & 1) + (w & 1);
                        const int IHc = (a.H - (h & 1) + 1) >> 1, IWc = (W - (w & 1) + 1) >> 1;
                        g[u][e] = pp < P ? a.dpar[a.dpo[q] + bc[u] * IHc * IWc + (int64_t)(h >> 1) * IWc + (w >> 1)] : 0.f;
                    }
                }
            } else {
                g[u] = *reinterpret_cast<const fv*>(a.d + o[u]);
            }
            if (a.d2) g[u] += *reinterpret_cast<const fv*>(a.d2 + o[u]);
            if (a.mask_mode == MASK_OUT8) {  // V mask bytes as 0 / 1 floats
                unsigned mb;
                if (V == 4) mb = *reinterpret_cast<const unsigned*>(a.mask8 + o[u]);
                else mb = a.mask8[o[u]];
#pragma unroll
                for (int e = 0; e < V; ++e) m[u][e] = (float)((mb >> (8 * e)) & 0xffu);
            } else {
                m[u] = a.mask_mode != MASK_NONE ? *reinterpret_cast<const fv*>(a.mask_src + o[u]) : fv{};
            }
            y1v[u] = a.y1 ? *reinterpret_cast<const fv*>(a.y1 + o[u]) : fv{};
            y2v[u] = a.y2 ? *reinterpret_cast<const fv*>(a.y2 + o[u]) : fv{};
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (!ok[u]) continue;
            const float dr = a.mask_mode == MASK_BN && a.drop ? a.drop[bc[u]] : 1.f;
            fv gv = g[u];
            float tg = 0.f, t1 = 0.f, t2 = 0.f;
#pragma unroll
            for (int e = 0; e < V; ++e) {
                if (a.mask_mode == MASK_OUT || a.mask_mode == MASK_OUT8) gv[e] = m[u][e] > 0.f ? gv[e] : 0.f;
                else if (a.mask_mode == MASK_BN) gv[e] = fmaf(m[u][e], mc.x, mc.y) > 0.f ? gv[e] * dr : 0.f;
                tg += gv[e];
                if (a.y1) t1 = fmaf(gv[e], (y1v[u][e] - c1.z) * c1.w, t1);
                if (a.y2) t2 = fmaf(gv[e], (y2v[u][e] - c2.z) * c2.w, t2);
            }
            if (a.g) *reinterpret_cast<fv*>(a.g + o[u]) = gv;
            sg += (double)tg;
            sx1 += (double)t1;
            sx2 += (double)t2;
        }
    }
    sg = block_sum(sg, red);
    sx1 = block_sum(sx1, red);
    sx2 = block_sum(sx2, red);
    if (threadIdx.x == 0) {
        a.p_g[(int64_t)c * nsl + sl] = (float)sg;
        if (a.p_x1) a.p_x1[(int64_t)c * nsl + sl] = (float)sx1;
        if (a.p_x2) a.p_x2[(int64_t)c * nsl + sl] = (float)sx2;
    }
}

// ------------------------------------------------------------------ elementwise (row tiled)
// rows = B*C planes of P elements; TP threads per row, 256/TP rows per block
struct RowTile {
    int64_t row;
    int col0, step;
};
__device__ __forceinline__ RowTile row_tile(int TP) {
    RowTile t;
    t.row = (int64_t)blockIdx.x * (256 / TP) + threadIdx.x / TP;
    t.col0 = threadIdx.x % TP;
    t.step = TP;
    return t;
}

// out = drop[b,c] * relu(y*s + t + res')   res' = res*rs + rt (rcf) | res | 0
__global__ __launch_bounds__(256) void bn_act_kernel(const float* __restrict__ y, const float4* __restrict__ cf,
                                                     const float* __restrict__ res, const float4* __restrict__ rcf,
                                                     const float* __restrict__ drop, float* __restrict__ out,
                                                     int64_t rows, int C, int64_t P, int TP) {
    const RowTile t = row_tile(TP);
    if (t.row >= rows) return;
    const int c = (int)(t.row % C);
    const float4 k = cf[c];
    const float4 rk = rcf ? rcf[c] : make_float4(1.f, 0.f, 0.f, 0.f);
    const float d = drop ? drop[t.row] : 1.f;
    const int64_t o = t.row * P;
    for (int64_t p = t.col0; p < P; p += t.step) {
        float v = fmaf(y[o + p], k.x, k.y);
        if (res) v += fmaf(res[o + p], rk.x, rk.y);
        out[o + p] = d * fmaxf(v, 0.f);
    }
}

// dy = a*(g - mb - (y - mean)*mgi)      (cf = {a, mb, mgi, mean})
__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(const float* g, const float* __restrict__ y,
                                                           const float4* __restrict__ cf, float* dy,
                                                           int64_t rows, int C, int64_t P, int TP) {
    const RowTile t = row_tile(TP);
    if (t.row >= rows) return;
    const float4 k = cf[(int)(t.row % C)];
    const int64_t o = t.row * P;
    for (int64_t p = t.col0; p < P; p += t.step)
        dy[o + p] = k.x * (g[o + p] - k.y - (y[o + p] - k.w) * k.z);
}

// Flat forms of the two kernels above for short rows (the 10 x 50 .. 3 x 13 planes of cnn_deep's later
// blocks): a row per 64-256 threads left most lanes idle and launched one block per 1-4 rows; here
// each thread takes 4 consecutive elements (one 16-byte access per operand, rows cross freely: the
// channel of each element follows from one division per quad), 2048 elements per block.
template <int OP>  // 0: bn_act, 1: bn_bwd_apply
__global__ __launch_bounds__(256) void bn_flat_kernel(const float* __restrict__ y, const float4* __restrict__ cf,
                                                      const float* __restrict__ res, const float4* __restrict__ rcf,
                                                      const float* __restrict__ drop, const float* g,
                                                      float* out, int64_t n, int C, int P) {
    for (int64_t q = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4; q < n; q += (int64_t)gridDim.x * 1024) {
        const int64_t row0 = q / P;
        int p = (int)(q - row0 * P), row = (int)row0, c = row % C;
        float4 yv, rv = make_float4(0.f, 0.f, 0.f, 0.f), gv = make_float4(0.f, 0.f, 0.f, 0.f);
        const bool full = q + 4 <= n;
        if (full) {
            yv = *reinterpret_cast<const float4*>(y + q);
            if (OP == 0 && res) rv = *reinterpret_cast<const float4*>(res + q);
            if (OP == 1) gv = *reinterpret_cast<const float4*>(g + q);
        } else {
            float t[4] = {0.f, 0.f, 0.f, 0.f}, r[4] = {0.f, 0.f, 0.f, 0.f}, u[4] = {0.f, 0.f, 0.f, 0.f};
            for (int j = 0; j < 4 && q + j < n; ++j) {
                t[j] = y[q + j];
                if (OP == 0 && res) r[j] = res[q + j];
                if (OP == 1) u[j] = g[q + j];
            }
            yv = make_float4(t[0], t[1], t[2], t[3]);
            rv = make_float4(r[0], r[1], r[2], r[3]);
            gv = make_float4(u[0], u[1], u[2], u[3]);
        }
        float yy[4] = {yv.x, yv.y, yv.z, yv.w}, rr[4] = {rv.x, rv.y, rv.z, rv.w}, gg[4] = {gv.x, gv.y, gv.z, gv.w};
        float o[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const float4 k = cf[c];
            if (OP == 0) {
                const float4 rk = rcf ? rcf[c] : make_float4(1.f, 0.f, 0.f, 0.f);
                const float d = drop ? drop[row] : 1.f;
                float v = fmaf(yy[j], k.x, k.y);
                if (res) v += fmaf(rr[j], rk.x, rk.y);
                o[j] = d * fmaxf(v, 0.f);
            } else {
                o[j] = k.x * (gg[j] - k.y - (yy[j] - k.w) * k.z);
            }
            if (++p == P) {
                p = 0;
                ++row;
                if (++c == C) c = 0;
            }
        }
        if (full) *reinterpret_cast<float4*>(out + q) = make_float4(o[0], o[1], o[2], o[3]);
        else
            for (int j = 0; j < 4 && q + j < n; ++j) out[q + j] = o[j];
    }
}

// MaxPool2d(3, stride 2, pad 1) of relu(BN(y))  (reference phoneme_cnn.py:211-216).  One block per
// channel plane (32-bit index math).  Also records, per window, the tap (kh*3 + kw) of its first
// maximum in row-major scan order (torch's tie rule), or 255 when that maximum is 0 (the ReLU then
// passes no gradient), so the backward never re-reads y.
__global__ __launch_bounds__(256) void maxpool3_fwd_kernel(const float* __restrict__ y, const float4* __restrict__ cf,
                                                           float* __restrict__ out, uint8_t* __restrict__ arg, int C,
                                                           int H, int W, int OH, int OW) {
    const int64_t row = blockIdx.x;
    const float4 k = cf[(int)(row % C)];
    const float* yp = y + row * H * W;
    float* op = out + row * OH * OW;
    uint8_t* ap = arg + row * OH * OW;
    // rows x columns walk (no per-element division): OW-wide row segments of 256 threads
    const int segs = (OW + 255) / 256;
    for (int q = 0; q < OH * segs; ++q) {
        const int oh = q / segs, ow = (q - oh * segs) * 256 + threadIdx.x;
        if (ow >= OW) continue;
        const int p = oh * OW + ow;
        float m = -INFINITY;
        int best = 0;
#pragma unroll
        for (int kh = 0; kh < 3; ++kh) {
            const int ih = 2 * oh - 1 + kh;
            if (ih < 0 || ih >= H) continue;
#pragma unroll
            for (int kw = 0; kw < 3; ++kw) {
                const int iw = 2 * ow - 1 + kw;
                if (iw < 0 || iw >= W) continue;
                const float v = fmaxf(fmaf(yp[ih * W + iw], k.x, k.y), 0.f);
                if (v > m) { m = v; best = kh * 3 + kw; }
            }
        }
        op[p] = m;
        ap[p] = m > 0.f ? (uint8_t)best : (uint8_t)255;
    }
}

// gradient of MaxPool(3,2,1)(relu(BN(y))) w.r.t. the BN output: each input position collects
// dout of the (at most 2 x 2) windows whose recorded first maximum it is
__global__ __launch_bounds__(256) void maxpool3_bwd_kernel(const uint8_t* __restrict__ arg,
                                                           const float* __restrict__ dout, float* __restrict__ dz,
                                                           int H, int W, int OH, int OW) {
    const int64_t row = blockIdx.x;
    const uint8_t* ap = arg + row * OH * OW;
    const float* dp = dout + row * OH * OW;
    float* zp = dz + row * H * W;
    const int segs = (W + 255) / 256;
    for (int q = 0; q < H * segs; ++q) {
        const int ih = q / segs, iw = (q - ih * segs) * 256 + threadIdx.x;
        if (iw >= W) continue;
        const int p = ih * W + iw;
        const int oh_lo = ih / 2, oh_hi = min(OH - 1, (ih + 1) / 2);
        const int ow_lo = iw / 2, ow_hi = min(OW - 1, (iw + 1) / 2);
        float g = 0.f;
        for (int oh = oh_lo; oh <= oh_hi; ++oh)
            for (int ow = ow_lo; ow <= ow_hi; ++ow) {
                const int kh = ih - (2 * oh - 1), kw = iw - (2 * ow - 1);
                if (ap[oh * OW + ow] == kh * 3 + kw) g += dp[oh * OW + ow];
            }
        zp[p] = g;
    }
}

// LDS-plane forms of the two kernels above (the stem planes, 40 x 200 at T = 200, fit): the plane is
// read once with coalesced (float4 when VEC = 4) loads, BN + ReLU applied on the way into LDS, and
// every window / gather then reads LDS.  Same results, same tie rule, bit for bit.
template <int VEC>
__global__ __launch_bounds__(256) void maxpool3_fwd_lds_kernel(const float* __restrict__ y,
                                                               const float4* __restrict__ cf, float* __restrict__ out,
                                                               uint8_t* __restrict__ arg, int C, int H, int W, int OH,
                                                               int OW) {
    extern __shared__ __attribute__((aligned(16))) float pl[];  // [H][W]
    const int64_t row = blockIdx.x;
    const float4 k = cf[(int)(row % C)];
    const int HW = H * W, OHW = OH * OW;
    const float* yp = y + row * HW;
    for (int i = threadIdx.x; i < HW / VEC; i += 256) {
        if (VEC == 4) {
            float4 v = reinterpret_cast<const float4*>(yp)[i];
            v.x = fmaxf(fmaf(v.x, k.x, k.y), 0.f);
            v.y = fmaxf(fmaf(v.y, k.x, k.y), 0.f);
            v.z = fmaxf(fmaf(v.z, k.x, k.y), 0.f);
            v.w = fmaxf(fmaf(v.w, k.x, k.y), 0.f);
            reinterpret_cast<float4*>(pl)[i] = v;
        } else {
            pl[i] = fmaxf(fmaf(yp[i], k.x, k.y), 0.f);
        }
    }
    __syncthreads();
    float* op = out + row * OHW;
    uint8_t* ap = arg + row * OHW;
    // output walk: p = tid + 256 j, (oh, ow) tracked without division
    int oh = threadIdx.x / OW, ow = threadIdx.x - oh * OW;
    const int doh = 256 / OW, dow = 256 - doh * OW;
    for (int p = threadIdx.x; p < OHW; p += 256) {
        float m = -INFINITY;
        int best = 0;
#pragma unroll
        for (int kh = 0; kh < 3; ++kh) {
            const int ih = 2 * oh - 1 + kh;
            if (ih < 0 || ih >= H) continue;
#pragma unroll
            for (int kw = 0; kw < 3; ++kw) {
                const int iw = 2 * ow - 1 + kw;
                if (iw < 0 || iw >= W) continue;
                const float v = pl[ih * W + iw];
                if (v > m) { m = v; best = kh * 3 + kw; }
            }
        }
        op[p] = m;
        ap[p] = m > 0.f ? (uint8_t)best : (uint8_t)255;
        oh += doh;
        ow += dow;
        if (ow >= OW) { ow -= OW; ++oh; }
    }
}

// MaxPool(3,2,1) + ReLU backward fused with the stem BN's backward sums (replaces
// maxpool3_bwd_kernel + bwd_prep_kernel on the stem): block (c, slice) walks its samples' planes of
// channel c; per plane the pooled gradient and the recorded taps are staged in LDS, every input
// pixel gathers its (at most 2 x 2) windows, g is written once and sum(g), sum(g * xhat) go to the
// same [C][nslice] partials bwd_prep_kernel produces.  SEL: the BN input of a pixel is the pooled
// ysel value of a window that selected it (every gradient-carrying pixel is some window's selection;
// the others contribute 0), so no y plane is read.
template <int VEC, bool SEL>
__global__ __launch_bounds__(256) void maxpool3_bwd_prep_kernel(const uint8_t* __restrict__ arg,
                                                                const float* __restrict__ dout,
                                                                const float* __restrict__ dout2,
                                                                const float* __restrict__ y,
                                                                const float4* __restrict__ cf, float* __restrict__ g,
                                                                float* __restrict__ p_g, float* __restrict__ p_x, int B,
                                                                int C, int H, int W, int OH, int OW, int bps) {
    // [OH*OW] gradients, (SEL) [OH*OW] selected inputs, then [OH*OW] taps
    extern __shared__ __attribute__((aligned(16))) float dl[];
    __shared__ double red[4];
    const int c = blockIdx.x, sl = blockIdx.y, nsl = gridDim.y;
    const int b0 = sl * bps, b1 = min(B, b0 + bps);
    const int HW = H * W, OHW = OH * OW, WQ = W / VEC, HWQ = HW / VEC;
    float* ysl = dl + OHW;
    uint8_t* al = reinterpret_cast<uint8_t*>(dl + (SEL ? 2 : 1) * OHW);
    const float4 k = cf[c];
    double sg = 0.0, sx = 0.0;
    const int q0h = threadIdx.x / WQ, q0w = threadIdx.x - q0h * WQ;
    const int dqh = 256 / WQ, dqw = 256 - dqh * WQ;
    for (int b = b0; b < b1; ++b) {
        const int64_t row = (int64_t)b * C + c;
        for (int i = threadIdx.x; i < OHW; i += 256) {
            dl[i] = dout2 ? dout[row * OHW + i] + dout2[row * OHW + i] : dout[row * OHW + i];
            al[i] = arg[row * OHW + i];
            if (SEL) ysl[i] = y[row * OHW + i];
        }
        __syncthreads();
        const float* yp = y + row * HW;
        float* gp = g + row * HW;
        int ih = q0h, iq = q0w;
        for (int q = threadIdx.x; q < HWQ; q += 256) {
            float gv[VEC], yv[VEC];
            if (SEL) {
#pragma unroll
                for (int e = 0; e < VEC; ++e) yv[e] = 0.f;
            } else if (VEC == 4) {
                const float4 t = reinterpret_cast<const float4*>(yp)[q];
                yv[0] = t.x; yv[1] = t.y; yv[2] = t.z; yv[3] = t.w;
            } else {
                yv[0] = yp[q];
            }
            const int oh_lo = ih >> 1, oh_hi = min(OH - 1, (ih + 1) >> 1);
#pragma unroll
            for (int e = 0; e < VEC; ++e) {
                const int iw = iq * VEC + e;
                const int ow_lo = iw >> 1, ow_hi = min(OW - 1, (iw + 1) >> 1);
                float acc = 0.f;
                for (int oh = oh_lo; oh <= oh_hi; ++oh)
                    for (int ow = ow_lo; ow <= ow_hi; ++ow) {
                        const int kh = ih - (2 * oh - 1), kw = iw - (2 * ow - 1);
                        if (al[oh * OW + ow] == kh * 3 + kw) {
                            acc += dl[oh * OW + ow];
                            if (SEL) yv[e] = ysl[oh * OW + ow];
                        }
                    }
                gv[e] = acc;
                sg += (double)acc;
                sx += (double)acc * (double)((yv[e] - k.z) * k.w);
            }
            if (VEC == 4) reinterpret_cast<float4*>(gp)[q] = make_float4(gv[0], gv[1], gv[2], gv[3]);
            else gp[q] = gv[0];
            ih += dqh;
            iq += dqw;
            if (iq >= WQ) { iq -= WQ; ++ih; }
        }
        __syncthreads();
    }
    sg = block_sum(sg, red);
    sx = block_sum(sx, red);
    if (threadIdx.x == 0) {
        p_g[(int64_t)c * nsl + sl] = (float)sg;
        p_x[(int64_t)c * nsl + sl] = (float)sx;
    }
}

// Class-planar stride-2 data gradient -> dx (the parity classes' dense planes written by the
// channel-last engine, ConvGArgs::par_out).  VW = 4 (W % 4 == 0): a thread writes 4 consecutive
// elements of a dx row (one 16-byte store) from two 8-byte loads of its row parity's two column
// classes; VW = 2 (W even): 2 elements (8-byte store) from one element of each; VW = 1: one element.
template <int VW>
__global__ __launch_bounds__(256) void par_interleave_kernel(const float* __restrict__ src, float* __restrict__ dx,
                                                             unsigned total, int IH, int IW, int acc, int64_t o1,
                                                             int64_t o2, int64_t o3) {
    const unsigned t = blockIdx.x * 256u + threadIdx.x;
    if (t >= total) return;
    const int64_t off[4] = {0, o1, o2, o3};
    if (VW == 2) {
        const unsigned IW2 = (unsigned)IW >> 1, per = (unsigned)IH * IW2;
        const unsigned pl = t / per, rem = t - pl * per, ih = rem / IW2, k = rem - ih * IW2;
        const int r = ih & 1, IWc = IW >> 1, IHc = (IH - r + 1) >> 1;
        const int64_t so = (int64_t)pl * IHc * IWc + (int64_t)(ih >> 1) * IWc + k;
        float2 v = make_float2(src[off[2 * r] + so], src[off[2 * r + 1] + so]);
        float2* d = reinterpret_cast<float2*>(dx + (int64_t)pl * IH * IW + (int64_t)ih * IW + 2 * k);
        if (acc) {
            const float2 u = *d;
            v.x += u.x;
            v.y += u.y;
        }
        *d = v;
    } else if (VW == 4) {
        const unsigned IW4 = (unsigned)IW >> 2, per = (unsigned)IH * IW4;
        const unsigned pl = t / per, rem = t - pl * per, ih = rem / IW4, k = rem - ih * IW4;
        const int r = ih & 1, IWc = IW >> 1, IHc = (IH - r + 1) >> 1;
        const int64_t CHW = (int64_t)IHc * IWc;
        const int64_t so = (int64_t)pl * CHW + (int64_t)(ih >> 1) * IWc + 2 * k;
        const float2 e = *reinterpret_cast<const float2*>(src + off[2 * r] + so);
        const float2 o = *reinterpret_cast<const float2*>(src + off[2 * r + 1] + so);
        float4 v = make_float4(e.x, o.x, e.y, o.y);
        float4* d = reinterpret_cast<float4*>(dx + (int64_t)pl * IH * IW + (int64_t)ih * IW + 4 * k);
        if (acc) {
            const float4 u = *d;
            v.x += u.x; v.y += u.y; v.z += u.z; v.w += u.w;
        }
        *d = v;
    } else {
        const unsigned per = (unsigned)IH * IW;
        const unsigned pl = t / per, rem = t - pl * per, ih = rem / IW, iw = rem - ih * IW;
        const int q = (ih & 1) * 2 + (iw & 1);
        const int IHc = (IH - (q >> 1) + 1) >> 1, IWc = (IW - (q & 1) + 1) >> 1;
        const float v = src[off[q] + (int64_t)pl * IHc * IWc + (int64_t)(ih >> 1) * IWc + (iw >> 1)];
        float* d = dx + t;
        *d = acc ? *d + v : v;
    }
}

__global__ void fill_cf_kernel(float4* cf, int C, float4 v) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c < C) cf[c] = v;
}

int row_threads(int64_t P) {
    int tp = 32;
    while (tp < 256 && tp < P) tp <<= 1;
    return tp;
}

}  // namespace

// ====================================================================== host launchers
int convg_nslice(const ConvGArgs& a, int64_t* kslice) {
    // weight-gradient split: enough (M-tile, N-tile, slice) blocks to fill the chip several times
    const int64_t K = (int64_t)a.B * a.OH * a.OW;
    const int wm = a.cout >= 128 ? 2 : 1;
    const int64_t mt = ceil_div(a.cout, 64 * wm), nt = ceil_div((int64_t)a.cin * a.KH * a.KW, 128);
    int64_t want = std::max<int64_t>(1, 2048 / (mt * nt));
    int64_t ks = (K + want - 1) / want;
    ks = std::max<int64_t>(ks, 256);
    ks = (ks + 31) / 32 * 32;  // the bf16 form advances 32 pixels per chunk
    *kslice = ks;
    return (int)((K + ks - 1) / ks);
}

namespace {
// fp32 A operand of modes 0 / 1 / 3 packed once per launch as [M][K rounded to 16] (tap-major k)
__global__ __launch_bounds__(256) void pack_wf32_kernel(const float* __restrict__ w, float* __restrict__ wp, int mode,
                                                        int cin, int cout, int KH, int KW, int par, int pad, int64_t M,
                                                        int64_t Kp, int64_t K) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= M * Kp) return;
    const int64_t m = i / Kp, k = i - m * Kp;
    float v = 0.f;
    if (k < K) {
        const int KK = KH * KW;
        if (mode == 0) {
            const int tap = (int)(k / cin), c = (int)(k - (int64_t)tap * cin);
            v = w[(m * cin + c) * KK + tap];
        } else if (mode == 1) {
            const int tap = (int)(k / cout), n = (int)(k - (int64_t)tap * cout);
            v = w[((int64_t)n * cin + m) * KK + tap];
        } else {
            const int ph = par >> 1, pw = par & 1;
            const int kh0 = (ph + pad) & 1, kw0 = (pw + pad) & 1, ntw = (KW - kw0 + 1) / 2;
            const int tp = (int)(k / cout), n = (int)(k - (int64_t)tp * cout);
            v = w[(((int64_t)n * cin + m) * KH + kh0 + 2 * (tp / ntw)) * KW + kw0 + 2 * (tp % ntw)];
        }
    }
    wp[i] = v;
}
}  // namespace

size_t convg_wpack_bytes(int mode, int cin, int cout, int k) {
    if (mode == 2) return 0;
    const int64_t M = mode == 0 ? cout : cin, K = (int64_t)(mode == 0 ? cin : cout) * k * k;
    return (size_t)M * ((K + KC - 1) / KC * KC) * 4;
}

int launch_convg(ConvGArgs a, hipStream_t s) {
    PCX_CHECK_ARG(a.stride == 1 || a.stride == 2, "convg: stride %d unsupported", a.stride);
    PCX_CHECK_ARG(a.B > 0 && a.cin > 0 && a.cout > 0, "convg: empty tensor");
    PCX_CHECK_ARG(!a.par_out || ((a.mode == 1 || a.mode == 3) && a.stride == 2 && (!a.bf16 || a.dyn)),
                  "convg: class-planar output only for the stride-2 data gradient (fp32 or channel-last)");
    if (a.mode == 1 && a.stride == 2) {
        for (int par = 0; par < 4; ++par) {  // each parity class of dx written exactly once
            // a class no tap reaches (1x1 stride-2 shortcut: classes 1..3) adds nothing: skipped when
            // accumulating (it used to re-read and re-write those class planes unchanged)
            const int kh0 = ((par >> 1) + a.pad) & 1, kw0 = ((par & 1) + a.pad) & 1;
            if (a.accumulate && ((a.KH - kh0 + 1) / 2) * ((a.KW - kw0 + 1) / 2) == 0) continue;
            ConvGArgs c = a;
            c.mode = 3;
            c.par = par;
            if (a.par_out) c.par_out = a.par_out + par_off(a.B, a.cin, a.IH, a.IW, par);
            const int rc = launch_convg(c, s);
            if (rc != PCX_OK) return rc;
        }
        return PCX_OK;
    }
    if (a.bf16) return launch_convg_bf16(a, s);
    const int64_t IHW = (int64_t)a.IH * a.IW, OHW = (int64_t)a.OH * a.OW;
    int64_t M, N;
    if (a.mode == 0) { M = a.cout; N = a.B * OHW; }
    else if (a.mode == 1) { M = a.cin; N = a.B * IHW; }
    else if (a.mode == 3) {
        M = a.cin;
        N = a.B * (int64_t)((a.IH - (a.par >> 1) + 1) / 2) * ((a.IW - (a.par & 1) + 1) / 2);
    } else { M = a.cout; N = (int64_t)a.cin * a.KH * a.KW; }
    // the kernel's index arithmetic divides in 32 bits (udiv32): pixels, columns, K indices and block ids < 2^31
    PCX_CHECK_ARG((int64_t)a.B * std::max(IHW, OHW) < ((int64_t)1 << 31) && N < ((int64_t)1 << 31) &&
                      (int64_t)std::max(a.cin, a.cout) * a.KH * a.KW < ((int64_t)1 << 31),
                  "convg: %lld x %lld problem exceeds 32-bit indexing", (long long)M, (long long)N);
    // narrow weight-gradient GEMMs (stem 7x7 of one channel: N = 49; 1x1 shortcuts of <= 64
    // channels) take 64-column tiles: a 128-column tile would multiply mostly padding
    const int wm = M >= 128 ? 2 : 1, wn = (a.mode == 2 && N <= 64 && (a.KH == 7 || a.KH == 1)) ? 1 : 2;
    const int64_t mt = ceil_div(M, 64 * wm), nt = ceil_div(N, 64 * wn);
    const int64_t nblocks = mt * nt * (a.mode == 2 ? a.nslice : 1);
    PCX_CHECK_ARG(nblocks < ((int64_t)1 << 31), "convg: grid too large");
    if (a.mode == 2) PCX_CHECK_ARG(a.kslice % KC == 0 && a.nslice >= 1, "convg: bad weight-gradient split");
    dim3 grid((unsigned)(8 * ((nblocks + 7) / 8)));  // (XCD-aware order inside the kernel)
    // tap-uniform K chunks: the K channel count (cin forward, cout data gradient) a multiple of 16
    // (mode 2 reuses the flag: false = dy computed as the BN backward of (bn_g, bn_y) while staging)
    const bool fk = a.mode == 2 ? a.bn_g == nullptr : (a.mode == 0 ? a.cin : a.cout) % KC == 0;
    if (a.mode != 2 && a.wpack) {
        const int64_t KK = (int64_t)a.KH * a.KW;
        int64_t K = a.mode == 0 ? a.cin * KK : a.cout * KK;
        if (a.mode == 3) {
            const int kh0 = ((a.par >> 1) + a.pad) & 1, kw0 = ((a.par & 1) + a.pad) & 1;
            K = (int64_t)a.cout * ((a.KH - kh0 + 1) / 2) * ((a.KW - kw0 + 1) / 2);
        }
        const int64_t Kp = (K + KC - 1) / KC * KC;
        if (M * Kp > 0)
            pack_wf32_kernel<<<(unsigned)ceil_div(M * Kp, 256), 256, 0, s>>>(a.w, static_cast<float*>(a.wpack), a.mode,
                                                                              a.cin, a.cout, a.KH, a.KW, a.par, a.pad,
                                                                              M, Kp, K);
        PCX_LAUNCH_CHECK("pack_wf32_kernel");
    }
    if (wn == 1) {
#define PCX_CG1(KH_, WM_)                                                                            \
        if (a.KH == KH_ && wm == WM_) {                                                              \
            if (fk) convg_kernel<2, KH_, KH_, WM_, 1, true><<<grid, 256, 0, s>>>(a);                 \
            else convg_kernel<2, KH_, KH_, WM_, 1, false><<<grid, 256, 0, s>>>(a);                   \
            PCX_LAUNCH_CHECK("convg_kernel");                                                        \
            return PCX_OK;                                                                           \
        }
        PCX_CG1(1, 1) PCX_CG1(1, 2) PCX_CG1(7, 1) PCX_CG1(7, 2)
#undef PCX_CG1
    }
#define PCX_CG(MODE_, KH_, WM_)                                                                      \
    if (a.mode == MODE_ && a.KH == KH_ && wm == WM_) {                                               \
        if (fk) convg_kernel<MODE_, KH_, KH_, WM_, 2, true><<<grid, 256, 0, s>>>(a);                 \
        else convg_kernel<MODE_, KH_, KH_, WM_, 2, false><<<grid, 256, 0, s>>>(a);                   \
        PCX_LAUNCH_CHECK("convg_kernel");                                                            \
        return PCX_OK;                                                                               \
    }
#define PCX_CG_K(KH_) PCX_CG(0, KH_, 1) PCX_CG(0, KH_, 2) PCX_CG(1, KH_, 1) PCX_CG(1, KH_, 2) \
                      PCX_CG(2, KH_, 1) PCX_CG(2, KH_, 2)
    PCX_CHECK_ARG(a.KH == a.KW, "convg: square kernels only");
    PCX_CG_K(1)
    PCX_CG_K(3)
    PCX_CG_K(7)
    PCX_CG(3, 1, 1) PCX_CG(3, 1, 2) PCX_CG(3, 3, 1) PCX_CG(3, 3, 2)
#undef PCX_CG_K
#undef PCX_CG
    set_error("convg: kernel size %d unsupported", a.KH);
    return PCX_EINVAL;
}

int chan_slices(int B, int C, int* bps) {
    // ~16384 blocks per launch: each block's run of planes is short enough that the launch is not one
    // long tail of latency-bound blocks (same-box B = 4096: deep fp32 125.2 -> 123.2 ms, bf16 51.0 ->
    // 50.2 against 2048, profiles/r4_chan_slices.txt; PCX_AB_CHAN_TARGET overrides)
    constexpr int target = PCX_AB_CHAN_TARGET < 256 ? 256 : PCX_AB_CHAN_TARGET;
    int want = std::max(1, std::min(B, target / std::max(C, 1)));
    *bps = ceil_div(B, want);
    return ceil_div(B, *bps);
}

int launch_chan_stats(const float* y, int B, int C, int64_t P, float* part0, float* part1, float* partn,
                      int* nslice, hipStream_t s) {
    int bps;
    const int ns = chan_slices(B, C, &bps);
    *nslice = ns;
    if (P % 4 == 0) chan_stats_kernel<4, 4><<<dim3(C, ns), 256, 0, s>>>(y, B, C, P, bps, part0, part1, partn);
    else chan_stats_kernel<1, 8><<<dim3(C, ns), 256, 0, s>>>(y, B, C, P, bps, part0, part1, partn);
    PCX_LAUNCH_CHECK("chan_stats_kernel");
    return PCX_OK;
}

int launch_bwd_prep(BwdPrepArgs a, int* nslice, hipStream_t s) {
    PCX_CHECK_ARG(a.mask_mode != MASK_OUT8 || a.mask8, "bwd_prep: MASK_OUT8 needs mask8");
    PCX_CHECK_ARG(a.dpar ? (a.H >= 1 && a.W >= 1 && (int64_t)a.H * a.W == a.P && a.P < (1 << 22) && !a.d2)
                         : a.d != nullptr,
                  "bwd_prep: bad upstream gradient arguments");
    const int ns = chan_slices(a.B, a.C, &a.bps);
    *nslice = ns;
    if (a.P % 4 == 0) bwd_prep_kernel<4, 2><<<dim3(a.C, ns), 256, 0, s>>>(a);
    else bwd_prep_kernel<1, 4><<<dim3(a.C, ns), 256, 0, s>>>(a);
    PCX_LAUNCH_CHECK("bwd_prep_kernel");
    return PCX_OK;
}

// short rows (flat form; PCX_AB_BN_ROWTILE: the row tiles)
static bool bn_flat(int64_t P, int64_t n, const void* a, const void* b, const void* c) {
    constexpr bool off = PCX_AB_BN_ROWTILE;
    auto al = [](const void* p) { return p == nullptr || ((uintptr_t)p & 15) == 0; };
    return !off && P < 1024 && n / P < ((int64_t)1 << 31) && al(a) && al(b) && al(c) && n > 0;
}

int launch_bn_act(const float* y, const float4* cf, const float* res, const float4* rcf, const float* drop,
                  float* out, int B, int C, int64_t P, hipStream_t s) {
    const int64_t n = (int64_t)B * C * P;
    if (bn_flat(P, n, y, res, out)) {
        const int64_t nb = std::min<int64_t>(ceil_div(n, 2048), (int64_t)1 << 20);
        bn_flat_kernel<0><<<(unsigned)nb, 256, 0, s>>>(y, cf, res, rcf, drop, nullptr, out, n, C, (int)P);
        PCX_LAUNCH_CHECK("bn_flat_kernel");
        return PCX_OK;
    }
    const int tp = row_threads(P);
    const int64_t rows = (int64_t)B * C;
    bn_act_kernel<<<ceil_div(rows, 256 / tp), 256, 0, s>>>(y, cf, res, rcf, drop, out, rows, C, P, tp);
    PCX_LAUNCH_CHECK("bn_act_kernel");
    return PCX_OK;
}

int launch_bn_bwd_apply(const float* g, const float* y, const float4* cf, float* dy, int B, int C, int64_t P,
                        hipStream_t s) {
    const int64_t n = (int64_t)B * C * P;
    if (bn_flat(P, n, g, y, dy)) {
        const int64_t nb = std::min<int64_t>(ceil_div(n, 2048), (int64_t)1 << 20);
        bn_flat_kernel<1><<<(unsigned)nb, 256, 0, s>>>(y, cf, nullptr, nullptr, nullptr, g, dy, n, C, (int)P);
        PCX_LAUNCH_CHECK("bn_flat_kernel");
        return PCX_OK;
    }
    const int tp = row_threads(P);
    const int64_t rows = (int64_t)B * C;
    bn_bwd_apply_kernel<<<ceil_div(rows, 256 / tp), 256, 0, s>>>(g, y, cf, dy, rows, C, P, tp);
    PCX_LAUNCH_CHECK("bn_bwd_apply_kernel");
    return PCX_OK;
}

int launch_maxpool3_fwd(const float* y, const float4* cf, float* out, uint8_t* arg, int B, int C, int H, int W,
                        int OH, int OW, hipStream_t s) {
    PCX_CHECK_ARG(OH == (H - 1) / 2 + 1 && OW == (W - 1) / 2 + 1, "maxpool3: output %dx%d for input %dx%d", OH, OW,
                  H, W);
    const int64_t rows = (int64_t)B * C;
    const size_t lds = (size_t)H * W * 4;
    if (lds <= 64 * 1024) {  // plane fits: LDS-staged form
        if ((H * W) % 4 == 0) maxpool3_fwd_lds_kernel<4><<<(unsigned)rows, 256, lds, s>>>(y, cf, out, arg, C, H, W, OH, OW);
        else maxpool3_fwd_lds_kernel<1><<<(unsigned)rows, 256, lds, s>>>(y, cf, out, arg, C, H, W, OH, OW);
        PCX_LAUNCH_CHECK("maxpool3_fwd_lds_kernel");
        return PCX_OK;
    }
    maxpool3_fwd_kernel<<<(unsigned)rows, 256, 0, s>>>(y, cf, out, arg, C, H, W, OH, OW);
    PCX_LAUNCH_CHECK("maxpool3_fwd_kernel");
    return PCX_OK;
}

bool maxpool3_bwd_prep_fits(int H, int W, int OH, int OW) {
    (void)H;
    (void)W;
    return (size_t)OH * OW * 9 <= 64 * 1024;
}

int launch_maxpool3_bwd_prep(const uint8_t* arg, const float* dout, const float* y, const float* ysel, const float4* cf,
                             float* g, float* p_g, float* p_x, int B, int C, int H, int W, int OH, int OW, int* nslice,
                             hipStream_t s, const float* dout2) {
    PCX_CHECK_ARG(OH == (H - 1) / 2 + 1 && OW == (W - 1) / 2 + 1, "maxpool3: output %dx%d for input %dx%d", OH, OW,
                  H, W);
    PCX_CHECK_ARG(maxpool3_bwd_prep_fits(H, W, OH, OW), "maxpool3_bwd_prep: %dx%d pooled plane exceeds LDS", OH, OW);
    PCX_CHECK_ARG(y || ysel, "maxpool3_bwd_prep: no BN input");
    int bps;
    const int ns = chan_slices(B, C, &bps);
    *nslice = ns;
    const size_t lds = ((size_t)OH * OW * (ysel ? 9 : 5) + 15) / 16 * 16;
#define PCX_MPB(V_, S_)                                                                                         \
    maxpool3_bwd_prep_kernel<V_, S_><<<dim3(C, ns), 256, lds, s>>>(arg, dout, dout2, S_ ? ysel : y, cf, g, p_g, p_x, B, C, \
                                                                   H, W, OH, OW, bps)
    if (W % 4 == 0) {
        if (ysel) PCX_MPB(4, true);
        else PCX_MPB(4, false);
    } else {
        if (ysel) PCX_MPB(1, true);
        else PCX_MPB(1, false);
    }
#undef PCX_MPB
    PCX_LAUNCH_CHECK("maxpool3_bwd_prep_kernel");
    return PCX_OK;
}

int launch_maxpool3_bwd(const uint8_t* arg, const float* dout, float* dz, int B, int C, int H, int W, int OH, int OW,
                        hipStream_t s) {
    const int64_t rows = (int64_t)B * C;
    maxpool3_bwd_kernel<<<(unsigned)rows, 256, 0, s>>>(arg, dout, dz, H, W, OH, OW);
    PCX_LAUNCH_CHECK("maxpool3_bwd_kernel");
    return PCX_OK;
}

int64_t par_off(int B, int C, int IH, int IW, int q) {
    int64_t off = 0;
    for (int k = 0; k < q; ++k)
        off += (int64_t)B * C * ((IH - (k >> 1) + 1) / 2) * ((IW - (k & 1) + 1) / 2);
    return off;
}

int launch_par_interleave(const float* src, float* dx, int B, int C, int IH, int IW, int accumulate, hipStream_t s) {
    const int64_t n = (int64_t)B * C * IH * IW;
    PCX_CHECK_ARG(n > 0 && n < ((int64_t)1 << 31), "par_interleave: %lld elements unsupported", (long long)n);
    const int64_t o1 = par_off(B, C, IH, IW, 1), o2 = par_off(B, C, IH, IW, 2), o3 = par_off(B, C, IH, IW, 3);
    if (IW % 4 == 0) {
        const unsigned total = (unsigned)(n / 4);
        par_interleave_kernel<4><<<ceil_div((int64_t)total, 256), 256, 0, s>>>(src, dx, total, IH, IW, accumulate, o1,
                                                                               o2, o3);
    } else if (IW % 2 == 0) {
        const unsigned total = (unsigned)(n / 2);
        par_interleave_kernel<2><<<ceil_div((int64_t)total, 256), 256, 0, s>>>(src, dx, total, IH, IW, accumulate, o1,
                                                                               o2, o3);
    } else {
        par_interleave_kernel<1><<<ceil_div(n, 256), 256, 0, s>>>(src, dx, (unsigned)n, IH, IW, accumulate, o1, o2,
                                                                   o3);
    }
    PCX_LAUNCH_CHECK("par_interleave_kernel");
    return PCX_OK;
}

int launch_fill_cf(float4* cf, int C, float4 v, hipStream_t s) {
    fill_cf_kernel<<<ceil_div(C, 256), 256, 0, s>>>(cf, C, v);
    PCX_LAUNCH_CHECK("fill_cf_kernel");
    return PCX_OK;
}

}  // namespace pcx
