// bf16-operand form of the general implicit-GEMM convolution (convg.hip), for PhonemeNetDeep with
// precision "bf16" (SURVEY 8(f) row 2): operands are rounded to bf16 (round-to-nearest-even) when
// they are staged into LDS and multiplied on v_mfma_f32_32x32x16_bf16 with float32 accumulation;
// activations, BN statistics, gradients and the optimizer stay float32 in HBM.
//
// Same GEMM views (modes 0 forward, 1 / 3 data gradient, 2 weight gradient), tap-major K order and
// deterministic epilogue as convg_kernel.  What changes is the staging: an MFMA lane consumes 8
// consecutive k of one row (A[m][8h .. 8h+7], B[8h .. 8h+7][n]), so every thread gathers whole
// k-runs of ONE row and writes them to LDS as one 16-byte store, rows stored k-contiguous (80-byte
// stride: conflict-free ds_read_b128).  K advances 32 per chunk (two MFMAs per tile, one barrier).
#include "kernels.h"

namespace pcx {
namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

constexpr int KB = 32;  // k per chunk
constexpr int RS = 40;  // LDS row stride in bf16 (32 k + 8 pad = 80 B)

struct Pix {  // (sample, row, column) of an output pixel index, advanced without division
    int64_t b;
    int oh = 0, ow = 0;
};

__device__ __forceinline__ void pix_step(Pix& p, int n, int OH, int OW) {
    p.ow += n;
    while (p.ow >= OW) {
        p.ow -= OW;
        if (++p.oh == OH) { p.oh = 0; ++p.b; }
    }
}

template <int N>
__device__ __forceinline__ void store_bf16(__bf16* dst, const float (&v)[N]) {
    static_assert(N % 4 == 0, "runs of 4 / 8 / 16");
#pragma unroll
    for (int q = 0; q < N / 8; ++q) {
        bf16x8 t;
#pragma unroll
        for (int j = 0; j < 8; ++j) t[j] = (__bf16)v[8 * q + j];
        *reinterpret_cast<bf16x8*>(dst + 8 * q) = t;
    }
    if constexpr (N % 8) {
        typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
        bf16x4 t;
#pragma unroll
        for (int j = 0; j < 4; ++j) t[j] = (__bf16)v[N - 4 + j];
        *reinterpret_cast<bf16x4*>(dst + N - 4) = t;
    }
}

// A operand of modes 0 / 1 / 3 packed once per launch: Wp[m][k] (bf16, tap-major k, rows padded
// with zeros to Kp = K rounded up to 32), so a thread's k-run is one or two 16-byte loads
__global__ __launch_bounds__(256) void pack_wbf16_kernel(const float* __restrict__ w, __bf16* __restrict__ wp,
                                                         int mode, int cin, int cout, int KH, int KW, int par,
                                                         int pad, int64_t M, int64_t Kp, int64_t K) {
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
    wp[i] = (__bf16)v;
}

template <int MODE, int KH, int KW, int WM, bool FK>
__global__ __launch_bounds__(256) void convg_bf16_kernel(ConvGArgs a) {
    constexpr int KK = KH * KW;
    constexpr int WN = 2;
    constexpr int BM = 64 * WM, BN = 64 * WN;
    constexpr int NA = KB * BM / 256, NB = KB * BN / 256;  // k per thread: 8 / 16, 16
    __shared__ __attribute__((aligned(16))) __bf16 As[2][BM][RS];
    __shared__ __attribute__((aligned(16))) __bf16 Bs[2][BN][RS];

    const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, l32 = lane & 31;
    const int wave = tid >> 6, wr = wave >> 1, wc = wave & 1;
    const int64_t OHW = (int64_t)a.OH * a.OW, IHW = (int64_t)a.IH * a.IW;
    const int s = a.stride, pad = a.pad;
    const int CK = MODE == 0 ? a.cin : a.cout;

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
    int64_t bid = blockIdx.x;
    const int64_t tq_ = udiv32(bid, mt), tm = bid - tq_ * mt;  // (32-bit index division: pcx_common.h)
    bid = tq_;
    const int64_t tr_ = udiv32(bid, nt), tn = bid - tr_ * nt;
    const int slice = (int)tr_;
    const int64_t m0 = tm * BM, n0 = tn * BN;
    int64_t k_begin = 0, k_end = K;
    if (MODE == 2) {
        k_begin = (int64_t)slice * a.kslice;
        k_end = min(K, k_begin + a.kslice);
    }
    const int nch = (int)((k_end - k_begin + KB - 1) / KB);

    // staging roles: A row am with k-run akg*NA.., B row bn with k-run bkg*NB..
    const int am = tid % BM, akg = tid / BM;
    const int bn = tid % BN, bkg = tid / BN;
    const int64_t arow = m0 + am, brow = n0 + bn;
    const bool avalid = arow < M, bvalid = brow < N;

    // modes 0/1/3: the B row is an output (or input-gradient) pixel
    int64_t xbase = 0;
    int ih0 = 0, iw0 = 0;
    if (MODE == 0 || MODE == 1 || MODE == 3) {
        const int64_t mm = bvalid ? brow : 0;
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
    // mode 2 (k-fast): a thread stages the pixel pair 2 kq2, 2 kq2 + 1 of each chunk for rows
    // rq + 16 j (A: output channels; B: (tap, input channel) columns), written as one bf16 pair
    constexpr int MA2 = BM / 16, MB2 = BN / 16;  // rows per thread
    const int kq2 = tid & 15, rq = tid >> 4;
    Pix p2{0, 0, 0};
    int boff[MODE == 2 ? MB2 : 1], bkhw[MODE == 2 ? MB2 : 1];
    if (MODE == 2) {
        const int64_t q = k_begin + 2 * kq2;
        p2.b = udiv32(q, OHW);
        const int64_t r = q - p2.b * OHW;
        p2.oh = (int)udiv32(r, a.OW);
        p2.ow = (int)(r - (int64_t)p2.oh * a.OW);
#pragma unroll
        for (int i = 0; i < MB2; ++i) {
            const int64_t jj = n0 + rq + 16 * i;
            const int tap = (int)udiv32(jj, a.cin), c = (int)(jj - (int64_t)tap * a.cin);
            const int kh = tap / KW - pad, kw = tap % KW - pad;
            boff[i] = (int)(c * IHW) + kh * a.IW + kw;
            // (kh, kw) for the bounds test; columns past N get kh far out of range (never load)
            bkhw[i] = jj < N ? ((kh + 16384) << 16) | (kw + 16384) : 0;
        }
    }

    float ra[NA], rb[NB];
    bf16x8 rap[NA / 8];
    const int64_t Kp = (K + KB - 1) / KB * KB;
    auto gather = [&](int chunk) {
        const int64_t kbase = k_begin + (int64_t)chunk * KB;
        if (MODE == 0 || MODE == 1 || MODE == 3) {
            // ---- A: weights of row m = arow, k-run kbase + akg*NA + j
            const int64_t k0 = kbase + akg * NA;
            if (a.wpack) {  // packed bf16 rows: the run is NA / 8 aligned 16-byte loads
                const bf16x8* src = reinterpret_cast<const bf16x8*>(static_cast<const __bf16*>(a.wpack) + arow * Kp + k0);
#pragma unroll
                for (int q = 0; q < NA / 8; ++q) rap[q] = avalid ? src[q] : bf16x8{};
            } else if (FK) {
                const int tap = (int)udiv32(kbase, CK), ch0 = (int)(k0 - (int64_t)tap * CK);
                const float* wp;
                int64_t wst;
                if (MODE == 0) { wp = a.w + (arow * a.cin + ch0) * KK + tap; wst = KK; }
                else if (MODE == 1) { wp = a.w + ((int64_t)ch0 * a.cin + arow) * KK + tap; wst = (int64_t)a.cin * KK; }
                else {
                    wp = a.w + (((int64_t)ch0 * a.cin + arow) * KH + kh0 + 2 * (tap / ntw)) * KW + kw0 + 2 * (tap % ntw);
                    wst = (int64_t)a.cin * KK;
                }
#pragma unroll
                for (int j = 0; j < NA; ++j) ra[j] = avalid ? wp[j * wst] : 0.f;
            } else {
#pragma unroll
                for (int j = 0; j < NA; ++j) {
                    const int64_t k = k0 + j;
                    float v = 0.f;
                    if (avalid && k < K) {
                        const int tap = (int)udiv32(k, CK), ch = (int)(k - (int64_t)tap * CK);
                        if (MODE == 0) v = a.w[(arow * a.cin + ch) * KK + tap];
                        else if (MODE == 1) v = a.w[((int64_t)ch * a.cin + arow) * KK + tap];
                        else
                            v = a.w[(((int64_t)ch * a.cin + arow) * KH + kh0 + 2 * (tap / ntw)) * KW + kw0 +
                                    2 * (tap % ntw)];
                    }
                    ra[j] = v;
                }
            }
            // ---- B: activations (mode 0) / output gradients (modes 1, 3) of pixel brow
            const int64_t kb0 = kbase + bkg * NB;
            if (FK) {
                const int tap = (int)udiv32(kbase, CK), c0 = (int)(kb0 - (int64_t)tap * CK);
                int ih, iw;
                bool ok;
                const float* src;
                int64_t cst;
                if (MODE == 0) {
                    ih = ih0 + tap / KW;
                    iw = iw0 + tap % KW;
                    ok = bvalid && ih >= 0 && ih < a.IH && iw >= 0 && iw < a.IW;
                    src = a.x + xbase + (int64_t)c0 * IHW + (int64_t)ih * a.IW + iw;
                    cst = IHW;
                } else {
                    int oh = 0, ow = 0;
                    if (MODE == 3) {
                        oh = (ih0 - (kh0 + 2 * (tap / ntw))) >> 1;
                        ow = (iw0 - (kw0 + 2 * (tap % ntw))) >> 1;
                        ok = true;
                    } else {
                        const int th = ih0 - tap / KW, tw = iw0 - tap % KW;
                        ok = th >= 0 && tw >= 0;
                        oh = th;
                        ow = tw;
                        if (s == 2) {
                            ok = ok && ((th | tw) & 1) == 0;
                            oh = th >> 1;
                            ow = tw >> 1;
                        }
                    }
                    ok = ok && bvalid && oh >= 0 && ow >= 0 && oh < a.OH && ow < a.OW;
                    src = a.dy + xbase + (int64_t)c0 * OHW + (int64_t)oh * a.OW + ow;
                    cst = OHW;
                }
#pragma unroll
                for (int i = 0; i < NB; ++i) rb[i] = ok ? src[i * cst] : 0.f;
            } else {
#pragma unroll
                for (int i = 0; i < NB; ++i) {
                    const int64_t k = kb0 + i;
                    float v = 0.f;
                    if (bvalid && k < K) {
                        const int tap = (int)udiv32(k, CK), ch = (int)(k - (int64_t)tap * CK);
                        if (MODE == 0) {
                            const int ih = ih0 + tap / KW, iw = iw0 + tap % KW;
                            if (ih >= 0 && ih < a.IH && iw >= 0 && iw < a.IW)
                                v = a.x[xbase + (int64_t)ch * IHW + (int64_t)ih * a.IW + iw];
                        } else {
                            int oh = 0, ow = 0;
                            bool ok;
                            if (MODE == 3) {
                                oh = (ih0 - (kh0 + 2 * (tap / ntw))) >> 1;
                                ow = (iw0 - (kw0 + 2 * (tap % ntw))) >> 1;
                                ok = true;
                            } else {
                                const int th = ih0 - tap / KW, tw = iw0 - tap % KW;
                                ok = th >= 0 && tw >= 0;
                                oh = th;
                                ow = tw;
                                if (s == 2) {
                                    ok = ok && ((th | tw) & 1) == 0;
                                    oh = th >> 1;
                                    ow = tw >> 1;
                                }
                            }
                            if (ok && oh >= 0 && ow >= 0 && oh < a.OH && ow < a.OW)
                                v = a.dy[xbase + (int64_t)ch * OHW + (int64_t)oh * a.OW + ow];
                        }
                    }
                    rb[i] = v;
                }
            }
        } else {
            // ---- mode 2: A = dy[b][n][pixel], B = x[b][c][pixel*s + tap] for the thread's pixel pair
            Pix q1 = p2;
            pix_step(q1, 1, a.OH, a.OW);
            const int64_t kq = kbase + 2 * kq2;
            const bool v0 = kq < k_end, v1 = kq + 1 < k_end;
            const int64_t pofs0 = (int64_t)p2.oh * a.OW + p2.ow, pofs1 = (int64_t)q1.oh * a.OW + q1.ow;
            const float* dy0 = a.dy + p2.b * a.cout * OHW + pofs0;
            const float* dy1 = a.dy + q1.b * a.cout * OHW + pofs1;
#pragma unroll
            for (int j = 0; j < MA2; ++j) {
                const int64_t n = m0 + rq + 16 * j;
                const bool nv = n < M;
                if (!FK) {  // mode 2: FK = false selects dy = BN backward of (g, y), computed here
                    const float4 kc = a.bn_cf[nv ? n : 0];
                    const int64_t o0 = p2.b * a.cout * OHW + pofs0 + n * OHW, o1 = q1.b * a.cout * OHW + pofs1 + n * OHW;
                    ra[2 * j] = (nv && v0) ? kc.x * (a.bn_g[o0] - kc.y - (a.bn_y[o0] - kc.w) * kc.z) : 0.f;
                    ra[2 * j + 1] = (nv && v1) ? kc.x * (a.bn_g[o1] - kc.y - (a.bn_y[o1] - kc.w) * kc.z) : 0.f;
                } else {
                    ra[2 * j] = (nv && v0) ? dy0[n * OHW] : 0.f;
                    ra[2 * j + 1] = (nv && v1) ? dy1[n * OHW] : 0.f;
                }
            }
            const float* x0 = a.x + p2.b * a.cin * IHW + (int64_t)p2.oh * s * a.IW + p2.ow * s;
            const float* x1 = a.x + q1.b * a.cin * IHW + (int64_t)q1.oh * s * a.IW + q1.ow * s;
            const int ih0b = p2.oh * s, iw0b = p2.ow * s, ih1b = q1.oh * s, iw1b = q1.ow * s;
#pragma unroll
            for (int i = 0; i < MB2; ++i) {
                const int kh = (bkhw[i] >> 16) - 16384, kw = (bkhw[i] & 0xffff) - 16384;
                const bool ok0 = v0 && ih0b + kh >= 0 && ih0b + kh < a.IH && iw0b + kw >= 0 && iw0b + kw < a.IW;
                const bool ok1 = v1 && ih1b + kh >= 0 && ih1b + kh < a.IH && iw1b + kw >= 0 && iw1b + kw < a.IW;
                rb[2 * i] = ok0 ? x0[boff[i]] : 0.f;
                rb[2 * i + 1] = ok1 ? x1[boff[i]] : 0.f;
            }
            pix_step(p2, KB, a.OH, a.OW);
        }
    };
    auto stash = [&](int buf) {
        if (MODE == 2) {
            typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
#pragma unroll
            for (int j = 0; j < MA2; ++j)
                *reinterpret_cast<bf16x2*>(&As[buf][rq + 16 * j][2 * kq2]) = bf16x2{(__bf16)ra[2 * j], (__bf16)ra[2 * j + 1]};
#pragma unroll
            for (int i = 0; i < MB2; ++i)
                *reinterpret_cast<bf16x2*>(&Bs[buf][rq + 16 * i][2 * kq2]) = bf16x2{(__bf16)rb[2 * i], (__bf16)rb[2 * i + 1]};
        } else {
            if (a.wpack) {
#pragma unroll
                for (int q = 0; q < NA / 8; ++q) *reinterpret_cast<bf16x8*>(&As[buf][am][akg * NA + 8 * q]) = rap[q];
            } else {
                store_bf16<NA>(&As[buf][am][akg * NA], ra);
            }
            store_bf16<NB>(&Bs[buf][bn][bkg * NB], rb);
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
        for (int ks = 0; ks < KB / 16; ++ks) {
            bf16x8 av[WM], bv[WN];
#pragma unroll
            for (int mi = 0; mi < WM; ++mi)
                av[mi] = *reinterpret_cast<const bf16x8*>(&As[buf][wr * 32 * WM + mi * 32 + l32][16 * ks + 8 * h]);
#pragma unroll
            for (int ni = 0; ni < WN; ++ni)
                bv[ni] = *reinterpret_cast<const bf16x8*>(&Bs[buf][wc * 32 * WN + ni * 32 + l32][16 * ks + 8 * h]);
#pragma unroll
            for (int mi = 0; mi < WM; ++mi)
#pragma unroll
                for (int ni = 0; ni < WN; ++ni)
                    acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[mi], bv[ni], acc[mi][ni], 0, 0, 0);
        }
        if (ch + 1 < nch) stash(buf ^ 1);
        __syncthreads();
    }

    // ---- epilogue (as convg_kernel)
#pragma unroll
    for (int ni = 0; ni < WN; ++ni) {
        const int64_t col = n0 + wc * 32 * WN + ni * 32 + l32;
        if (col >= N) continue;
        int64_t obase, ostride;
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
            const int ihc = (int)udiv32(p, IWc), iwc = (int)(p - (int64_t)ihc * IWc);
            obase = b * a.cin * IHW + (int64_t)(2 * ihc + ph) * a.IW + 2 * iwc + pw;
            ostride = IHW;
        } else {
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
                    float* o = a.out + obase + row * ostride;
                    if ((MODE == 1 || MODE == 3) && a.accumulate) *o += acc[mi][ni][r];
                    else *o = acc[mi][ni][r];
                }
            }
    }
}

}  // namespace

int launch_convg_bf16(ConvGArgs a, hipStream_t s) {
    const int64_t IHW = (int64_t)a.IH * a.IW, OHW = (int64_t)a.OH * a.OW;
    int64_t M, N;
    if (a.mode == 0) { M = a.cout; N = a.B * OHW; }
    else if (a.mode == 1) { M = a.cin; N = a.B * IHW; }
    else if (a.mode == 3) {
        M = a.cin;
        N = a.B * (int64_t)((a.IH - (a.par >> 1) + 1) / 2) * ((a.IW - (a.par & 1) + 1) / 2);
    } else { M = a.cout; N = (int64_t)a.cin * a.KH * a.KW; }
    const int wm = M >= 128 ? 2 : 1;
    const int64_t mt = ceil_div(M, 64 * wm), nt = ceil_div(N, 128);
    const int64_t nblocks = mt * nt * (a.mode == 2 ? a.nslice : 1);
    PCX_CHECK_ARG(nblocks < ((int64_t)1 << 31), "convg_bf16: grid too large");
    // (32-bit index divisions in the kernel: udiv32)
    PCX_CHECK_ARG((int64_t)a.B * std::max(IHW, OHW) < ((int64_t)1 << 31) && N < ((int64_t)1 << 31) &&
                      (int64_t)std::max(a.cin, a.cout) * a.KH * a.KW < ((int64_t)1 << 31),
                  "convg_bf16: %lld x %lld problem exceeds 32-bit indexing", (long long)M, (long long)N);
    if (a.mode == 2) PCX_CHECK_ARG(a.kslice % KB == 0 && a.nslice >= 1, "convg_bf16: bad weight-gradient split");
    // (mode 2 reuses the flag: false = dy computed as the BN backward of (bn_g, bn_y) while staging)
    const bool fk = a.mode == 2 ? a.bn_g == nullptr : (a.mode == 0 ? a.cin : a.cout) % KB == 0;
    // channel-last operands supplied: the convn.hip engine (packs its own weight rows)
    if (a.mode == 2 ? (a.xn && a.dyn) : a.mode == 0 ? a.xn != nullptr : a.dyn != nullptr) return launch_convn(a, s);
    if (a.mode != 2 && a.wpack) {
        const int64_t KK = (int64_t)a.KH * a.KW;
        int64_t K = a.mode == 0 ? a.cin * KK : a.cout * KK;
        if (a.mode == 3) {
            const int kh0 = ((a.par >> 1) + a.pad) & 1, kw0 = ((a.par & 1) + a.pad) & 1;
            K = (int64_t)a.cout * ((a.KH - kh0 + 1) / 2) * ((a.KW - kw0 + 1) / 2);
        }
        const int64_t Kp = (K + KB - 1) / KB * KB;
        if (M * Kp > 0)  // (a 1x1 stride-2 class without taps has K = 0: zero output, nothing to pack)
            pack_wbf16_kernel<<<(unsigned)ceil_div(M * Kp, 256), 256, 0, s>>>(a.w, static_cast<__bf16*>(a.wpack), a.mode,
                                                                           a.cin, a.cout, a.KH, a.KW, a.par, a.pad, M,
                                                                           Kp, K);
        PCX_LAUNCH_CHECK("pack_wbf16_kernel");
    }
    dim3 grid((unsigned)nblocks);
#define PCX_CB(MODE_, KH_, WM_)                                                                 \
    if (a.mode == MODE_ && a.KH == KH_ && wm == WM_) {                                          \
        if (fk) convg_bf16_kernel<MODE_, KH_, KH_, WM_, true><<<grid, 256, 0, s>>>(a);          \
        else convg_bf16_kernel<MODE_, KH_, KH_, WM_, false><<<grid, 256, 0, s>>>(a);            \
        PCX_LAUNCH_CHECK("convg_bf16_kernel");                                                  \
        return PCX_OK;                                                                          \
    }
#define PCX_CB_K(KH_) PCX_CB(0, KH_, 1) PCX_CB(0, KH_, 2) PCX_CB(1, KH_, 1) PCX_CB(1, KH_, 2) \
                      PCX_CB(2, KH_, 1) PCX_CB(2, KH_, 2)
    PCX_CB_K(1)
    PCX_CB_K(3)
    PCX_CB_K(7)
    PCX_CB(3, 1, 1) PCX_CB(3, 1, 2) PCX_CB(3, 3, 1) PCX_CB(3, 3, 2)
#undef PCX_CB_K
#undef PCX_CB
    set_error("convg_bf16: kernel size %d unsupported", a.KH);
    return PCX_EINVAL;
}

}  // namespace pcx

namespace pcx {
size_t convg_bf16_wpack_bytes(int mode, int cin, int cout, int k) {
    if (mode == 2) return 0;
    const int64_t M = mode == 0 ? cout : cin, K = (int64_t)(mode == 0 ? cin : cout) * k * k;
    return (size_t)M * ((K + KB - 1) / KB * KB) * 2;
}
}  // namespace pcx

// ---------------------------------------------------------------------------------------------
// The cnn_deep convolution engine as a standalone operation (include/pcx.h: pcx_conv2d): used by
// the kernel-level parity tests of both precisions and by micro-benchmarks.
namespace {
// channel-last scratch of the bf16 engine (convn.hip) behind pcx_conv2d: x image, dy image
struct Conv2dNhwc {
    bool on;
    size_t xb, dyb;
};
Conv2dNhwc conv2d_nhwc(int mode, int precision, int B, int cin, int cout, int IH, int IW, int OH, int OW, int k,
                       int pad) {
    pcx::ConvGArgs a{};
    a.mode = mode; a.cin = cin; a.cout = cout; a.KH = a.KW = k; a.pad = pad;
    Conv2dNhwc r{false, 0, 0};
    if (!precision || !pcx::convn_fits(a)) return r;
    r.on = true;
    if (mode != 1) r.xb = (pcx::nhwc_bytes(B, cin, IH, IW) + 255) / 256 * 256;
    if (mode != 0) r.dyb = (pcx::nhwc_bytes(B, cout, OH, OW) + 255) / 256 * 256;
    return r;
}
// fp32 stride-1 3x3 forward / data gradient with rows >= 31 columns: the Winograd conv (conv_wino.hip),
// as in the networks; workspace = transformed weights + the forward's statistics partials
bool conv2d_wino(int mode, int precision, int B, int cin, int cout, int IH, int IW, int k, int stride, int pad) {
    if (precision || mode == 2 || k != 3 || stride != 1 || pad != 1) return false;
    return mode == 0 ? pcx::wino_geometry(B, IH, IW, cin, cout, nullptr) : pcx::wino_geometry(B, IH, IW, cout, cin, nullptr);
}
size_t conv2d_wino_bytes(int B, int cin, int cout, int H, int W) {
    const size_t nblk = pcx::wino_nblk(B, H, W, cin, cout);
    return ((size_t)16 * cin * cout * 4 + 255) / 256 * 256 + ((2 * (size_t)std::max(cin, cout) + 1) * nblk * 4 + 255) / 256 * 256;
}
size_t conv2d_base_bytes(int mode, int precision, int B, int cin, int cout, int OH, int OW, int k) {
    if (mode != 2 && conv2d_wino(mode, precision, B, cin, cout, OH, OW, k, 1, 1))
        return std::max(conv2d_wino_bytes(B, cin, cout, OH, OW),
                        (pcx::convg_wpack_bytes(mode, cin, cout, k) + 255) / 256 * 256);
    if (mode != 2)
        return ((precision ? pcx::convg_bf16_wpack_bytes(mode, cin, cout, k) : pcx::convg_wpack_bytes(mode, cin, cout, k)) +
                255) / 256 * 256;
    pcx::ConvGArgs a{};
    a.B = B; a.cin = cin; a.cout = cout; a.OH = OH; a.OW = OW; a.KH = a.KW = k;
    int64_t ks;
    const int ns = pcx::convg_nslice(a, &ks);
    return ((size_t)ns * cout * cin * k * k * 4 + 255) / 256 * 256;
}
}  // namespace

// (the input resolution is implied: the bf16 channel-last scratch is sized for stride 1, the larger)
extern "C" size_t pcx_conv2d_workspace_bytes(int mode, int precision, int B, int cin, int cout, int OH, int OW,
                                             int k) {
    const size_t base = conv2d_base_bytes(mode, precision, B, cin, cout, OH, OW, k);
    if (!precision) return base;
    // upper bound of the input image over strides 1 and 2: IH <= 2 OH + k, IW <= 2 OW + k
    const Conv2dNhwc n = conv2d_nhwc(mode, precision, B, cin, cout, 2 * OH + k, 2 * OW + k, OH, OW, k, 1);
    return base + n.xb + n.dyb;
}

extern "C" int pcx_conv2d(int mode, int precision, int B, int cin, int cout, int IH, int IW, int OH, int OW, int k,
                          int stride, int pad, const float* x, const float* w, const float* dy, float* out,
                          int accumulate, void* ws, size_t ws_bytes, hipStream_t stream) {
    using namespace pcx;
    PCX_CHECK_ARG(mode >= 0 && mode <= 2, "pcx_conv2d: mode %d (0 forward, 1 data gradient, 2 weight gradient)", mode);
    PCX_CHECK_ARG(precision == 0 || precision == 1, "pcx_conv2d: precision %d (0 fp32, 1 bf16)", precision);
    PCX_CHECK_ARG(B > 0 && cin > 0 && cout > 0 && k > 0 && IH > 0 && IW > 0, "pcx_conv2d: empty shape");
    PCX_CHECK_ARG(OH == (IH + 2 * pad - k) / stride + 1 && OW == (IW + 2 * pad - k) / stride + 1,
                  "pcx_conv2d: output %dx%d inconsistent with input %dx%d, k %d, stride %d, pad %d", OH, OW, IH, IW,
                  k, stride, pad);
    PCX_CHECK_ARG(out && (mode == 2 ? (x && dy) : mode == 1 ? (w && dy) : (x && w)), "pcx_conv2d: NULL operand");
    if (conv2d_wino(mode, precision, B, cin, cout, IH, IW, k, stride, pad)) {
        const size_t need = conv2d_wino_bytes(B, cin, cout, IH, IW);
        PCX_CHECK_ARG(ws && ws_bytes >= need, "pcx_conv2d: needs %zu workspace bytes, got %zu", need, ws_bytes);
        float* u = static_cast<float*>(ws);
        float* part = u + ((size_t)16 * cin * cout * 4 + 255) / 256 * 64;
        ConvArgs c{};
        c.B = B; c.H = IH; c.W = IW;
        c.cin = mode == 0 ? cin : cout;
        c.cout = mode == 0 ? cout : cin;
        c.src = mode == 0 ? x : dy;
        c.srcH = IH; c.srcW = IW;
        c.wpack = u;
        c.out = out;
        c.accumulate = accumulate;
        c.nblk = (int)wino_nblk(B, IH, IW, c.cin, c.cout);
        c.part0 = part;
        c.part1 = part + (size_t)c.cout * c.nblk;
        c.partn = part + (size_t)2 * c.cout * c.nblk;
        const int rc = launch_wino_pack(w, u, c.cout, c.cin, mode, stream);
        if (rc != PCX_OK) return rc;
        return launch_conv3x3_wino(PRO_RAW, mode == 0 ? EPI_FWD : EPI_BWD_STORE, c, stream);
    }
    ConvGArgs a{};
    a.mode = mode;
    a.B = B; a.cin = cin; a.cout = cout;
    a.IH = IH; a.IW = IW; a.OH = OH; a.OW = OW;
    a.KH = a.KW = k; a.stride = stride; a.pad = pad;
    a.x = x; a.w = w; a.dy = dy; a.out = out;
    a.accumulate = accumulate;
    a.bf16 = precision;
    const size_t base = conv2d_base_bytes(mode, precision, B, cin, cout, OH, OW, k);
    const Conv2dNhwc n = conv2d_nhwc(mode, precision, B, cin, cout, IH, IW, OH, OW, k, pad);
    const size_t need = base + n.xb + n.dyb;
    PCX_CHECK_ARG(need == 0 || (ws && ws_bytes >= need), "pcx_conv2d: needs %zu workspace bytes, got %zu", need,
                  ws_bytes);
    if (n.on) {  // channel-last bf16 operands for convn.hip
        char* nb = static_cast<char*>(ws) + base;
        if (n.xb) {
            NhwcArgs t{};
            t.op = NHWC_COPY; t.B = B; t.C = cin; t.H = IH; t.W = IW; t.src = x; t.dst = nb;
            const int rc = launch_to_nhwc(t, stream);
            if (rc != PCX_OK) return rc;
            a.xn = nb;
        }
        if (n.dyb) {
            NhwcArgs t{};
            t.op = NHWC_COPY; t.B = B; t.C = cout; t.H = OH; t.W = OW; t.src = dy; t.dst = nb + n.xb;
            const int rc = launch_to_nhwc(t, stream);
            if (rc != PCX_OK) return rc;
            a.dyn = nb + n.xb;
        }
    }
    if (mode != 2) {
        a.wpack = ws;
        return launch_convg(a, stream);
    }
    a.nslice = convg_nslice(a, &a.kslice);
    a.out = static_cast<float*>(ws);
    const int rc = launch_convg(a, stream);
    if (rc != PCX_OK) return rc;
    return launch_sum_slices(a.out, a.nslice, (int64_t)cout * cin * k * k, out, stream);
}
