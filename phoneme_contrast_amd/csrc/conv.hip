// Direct (non-GEMM) kernels of the cnn_small trunk on CDNA4 (gfx950), fp32 throughout.
//
//  * conv1_fwd_kernel — the Cin = 1 first conv (reference src/models/phoneme_cnn.py:36): direct,
//                       HBM-write-bound, with the BN statistics of its output in the epilogue.
//  * wgrad1_kernel    — its weight gradient (the 3x3 implicit-GEMM convs live in conv_dma.hip,
//                       their weight gradients in wgrad_s.hip / wgrad_w32.hip).
//  * sum_slices / pack kernels — deterministic slice reduction and GEMM weight layouts.
//
// Tensor layout is the reference's planar NCHW.
#include "conv_epilogue.h"

namespace pcx {
namespace {

void tile_shape(int cout, int* wm, int* wn) {
    if (cout == 32) { *wm = 1; *wn = 4; }
    else { *wm = 2; *wn = 2; }
}

typedef const __attribute__((address_space(4))) float* cfloat4p;  // constant space: scalar loads

// ------------------------------------------------------------------ Cin = 1 first conv
constexpr int C1W_CPW = 8;  // output channels per wave (register weight gradient)
constexpr int C1F_CPW = 8;  // output channels per wave (forward)
#ifndef PCX_AB_C1_NT
#define PCX_AB_C1_NT 1      // nontemporal y1 stores (same-box A/B: 0.917 -> 0.879 ms; 0: plain stores)
#endif

// 3 x 6 input window of a pixel quad (columns w0 - 1 .. w0 + 4, rows hh - 1 .. hh + 1), zero outside
// the sample.  FULL: W % 4 == 0 (16-byte row quads; no partial quad)
template <bool FULL>
__device__ __forceinline__ void c1_window(const float* xb, int H, int W, int hh, int w0, float (&xr)[3][6]) {
#pragma unroll
    for (int dh = 0; dh < 3; ++dh) {
        const int y = hh + dh - 1;
        if (y < 0 || y >= H) {
#pragma unroll
            for (int e = 0; e < 6; ++e) xr[dh][e] = 0.f;
            continue;
        }
        const float* row = xb + (int64_t)y * W;
        if (FULL) {
            const float4 v = ld4(row + w0);
            xr[dh][1] = v.x; xr[dh][2] = v.y; xr[dh][3] = v.z; xr[dh][4] = v.w;
        } else {
#pragma unroll
            for (int e = 0; e < 4; ++e) xr[dh][1 + e] = w0 + e < W ? row[w0 + e] : 0.f;
        }
        xr[dh][0] = w0 > 0 ? row[w0 - 1] : 0.f;
        xr[dh][5] = w0 + 4 < W ? row[w0 + 4] : 0.f;
    }
}

// The same window with every load unconditional (row / column clamped into the sample, the value
// zeroed afterwards): a straight-line load group the compiler can issue ahead of the previous quad's
// stores.  W % 4 == 0.
__device__ __forceinline__ void c1_window_ld(const float* xb, int H, int W, int hh, int w0, float (&xr)[3][6]) {
#pragma unroll
    for (int dh = 0; dh < 3; ++dh) {
        const int y = hh + dh - 1;
        const int yc = min(max(y, 0), H - 1);
        const float* row = xb + (int64_t)yc * W;
        const float4 v = ld4(row + w0);
        const float l = row[max(w0 - 1, 0)], r = row[min(w0 + 4, W - 1)];
        const bool ok = y == yc;
        xr[dh][1] = ok ? v.x : 0.f;
        xr[dh][2] = ok ? v.y : 0.f;
        xr[dh][3] = ok ? v.z : 0.f;
        xr[dh][4] = ok ? v.w : 0.f;
        xr[dh][0] = ok && w0 > 0 ? l : 0.f;
        xr[dh][5] = ok && w0 + 4 < W ? r : 0.f;
    }
}

// A block owns rows_per_blk consecutive (sample, row) image rows; wave w computes output channels
// 8w .. 8w + 7 (+ 32k) for every pixel quad of those rows: lanes take consecutive quads (1 KB per
// store instruction), the 3 x 6 input window comes from L1/L2 (the input is 1/32 of the output).
// HBM-write-bound (the output is 32x the input).  BN partial statistics per (channel, block) as
// {sum, M2 about the block's first output} (shifted one-pass form).
template <bool FULL>
__global__ __launch_bounds__(256) void conv1_fwd_kernel(Conv1Args a) {
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int HW = a.H * a.W;
    const int nrows = a.B * a.H;
    const int r0 = blockIdx.x * a.rows_per_blk;
    const int r1 = min(nrows, r0 + a.rows_per_blk);
    const int nq = (a.W + 3) >> 2;
    const int ntask = (r1 - r0) * nq;
    for (int cg = wave * C1F_CPW; cg < a.cout; cg += 4 * C1F_CPW) {
        float wt[C1F_CPW][9];
#pragma unroll
        for (int j = 0; j < C1F_CPW; ++j)
#pragma unroll
            for (int t = 0; t < 9; ++t) wt[j][t] = a.w[(cg + j) * 9 + t];
        // shift for the one-pass variance: the output at the block's first pixel
        float K[C1F_CPW];
        {
            const int b = r0 / a.H, hh = r0 - b * a.H;
            float xr[3][6];
            c1_window<false>(a.x + (int64_t)b * HW, a.H, a.W, hh, 0, xr);
#pragma unroll
            for (int j = 0; j < C1F_CPW; ++j) {
                float v = 0.f;
#pragma unroll
                for (int t = 0; t < 9; ++t) v = fmaf(wt[j][t], xr[t / 3][1 + t % 3 - 1], v);
                K[j] = v;
            }
        }
        float s1[C1F_CPW], s2[C1F_CPW];
#pragma unroll
        for (int j = 0; j < C1F_CPW; ++j) s1[j] = s2[j] = 0.f;
        // FULL: the next quad's window is loaded before this quad's stores are issued, so waiting for
        // it never waits for the stores (vmcnt counts both, in issue order)
        float xn[3][6];
        auto locate = [&](int t, int& b, int& hh, int& w0) {
            const int rr = t / nq, q = t - rr * nq;
            const int gr = r0 + rr;
            b = gr / a.H;
            hh = gr - b * a.H;
            w0 = 4 * q;
        };
        if (FULL && lane < ntask) {
            int b, hh, w0;
            locate(lane, b, hh, w0);
            c1_window_ld(a.x + (int64_t)b * HW, a.H, a.W, hh, w0, xn);
        }
        for (int t = lane; t < ntask; t += 64) {
            int b, hh, w0;
            locate(t, b, hh, w0);
            float xr[3][6];
            if (FULL) {
#pragma unroll
                for (int i = 0; i < 3; ++i)
#pragma unroll
                    for (int e = 0; e < 6; ++e) xr[i][e] = xn[i][e];
                int bn, hn, wn;  // (unconditional: the last quad's prefetch repeats a valid one)
                locate(min(t + 64, ntask - 1), bn, hn, wn);
                c1_window_ld(a.x + (int64_t)bn * HW, a.H, a.W, hn, wn, xn);
            } else {
                c1_window<FULL>(a.x + (int64_t)b * HW, a.H, a.W, hh, w0, xr);
            }
            float* ob = a.out + ((int64_t)b * a.cout + cg) * HW + (int64_t)hh * a.W + w0;
#pragma unroll
            for (int j = 0; j < C1F_CPW; ++j) {
                float v[4];
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    float acc = 0.f;
#pragma unroll
                    for (int tp = 0; tp < 9; ++tp) acc = fmaf(wt[j][tp], xr[tp / 3][e + tp % 3], acc);
                    v[e] = acc;
                }
                if (FULL) {
                    if constexpr (PCX_AB_C1_NT) {
                        typedef float nf4 __attribute__((ext_vector_type(4)));
                        __builtin_nontemporal_store(nf4{v[0], v[1], v[2], v[3]}, reinterpret_cast<nf4*>(ob + (int64_t)j * HW));
                    } else {
                        st4(ob + (int64_t)j * HW, make_float4(v[0], v[1], v[2], v[3]));
                    }
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        const float d = v[e] - K[j];
                        s1[j] += d;
                        s2[j] = fmaf(d, d, s2[j]);
                    }
                } else {
#pragma unroll
                    for (int e = 0; e < 4; ++e)
                        if (w0 + e < a.W) {
                            ob[(int64_t)j * HW + e] = v[e];
                            const float d = v[e] - K[j];
                            s1[j] += d;
                            s2[j] = fmaf(d, d, s2[j]);
                        }
                }
            }
        }
        const float n = (float)((r1 - r0) * a.W);
#pragma unroll
        for (int j = 0; j < C1F_CPW; ++j) {
            float t1 = wave_sum(s1[j]), t2 = wave_sum(s2[j]);
            if (lane == 0) {
                a.part0[(int64_t)(cg + j) * a.nblk + blockIdx.x] = n * K[j] + t1;
                a.part1[(int64_t)(cg + j) * a.nblk + blockIdx.x] = fmaxf(t2 - t1 * t1 / n, 0.f);
            }
        }
        if (lane == 0 && cg == 0) a.partn[blockIdx.x] = n;
    }
}

// ------------------------------------------------------------------ weight gradient, Cin = 1
// dW[n][tap] = sum dy[n] x(shifted), dy = BN backward of (dz, y).  Same quad walk as the forward:
// wave w owns channels 8w .. 8w + 7 (+ 32k), lanes consecutive pixel quads (16-byte dz / y loads);
// HBM-read-bound.  Partials per slice.  RC (round 4): y is not read but recomputed from the input
// window the gradient needs anyway, with conv1_fwd_kernel's weights and FMA order (the same float
// bits): 9 FMAs per output instead of 4 bytes of HBM -- dz alone is streamed (4.2 instead of 8.4 GB
// per B = 4096 step).
template <bool FULL, bool RC>
__global__ __launch_bounds__(256) void wgrad1_kernel(Wgrad1Args a) {
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int HW = a.H * a.W;
    const int nrows = a.B * a.H;
    const int r0 = blockIdx.x * a.rows_per_slice;
    const int r1 = min(nrows, r0 + a.rows_per_slice);
    const int nq = (a.W + 3) >> 2;
    const int ntask = (r1 - r0) * nq;
    for (int cg = wave * C1W_CPW; cg < a.cout; cg += 4 * C1W_CPW) {
        float acc[C1W_CPW][9];
        float A1[C1W_CPW], A2[C1W_CPW], A3[C1W_CPW];
        float wt[RC ? C1W_CPW : 1][9];  // wave-uniform: constant-space loads into scalar registers
        if constexpr (RC) {
            const cfloat4p wp = (cfloat4p)a.w;
#pragma unroll
            for (int j = 0; j < C1W_CPW; ++j)
#pragma unroll
                for (int t = 0; t < 9; ++t) wt[j][t] = wp[(cg + j) * 9 + t];
        }
#pragma unroll
        for (int j = 0; j < C1W_CPW; ++j) {
            const float4 k = a.cf_dy[cg + j];  // dy = a (dz - mb - (y - mean) mgi)
            A1[j] = k.x;
            A2[j] = -k.x * k.z;
            A3[j] = k.x * (k.w * k.z - k.y);
#pragma unroll
            for (int t = 0; t < 9; ++t) acc[j][t] = 0.f;
        }
        for (int t = lane; t < ntask; t += 64) {
            const int rr = t / nq, q = t - rr * nq;
            const int gr = r0 + rr, b = gr / a.H, hh = gr - b * a.H;
            const int w0 = 4 * q;
            float xr[3][6];
            c1_window<FULL>(a.x + (int64_t)b * HW, a.H, a.W, hh, w0, xr);
            const int64_t o = ((int64_t)b * a.cout + cg) * HW + (int64_t)hh * a.W + w0;
#pragma unroll
            for (int j = 0; j < C1W_CPW; ++j) {
                float dz[4], yy[4];
                if (FULL) {
                    const float4 u = ld4(a.dz + o + (int64_t)j * HW);
                    dz[0] = u.x; dz[1] = u.y; dz[2] = u.z; dz[3] = u.w;
                    if constexpr (!RC) {
                        const float4 v = ld4(a.y + o + (int64_t)j * HW);
                        yy[0] = v.x; yy[1] = v.y; yy[2] = v.z; yy[3] = v.w;
                    }
                }
                if constexpr (RC) {  // conv1_fwd_kernel's arithmetic, term for term
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        float v = 0.f;
#pragma unroll
                        for (int tp = 0; tp < 9; ++tp) v = fmaf(wt[j][tp], xr[tp / 3][e + tp % 3], v);
                        yy[e] = v;
                    }
                }
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    if (!FULL) {
                        const bool ok = w0 + e < a.W;
                        dz[e] = ok ? a.dz[o + (int64_t)j * HW + e] : 0.f;
                        if constexpr (!RC) yy[e] = ok ? a.y[o + (int64_t)j * HW + e] : 0.f;
                    }
                    float dy = fmaf(A1[j], dz[e], fmaf(A2[j], yy[e], A3[j]));
                    if (!FULL && w0 + e >= a.W) dy = 0.f;
#pragma unroll
                    for (int tp = 0; tp < 9; ++tp) acc[j][tp] = fmaf(dy, xr[tp / 3][e + tp % 3], acc[j][tp]);
                }
            }
        }
#pragma unroll
        for (int j = 0; j < C1W_CPW; ++j)
#pragma unroll
            for (int t = 0; t < 9; ++t) {
                float v = wave_sum(acc[j][t]);
                if (lane == 0) a.part[((int64_t)blockIdx.x * a.cout + cg + j) * 9 + t] = v;
            }
    }
}

// Round 6: the same weight gradient with dz streamed HBM -> LDS by LDS-DMA (W % 4 == 0, W <= 252).  The
// register kernel above alternated a wait for each quad's 16-byte loads with its ~650 VALU (1.13 ms at
// B = 4096: 3.8 TB/s); here a block walks its slice's (sample, row) rows with the next row's 32 dz channel
// rows and 3 input rows in flight (double-buffered, no VGPRs held) while the current row is computed from
// LDS.  Thread (channel c = tid >> 3, quad group g = tid & 7) owns one channel: its 9 weights, BN-backward
// coefficients and 9 accumulators live in registers (no SGPR pressure), quads q = g, g + 8, ... of the row.
// Arithmetic per output is conv1_fwd_kernel's recompute of y and wgrad1_kernel's dy / tap order, term for
// term, so each slice's partial sums are the same float operations in the same order as before per pixel;
// only the slice boundaries (rows per slice) differ.
constexpr int W1D_CS = 288;             // LDS floats per dz channel row: 1 KB of DMA + 32 floats, so the 8
                                        // lanes of the next channel read the other 32 banks
constexpr int W1D_XS = 260;             // LDS floats per input row: [4 zero][W][zeros]
constexpr int W1D_BUF = 32 * W1D_CS + 3 * W1D_XS;

__device__ __forceinline__ void w1d_dma(__amdgpu_buffer_rsrc_t r, unsigned voff, unsigned lds_byte_addr) {
    const unsigned m0 = __builtin_amdgcn_readfirstlane(lds_byte_addr);
    asm volatile("s_nop 0\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds" :: "v"(voff), "s"(r), "{m0}"(m0) : "memory");
}

__global__ __launch_bounds__(256) void wgrad1_dma_kernel(Wgrad1Args a) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int c = tid >> 3, g = tid & 7;
    const int H = a.H, W = a.W, HW = H * W, nq = W >> 2;
    const int nrows = a.B * H;
    const int r0 = blockIdx.x * a.rows_per_slice, r1 = min(nrows, r0 + a.rows_per_slice);
    const unsigned lds0 = (unsigned)(uintptr_t)(__attribute__((address_space(3))) void*)smem;
    // zero both buffers once: the input rows' left pad (never written by the DMA) reads 0
    for (int i = tid; i < 2 * W1D_BUF; i += 256) smem[i] = 0.f;
    float wt[9], acc[9];
#pragma unroll
    for (int t = 0; t < 9; ++t) {
        wt[t] = a.w[c * 9 + t];
        acc[t] = 0.f;
    }
    const float4 k = a.cf_dy[c];  // dy = a (dz - mb - (y - mean) mgi)
    const float A1 = k.x, A2 = -k.x * k.z, A3 = k.x * (k.w * k.z - k.y);
    // DMA of row task gr into buffer buf: 32 dz channel rows (wave w: channels w, w + 4, ...) and the input
    // rows h - 1 .. h + 1 (waves 0..2); lanes >= W / 4 and rows outside the sample read 0 (out of range)
    const unsigned lq = (unsigned)lane < (unsigned)nq ? 16u * (unsigned)lane : 0x80000000u;
    auto issue = [&](int gr, int buf) {
        const int b = gr / H, h = gr - b * H;
        const unsigned base = lds0 + 4u * (unsigned)(buf * W1D_BUF);
        const __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<float*>(a.dz + ((int64_t)b * 32 * H + h) * W), (short)0, (int)(((int64_t)31 * HW + W) * 4),
            0x00020000);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int ch = wave + 4 * j;
            w1d_dma(rd, lq == 0x80000000u ? lq : lq + 4u * (unsigned)(ch * HW), base + 4u * (unsigned)(ch * W1D_CS));
        }
        if (wave < 3) {
            const int y = h - 1 + wave;
            const bool ok = (unsigned)y < (unsigned)H;
            const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
                const_cast<float*>(a.x + ((int64_t)b * H + (ok ? y : 0)) * W), (short)0, ok ? W * 4 : 0, 0x00020000);
            w1d_dma(rx, lq, base + 4u * (unsigned)(32 * W1D_CS + wave * W1D_XS + 4));
        }
    };
    __syncthreads();  // the zeroing is done before any DMA lands
    if (r0 < r1) issue(r0, 0);
    for (int gr = r0; gr < r1; ++gr) {
        const int buf = (gr - r0) & 1;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();  // row gr landed for every wave; row gr - 1's buffer fully read
        if (gr + 1 < r1) issue(gr + 1, buf ^ 1);
        const float* dz = smem + buf * W1D_BUF + c * W1D_CS;
        const float* xs = smem + buf * W1D_BUF + 32 * W1D_CS + 4;  // input row 0 (= image row h - 1), column 0
        for (int q = g; q < nq; q += 8) {
            const int w0 = 4 * q;
            const float4 u = *reinterpret_cast<const float4*>(dz + w0);
            float xr[3][6];
#pragma unroll
            for (int r = 0; r < 3; ++r) {
                const float* row = xs + r * W1D_XS + w0;
                const float4 v = *reinterpret_cast<const float4*>(row);
                xr[r][0] = row[-1];
                xr[r][1] = v.x; xr[r][2] = v.y; xr[r][3] = v.z; xr[r][4] = v.w;
                xr[r][5] = row[4];
            }
            const float dzv[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                float yv = 0.f;  // conv1_fwd_kernel's arithmetic, term for term
#pragma unroll
                for (int tp = 0; tp < 9; ++tp) yv = fmaf(wt[tp], xr[tp / 3][e + tp % 3], yv);
                const float dy = fmaf(A1, dzv[e], fmaf(A2, yv, A3));
#pragma unroll
                for (int tp = 0; tp < 9; ++tp) acc[tp] = fmaf(dy, xr[tp / 3][e + tp % 3], acc[tp]);
            }
        }
    }
    // the 8 quad groups of a channel are 8 consecutive lanes
#pragma unroll
    for (int t = 0; t < 9; ++t) {
        float v = acc[t];
        v += __shfl_xor(v, 1, 64);
        v += __shfl_xor(v, 2, 64);
        v += __shfl_xor(v, 4, 64);
        if (g == 0) a.part[((int64_t)blockIdx.x * 32 + c) * 9 + t] = v;
    }
}

// ------------------------------------------------------------------ 7x7 stem (Cin = 1), cnn_deep
// PhonemeNetDeep's stem conv (reference phoneme_cnn.py:211-216: Conv2d(1, C0, 7, padding 3)): its
// output is C0 (64) times the input, so the forward is HBM-write-bound and the weight gradient
// (reads dz0, y0) HBM-read-bound -- direct VALU kernels instead of the general implicit GEMM
// (which gathered a 49-long K per pixel: 20-30 % of the MFMA roof).
//  * a block walks whole samples; each sample's input is staged once in LDS with a zero border
//    (3 rows, 4 columns), so a lane's 7 x 12 window is 21 unconditional ds_read_b128;
//  * lanes own pixel quads; forward: a wave owns CPW output channels whose weights are
//    wave-uniform scalar loads (SGPR operands); BN partial statistics shifted sums in the same
//    pass; weight gradient: a wave owns 2 output channels x 49 taps of accumulators and computes
//    dy = BN backward of (dz0, y0) from its 16-byte loads (no dy pass);
//  * BF16 (precision "bf16"): operands rounded to bf16 as the bf16 implicit GEMM rounds them
//    (input, weights, dy), products exact, float32 sums.
constexpr int ST_K = 7, ST_T = 49, ST_WCPW = 2;

__device__ __forceinline__ float bf16r(float v) { return (float)(__bf16)v; }

__host__ __device__ constexpr int st_rw(int W) { return ((W + 8) + 3) & ~3; }  // LDS row: 4 | W | >= 4

// LDS image of one sample: [H + 6][RW] with the input at (row 3, column 4) and zeros around.
// The border never changes: st_zero clears the whole image once per block, st_stage rewrites
// the interior per sample (16-byte loads, all issued before the LDS writes, when W % 4 == 0).
__device__ __forceinline__ void st_zero(int H, int W, float* xs) {
    const int n = (H + 6) * st_rw(W);
    for (int i = threadIdx.x; i < n; i += blockDim.x) xs[i] = 0.f;
}

template <bool BF>
__device__ __forceinline__ void st_stage(const float* xb, int H, int W, float* xs) {
    const int RW = st_rw(W);
    if ((W & 3) == 0) {
        const int nq = W >> 2, n = H * nq;
        constexpr int U = 8;
        for (int base = 0; base < n; base += U * 256) {
            float4 t[U];
#pragma unroll
            for (int k = 0; k < U; ++k) {
                const int i = base + k * 256 + (int)threadIdx.x;
                t[k] = i < n ? ld4(xb + 4 * i) : make_float4(0.f, 0.f, 0.f, 0.f);
            }
#pragma unroll
            for (int k = 0; k < U; ++k) {
                const int i = base + k * 256 + (int)threadIdx.x;
                if (i < n) {
                    const int r = i / nq, q = i - r * nq;
                    float4 v = t[k];
                    if (BF) { v.x = bf16r(v.x); v.y = bf16r(v.y); v.z = bf16r(v.z); v.w = bf16r(v.w); }
                    *reinterpret_cast<float4*>(xs + (r + 3) * RW + 4 + 4 * q) = v;
                }
            }
        }
    } else {
        const int n = H * W;
        for (int i = threadIdx.x; i < n; i += blockDim.x) {
            const int r = i / W, c = i - r * W;
            const float v = xb[i];
            xs[(r + 3) * RW + 4 + c] = BF ? bf16r(v) : v;
        }
    }
}

// window of the quad at (hh, w0): v[dh][e] = x[hh + dh - 3][w0 - 4 + e], e < 12
__device__ __forceinline__ void st_window(const float* xs, int RW, int hh, int w0, float (&v)[ST_K][12]) {
#pragma unroll
    for (int dh = 0; dh < ST_K; ++dh) {
        const float* r = xs + (hh + dh) * RW + w0;
#pragma unroll
        for (int q = 0; q < 3; ++q) {
            const float4 t = *reinterpret_cast<const float4*>(r + 4 * q);
            v[dh][4 * q] = t.x; v[dh][4 * q + 1] = t.y; v[dh][4 * q + 2] = t.z; v[dh][4 * q + 3] = t.w;
        }
    }
}

template <bool BF, int CPW>
__global__ __launch_bounds__(256) void stem_fwd_kernel(StemArgs a) {
    extern __shared__ __attribute__((aligned(16))) float xs[];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int H = a.H, W = a.W, HW = H * W, RW = st_rw(W);
    const int nq = (W + 3) >> 2, ntask = H * nq;
    const int cg = wave * CPW;  // a.cout == 4 CPW
    cfloat4p w = (cfloat4p)a.w;  // [C][49] (bf16-rounded for BF)
    float K[CPW], s1[CPW], s2[CPW];
#pragma unroll
    for (int j = 0; j < CPW; ++j) s1[j] = s2[j] = 0.f;
    int nsamp = 0;
    st_zero(H, W, xs);
    for (int b = blockIdx.x; b < a.B; b += gridDim.x, ++nsamp) {
        __syncthreads();
        st_stage<BF>(a.x + (int64_t)b * HW, H, W, xs);
        __syncthreads();
        if (b == (int)blockIdx.x) {  // shift for the one-pass variance: the block's first output
            float v[ST_K][12];
            st_window(xs, RW, 0, 0, v);
#pragma unroll
            for (int j = 0; j < CPW; ++j) {
                float acc = 0.f;
#pragma unroll
                for (int t = 0; t < ST_T; ++t) acc = fmaf(w[(cg + j) * ST_T + t], v[t / ST_K][4 + t % ST_K - 3], acc);
                K[j] = acc;
            }
        }
        float* ob = a.out + ((int64_t)b * a.cout + cg) * HW;
        for (int t = lane; t < ntask; t += 64) {
            const int hh = t / nq, w0 = 4 * (t - hh * nq);
            float v[ST_K][12];
            st_window(xs, RW, hh, w0, v);
#pragma unroll
            for (int j = 0; j < CPW; ++j) {
                // an opaque zero keeps the weight loads inside the task loop: 49 SGPRs live per
                // channel instead of CPW x 49 hoisted ones spilling to VGPR lanes
                int z;
                asm volatile("s_mov_b32 %0, 0" : "=s"(z));
                const cfloat4p wj = w + (cg + j) * ST_T + z;
                float o[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int tp = 0; tp < ST_T; ++tp) {
                    const float wt = wj[tp];
#pragma unroll
                    for (int e = 0; e < 4; ++e) o[e] = fmaf(wt, v[tp / ST_K][e + 4 + tp % ST_K - 3], o[e]);
                }
                float* op = ob + (int64_t)j * HW + hh * W + w0;
                if ((W & 3) == 0) {
                    st4(op, make_float4(o[0], o[1], o[2], o[3]));
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        const float d = o[e] - K[j];
                        s1[j] += d;
                        s2[j] = fmaf(d, d, s2[j]);
                    }
                } else {
#pragma unroll
                    for (int e = 0; e < 4; ++e)
                        if (w0 + e < W) {
                            op[e] = o[e];
                            const float d = o[e] - K[j];
                            s1[j] += d;
                            s2[j] = fmaf(d, d, s2[j]);
                        }
                }
            }
        }
    }
    const float n = (float)nsamp * (float)HW;
#pragma unroll
    for (int j = 0; j < CPW; ++j) {
        const float t1 = wave_sum(s1[j]), t2 = wave_sum(s2[j]);
        if (lane == 0) {
            a.part0[(int64_t)(cg + j) * a.nblk + blockIdx.x] = n * K[j] + t1;
            a.part1[(int64_t)(cg + j) * a.nblk + blockIdx.x] = n > 0.f ? fmaxf(t2 - t1 * t1 / n, 0.f) : 0.f;
        }
    }
    if (threadIdx.x == 0) a.partn[blockIdx.x] = n;
}

// bf16 precision, cout = 64: the 7x7 stem as a bf16 MFMA GEMM per 32-pixel tile (v_mfma_f32_32x32x16_bf16),
// C[cout][pixel] = W[cout][tap] x im2col[tap][pixel] with fp32 accumulation.  The operands are the values
// stem_fwd_kernel<true> multiplies (x and w rounded to bf16), so only the summation order differs.
// K = 64 is an 8 x 8 tap grid (dh = 2s + h, dw = j for K-step s, lane half h, element j; dh or dw = 7 carry
// zero weights), which makes every B offset lane-uniform: element j of K-step s is xs[2s RW + j] from the
// lane's (pixel, h) base.  Per tile: 32 LDS reads, 8 MFMAs, 32 coalesced 128-byte row stores; BN partials
// as stem_fwd_kernel's (per-block shift = the outputs of the block's first pixel, sum and M2).
typedef __bf16 st_bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned st_u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned st_u32x2 __attribute__((ext_vector_type(2)));

// bf16 image of one stem sample for the MFMA forms: rows of st_rw2 elements, the input at (row 3,
// column 4), zeros around, held twice -- copy k shifted right by k elements -- so that any run of
// consecutive elements starting at column c is read as dwords from copy (c & 1) (2-element aligned);
// the copy stride makes copy 1's dwords start half-way round the banks.
__host__ __device__ constexpr int st_rw2(int W) { return st_rw(W) + 2; }
__host__ __device__ constexpr int st_cp2(int rows, int W) {
    return ((rows * st_rw2(W) / 2 + 31) / 32 * 32 + 16) * 2;  // elements; (st_cp2 / 2) % 32 == 16
}
__device__ __forceinline__ void st2_zero(__bf16* xs, int rows, int W) {
    const int n = st_cp2(rows, W);  // both copies: 2 n elements = n dwords
    for (int i = threadIdx.x; i < n; i += blockDim.x) reinterpret_cast<unsigned*>(xs)[i] = 0u;
}
// the interior (rows 3 .. H + 2, columns 4 .. W + 3) of both copies; loads batched ahead of the writes
__device__ __forceinline__ void st2_stage(const float* __restrict__ xb, int H, int W, __bf16* xs, int rows) {
    const int RW2 = st_rw2(W), CP = st_cp2(rows, W), n = H * W;
    constexpr int U = 8;
    const int dq = (int)blockDim.x / W, dr = (int)blockDim.x - dq * W;
    int r0 = (int)threadIdx.x / W, c0 = (int)threadIdx.x - r0 * W;
    for (int base = 0; base < n; base += U * (int)blockDim.x) {
        float v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int i = base + u * (int)blockDim.x + (int)threadIdx.x;
            v[u] = xb[i < n ? i : 0];
        }
        int r = r0, c = c0;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int i = base + u * (int)blockDim.x + (int)threadIdx.x;
            if (i < n) {
                const __bf16 bv = (__bf16)v[u];
                const int o = (r + 3) * RW2 + c + 4;
                xs[o] = bv;
                xs[CP + o + 1] = bv;
            }
            r += dq;
            c += dr;
            if (c >= W) { c -= W; ++r; }
        }
        r0 = r;
        c0 = c;
    }
}
// 8 consecutive elements of row r from column c (both copies: 4 dword reads)
__device__ __forceinline__ st_bf16x8 st2_ld8(const __bf16* xs, int CP, int o) {
    const int k = o & 1;  // (RW2 even: the column's parity)
    const unsigned* p = reinterpret_cast<const unsigned*>(xs + k * CP + o + k);
    st_u32x4 v;
    v.x = p[0]; v.y = p[1]; v.z = p[2]; v.w = p[3];
    return __builtin_bit_cast(st_bf16x8, v);
}
__device__ __forceinline__ st_u32x2 st2_ld4(const __bf16* xs, int CP, int o) {
    const int k = o & 1;
    const unsigned* p = reinterpret_cast<const unsigned*>(xs + k * CP + o + k);
    st_u32x2 v;
    v.x = p[0]; v.y = p[1];
    return v;
}

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void stem_fwd_mfma_kernel(StemArgs a) {
    extern __shared__ __attribute__((aligned(16))) float xs_f[];  // two bf16 copies of (H + 7) rows (spare zero row)
    __bf16* xs = reinterpret_cast<__bf16*>(xs_f);
    __shared__ float red[2][64][2];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, h = lane >> 5, l32 = lane & 31;
    const int mt = wave >> 1, wt = wave & 1;  // waves 2 mt, 2 mt + 1: couts 32 mt .. 32 mt + 31, alternate tiles
    const int H = a.H, W = a.W, HW = H * W, RW2 = st_rw2(W), CP = st_cp2(H + 7, W);
    st_bf16x8 A[4];
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int dh = 2 * s + h, dw = j;
            A[s][j] = (__bf16)((dh < ST_K && dw < ST_K) ? a.w[(32 * mt + l32) * ST_T + dh * ST_K + dw] : 0.f);
        }
    st2_zero(xs, H + 7, W);
    const int ntile = (HW + 31) >> 5;
    auto tile = [&](int tt, int& p) {
        p = tt * 32 + l32;
        const int pc = min(p, HW - 1);
        const int hh = pc / W, ww = pc - hh * W;
        const int o = (hh + h) * RW2 + ww + 1;
        f32x16 acc = {0.f};
#pragma unroll
        for (int s = 0; s < 4; ++s) acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[s], st2_ld8(xs, CP, o + 2 * s * RW2), acc, 0, 0, 0);
        return acc;
    };
    float K[16], s1[16], s2[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) s1[r] = s2[r] = 0.f;
    int nsamp = 0;
    for (int b = blockIdx.x; b < a.B; b += gridDim.x, ++nsamp) {
        __syncthreads();
        st2_stage(a.x + (int64_t)b * HW, H, W, xs, H + 7);
        __syncthreads();
        if (b == (int)blockIdx.x) {  // shift: every wave evaluates the block's first pixel itself
            int p;
            const f32x16 acc = tile(0, p);
#pragma unroll
            for (int r = 0; r < 16; ++r) K[r] = __shfl(acc[r], 32 * h, 64);
        }
        float* ob = a.out ? a.out + ((int64_t)b * a.cout + 32 * mt) * HW : nullptr;  // none: statistics only
        for (int tt = wt; tt < ntile; tt += 2) {
            int p;
            const f32x16 acc = tile(tt, p);
            if (p < HW) {
                float* op = ob + p;
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const float v = acc[r];
                    if (ob) op[acc_row(r, h) * HW] = v;
                    const float d = v - K[r];
                    s1[r] += d;
                    s2[r] = fmaf(d, d, s2[r]);
                }
            }
        }
    }
    // per channel: the 32 pixel lanes of each half, then the two waves of the cout half
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        float t1 = s1[r], t2 = s2[r];
#pragma unroll
        for (int o = 1; o < 32; o <<= 1) {
            t1 += __shfl_xor(t1, o, 64);
            t2 += __shfl_xor(t2, o, 64);
        }
        if (l32 == 0) {
            red[wt][32 * mt + acc_row(r, h)][0] = t1;
            red[wt][32 * mt + acc_row(r, h)][1] = t2;
        }
    }
    __syncthreads();
    const float n = (float)nsamp * (float)HW;
    if (wt == 0 && l32 == 0) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int c = 32 * mt + acc_row(r, h);
            const float t1 = red[0][c][0] + red[1][c][0], t2 = red[0][c][1] + red[1][c][1];
            a.part0[(int64_t)c * a.nblk + blockIdx.x] = n * K[r] + t1;
            a.part1[(int64_t)c * a.nblk + blockIdx.x] = n > 0.f ? fmaxf(t2 - t1 * t1 / n, 0.f) : 0.f;
        }
    }
    if (threadIdx.x == 0) a.partn[blockIdx.x] = n;
}

// float32 precision, cout = 64: the 7x7 stem on fp32 MFMA (v_mfma_f32_32x32x2_f32), C[cout][pixel] =
// W[cout][tap] x im2col[tap][pixel] per 32-pixel tile, K = the 49 taps in 25 K-steps (tap 2 ks + h in
// lane half h; the 50th carries a zero weight).  Weights stay in registers (A: 25 per lane), B = x of
// the fp32 LDS image at the lane's pixel + the tap's offset (one ds_read_b32 per K-step).  Products
// and sums in float32; only the summation order differs from stem_fwd_kernel<false>.  Stores and BN
// partials as stem_fwd_mfma_kernel's.
__global__ __launch_bounds__(256) void stem_fwd_f32_kernel(StemArgs a) {
    extern __shared__ __attribute__((aligned(16))) float xs[];  // (H + 8) rows of the sample
    __shared__ float red[2][64][2];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, h = lane >> 5, l32 = lane & 31;
    const int mt = wave >> 1, wt = wave & 1;
    const int H = a.H, W = a.W, HW = H * W, RW = st_rw(W);
    constexpr int NK = (ST_T + 1) / 2;
    float A[NK];
    int toff[NK];
#pragma unroll
    for (int s = 0; s < NK; ++s) {
        const int t = 2 * s + h;
        A[s] = t < ST_T ? a.w[(32 * mt + l32) * ST_T + t] : 0.f;
        toff[s] = t < ST_T ? (t / ST_K) * RW + t % ST_K : 0;
    }
    for (int i = threadIdx.x; i < (H + 8) * RW; i += 256) xs[i] = 0.f;
    const int ntile = (HW + 31) >> 5;
    auto tile = [&](int tt, int& p) {
        p = tt * 32 + l32;
        const int pc = min(p, HW - 1);
        const int hh = pc / W, ww = pc - hh * W;
        const float* xb = xs + hh * RW + ww + 1;
        f32x16 acc = {0.f};
#pragma unroll
        for (int s = 0; s < NK; ++s) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(A[s], xb[toff[s]], acc, 0, 0, 0);
        return acc;
    };
    float K[16], s1[16], s2[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) s1[r] = s2[r] = 0.f;
    int nsamp = 0;
    for (int b = blockIdx.x; b < a.B; b += gridDim.x, ++nsamp) {
        __syncthreads();
        st_stage<false>(a.x + (int64_t)b * HW, H, W, xs);
        __syncthreads();
        if (b == (int)blockIdx.x) {  // shift: every wave evaluates the block's first pixel itself
            int p;
            const f32x16 acc = tile(0, p);
#pragma unroll
            for (int r = 0; r < 16; ++r) K[r] = __shfl(acc[r], 32 * h, 64);
        }
        float* ob = a.out + ((int64_t)b * a.cout + 32 * mt) * HW;
        for (int tt = wt; tt < ntile; tt += 2) {
            int p;
            const f32x16 acc = tile(tt, p);
            if (p < HW) {
                float* op = ob + p;
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const float v = acc[r];
                    op[acc_row(r, h) * HW] = v;
                    const float d = v - K[r];
                    s1[r] += d;
                    s2[r] = fmaf(d, d, s2[r]);
                }
            }
        }
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        float t1 = s1[r], t2 = s2[r];
#pragma unroll
        for (int o = 1; o < 32; o <<= 1) {
            t1 += __shfl_xor(t1, o, 64);
            t2 += __shfl_xor(t2, o, 64);
        }
        if (l32 == 0) {
            red[wt][32 * mt + acc_row(r, h)][0] = t1;
            red[wt][32 * mt + acc_row(r, h)][1] = t2;
        }
    }
    __syncthreads();
    const float n = (float)nsamp * (float)HW;
    if (wt == 0 && l32 == 0) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int c = 32 * mt + acc_row(r, h);
            const float t1 = red[0][c][0] + red[1][c][0], t2 = red[0][c][1] + red[1][c][1];
            a.part0[(int64_t)c * a.nblk + blockIdx.x] = n * K[r] + t1;
            a.part1[(int64_t)c * a.nblk + blockIdx.x] = n > 0.f ? fmaxf(t2 - t1 * t1 / n, 0.f) : 0.f;
        }
    }
    if (threadIdx.x == 0) a.partn[blockIdx.x] = n;
}

// ------------------------------------------------------------------ fused bf16 stem (no y0 plane)
// At T = 200 the stem's 64 x 40 x 200 fp32 output is 8.4 GB per 4096-sample step, written once and
// read three times (pool, pool backward, weight gradient) -- more HBM traffic than the rest of the
// network's activations.  The bf16 stem GEMM is ~65 MFLOP per sample (0.1 ms of MFMA per step), so
// the fused form recomputes y0 wherever it is needed instead: stem_fwd_mfma_kernel with out = nullptr
// (BN statistics), stem_pool_kernel (pool outputs), stem_wgrad_rc_kernel (weight gradient from dz0).
// Every recomputation multiplies the same bf16 operands in the same K order as the statistics pass.
typedef __bf16 st_bf16x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x2_t __attribute__((ext_vector_type(2)));
typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));
constexpr int SP_CB = 15;  // pooled windows per column block (30 image columns + a halo column each side)
constexpr int SP_LRW = 44; // bf16 row stride of a column block's staged x (40 columns + 4 shifted copies' slack)

__host__ __device__ constexpr int sp_ncb(int OW) { return (OW + SP_CB - 1) / SP_CB; }
__host__ __device__ constexpr int sp_copy(int H) { return (H + 7) * SP_LRW; }  // bf16 elements per shifted copy

__device__ __forceinline__ float sp_relu(float y, float kx, float ky) { return fmaxf(fmaf(y, kx, ky), 0.f); }

// One wave per (sample b, cout half mt, column block k): image columns c0 - 1 .. c0 + 30 (c0 = 30 k) are
// the wave's 32 MFMA pixel lanes, pooled windows j = 15 k .. 15 k + 14 are centred on its odd lanes.
// The x columns it needs (c0 - 4 .. c0 + 35, 7 x 7 taps) are staged as bf16 in four copies shifted by
// 0..3 elements, so that every lane reads its 8 consecutive taps of a K-step as two aligned ds_read_b64
// (no 16-bit reads).  Per pooled row i: the y0 tiles of rows 2 i and 2 i + 1 (the statistics pass's MFMA
// orientation and K order: the same values bit for bit; row 2 i - 1 is the previous step's second tile,
// kept in registers), the column maximum of ReLU(BN0(y0)) over the window rows in registers, then the
// 3-column windows from the two neighbouring lanes (shuffles) with the maxpool3_fwd tie rule (first
// maximum in row-major window order; 255 when the maximum is <= 0).  Writes a0, the tap, y0 at the tap
// and (optional) the padded NHWC bf16 image of a0 (borders included).  No block barrier after staging.
// (round 5) Two waves per block, one per cout half, sharing the staged x: half the LDS and half the staging
// per wave (the one-wave blocks held ~2 waves per SIMD at 16.5 KB of LDS each).
__global__ __launch_bounds__(128, 2) void stem_pool_kernel(StemArgs a) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    __bf16* xs = reinterpret_cast<__bf16*>(smem);
    const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, l = lane & 31;
    const int mt = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int H = a.H, W = a.W, OH = a.OH, OW = a.OW, C = a.cout, ncb = sp_ncb(OW);
    const int k = blockIdx.x % ncb, b = blockIdx.x / ncb;
    const int c0 = 2 * SP_CB * k, CP = sp_copy(H);
    {  // stage x columns c0 - 4 .. c0 + 35 (zero outside the image) into the four shifted copies; the
       // loads of a batch are all issued before its LDS writes (one memory latency per batch)
        const auto rs_x = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.x + (int64_t)b * H * W), (short)0,
                                                            H * W * 4, 0x00020000);
        constexpr int NB = 5;
        const int n = (H + 7) * 40;
        for (int base = 0; base < n; base += NB * 128) {
            float v[NB];
#pragma unroll
            for (int u = 0; u < NB; ++u) {
                const int idx = base + u * 128 + tid;
                const int sr = idx / 40, lc = idx - sr * 40;
                const int xr = sr - 3, xc = c0 - 4 + lc;
                const bool ok = idx < n && xr >= 0 && xr < H && xc >= 0 && xc < W;  // else 0 (out-of-range offset)
                v[u] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs_x, ok ? (xr * W + xc) * 4 : 0x7fff0000, 0, 0));
            }
#pragma unroll
            for (int u = 0; u < NB; ++u) {
                const int idx = base + u * 128 + tid;
                if (idx < n) {
                    const int sr = idx / 40, lc = idx - sr * 40;
                    const __bf16 bv = (__bf16)v[u];
#pragma unroll
                    for (int q = 0; q < 4; ++q) xs[q * CP + sr * SP_LRW + lc + q] = bv;
                }
            }
        }
    }
    st_bf16x8 A[4];
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int dh = 2 * s + h, dw = j;
            A[s][j] = (__bf16)((dh < ST_K && dw < ST_K) ? a.w[(32 * mt + l) * ST_T + dh * ST_K + dw] : 0.f);
        }
    float kx[16], ky[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const float4 cf = a.cf[32 * mt + acc_row(r, h)];
        kx[r] = cf.x;
        ky[r] = cf.y;
    }
    __syncthreads();
    // lane l reads local columns l .. l + 7 from the copy that puts l at a multiple of 4 elements
    const int q = (4 - (l & 3)) & 3;
    const __bf16* xl = xs + q * CP + l + q;
    auto tile = [&](int row) {  // y0 of image row `row`, columns c0 - 1 + l, the lane's 16 couts
        f32x16 acc = {0.f};
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            const __bf16* p = xl + (row + 2 * s + h) * SP_LRW;
            const st_bf16x4 lo = *reinterpret_cast<const st_bf16x4*>(p);
            const st_bf16x4 hi = *reinterpret_cast<const st_bf16x4*>(p + 4);
            st_bf16x8 Bv;
#pragma unroll
            for (int e = 0; e < 4; ++e) { Bv[e] = lo[e]; Bv[4 + e] = hi[e]; }
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[s], Bv, acc, 0, 0, 0);
        }
        return acc;
    };
    const int col = c0 - 1 + l;
    const bool cvalid = col >= 0 && col < W;
    const int j = SP_CB * k + ((l - 1) >> 1);
    const bool center = (l & 1) && l < 2 * SP_CB && j < OW;
    const int Wp = OW + 2, OHW = OH * OW;
    // outputs (pooled NHWC [B][OH][OW][C]: the 32 couts of a window are one 128-byte line of y0 at the
    // tap, 32 bytes of taps) through buffer stores: the lane's window in voffset (out of range for lanes
    // that centre none: the store is dropped), the 8-cout group in soffset
    constexpr int OOBV = 0x7fff0000;
    const int64_t pbase = (int64_t)b * OHW * C + 32 * mt;
    const auto rs_ysel = __builtin_amdgcn_make_buffer_rsrc(a.pool_ysel + pbase, (short)0, (OHW * C - 32 * mt) * 4, 0x00020000);
    const auto rs_arg = __builtin_amdgcn_make_buffer_rsrc(a.pool_arg + pbase, (short)0, OHW * C - 32 * mt, 0x00020000);
    __bf16* nimg = a.pool_nhwc ? static_cast<__bf16*>(a.pool_nhwc) + (int64_t)b * (OH + 2) * Wp * C + 32 * mt
                               : nullptr;
    const auto rs_nhwc = __builtin_amdgcn_make_buffer_rsrc(nimg, (short)0, ((OH + 2) * Wp * C - 32 * mt) * 2, 0x00020000);
    // carried row 2 i - 1: raw y0 and its activation (-inf before the first row: no such window row)
    f32x16 cy = {0.f}, cv;
#pragma unroll
    for (int r = 0; r < 16; ++r) cv[r] = -INFINITY;
    for (int i = 0; i < OH; ++i) {
        const int r0 = 2 * i, r1 = 2 * i + 1;
        const bool has1 = r1 < H;
        const f32x16 t0 = tile(r0);
        const f32x16 t1 = tile(has1 ? r1 : r0);
        // column maxima of ReLU(BN0(y0)) over the window rows 2 i - 1 (kh 0), 2 i (1), 2 i + 1 (2): the
        // first maximal row (max3, then the first row equal to it); -inf for columns outside the image
        float ym[16], vm[16];
        unsigned khp = 0;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const float v0 = sp_relu(t0[r], kx[r], ky[r]);
            const float v1 = has1 ? sp_relu(t1[r], kx[r], ky[r]) : -INFINITY;
            const float m = __builtin_fmaxf(__builtin_fmaxf(cv[r], v0), v1);
            const bool e0 = cv[r] == m, e1 = v0 == m;
            const unsigned kh = e0 ? 0u : (e1 ? 1u : 2u);
            ym[r] = e0 ? cy[r] : (e1 ? t0[r] : t1[r]);
            vm[r] = cvalid ? m : -INFINITY;
            khp |= kh << (2 * r);
            cv[r] = v1;
        }
        cy = t1;
        const unsigned khl = (unsigned)__shfl((int)khp, lane - 1, 64), khr = (unsigned)__shfl((int)khp, lane + 1, 64);
        const int vo = center ? ((i * OW + j) * C + 4 * h) : OOBV;                // element offset
        const int vn = center && nimg ? (((i + 1) * Wp + j + 1) * C + 4 * h) * 2 : OOBV;  // NHWC byte offset
        st_bf16x4 nv;
        f32x4_t yv;
        unsigned av = 0;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            // the window over columns (l - 1, l, l + 1): maximum, then the first tap holding it in
            // row-major order (kh 3 + kw); activations are exact copies, so equality is exact
            const float vl = __shfl(vm[r], lane - 1, 64), vr = __shfl(vm[r], lane + 1, 64);
            const float yl = __shfl(ym[r], lane - 1, 64), yr = __shfl(ym[r], lane + 1, 64);
            const float m = __builtin_fmaxf(__builtin_fmaxf(vl, vm[r]), vr);
            const unsigned tl = ((khl >> (2 * r)) & 3u) * 3u, tc = ((khp >> (2 * r)) & 3u) * 3u + 1u,
                           tr = ((khr >> (2 * r)) & 3u) * 3u + 2u;
            const unsigned sl = vl == m ? tl : 15u, sc = vm[r] == m ? tc : 15u, sr = vr == m ? tr : 15u;
            const unsigned sel = min(min(sl, sc), sr);
            // registers 4 g .. 4 g + 3 are couts 32 mt + 8 g + 4 h .. + 3: one 16-byte y0 store, one
            // 4-byte tap store, one 8-byte NHWC store per group
            yv[r & 3] = sel == sl ? yl : (sel == sc ? ym[r] : yr);
            av |= (m > 0.f ? sel : 255u) << (8 * (r & 3));
            nv[r & 3] = (__bf16)m;
            if ((r & 3) == 3) {
                const int g = r >> 2;
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, yv), rs_ysel, vo * 4, 32 * g, 0);
                __builtin_amdgcn_raw_buffer_store_b32(av, rs_arg, vo, 8 * g, 0);
                if (nimg) __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2_t, nv), rs_nhwc, vn, 16 * g, 0);
                av = 0;
            }
        }
    }
    if (nimg) {  // zero ring: rows 0 and OH + 1 over this block's columns, columns 0 / OW + 1 of the edge blocks
        const int jlo = k == 0 ? 0 : SP_CB * k + 1, jhi = min(SP_CB * k + SP_CB, OW) + (k == ncb - 1 ? 1 : 0);
        const int nrow = jhi - jlo + 1, ncol = (k == 0 ? OH : 0) + (k == ncb - 1 ? OH : 0);
        for (int t = lane; t < 8 * (2 * nrow + ncol); t += 64) {
            const int pos = t >> 3, part = t & 7;
            int rr, cc;
            if (pos < 2 * nrow) {
                rr = pos < nrow ? 0 : OH + 1;
                cc = jlo + (pos < nrow ? pos : pos - nrow);
            } else {
                const int e = pos - 2 * nrow;
                rr = 1 + (k == 0 ? (e < OH ? e : e - OH) : e);
                cc = (k == 0 && e < OH) ? 0 : OW + 1;
            }
            *reinterpret_cast<st_bf16x4*>(nimg + ((int64_t)rr * Wp + cc) * C + 4 * part) = st_bf16x4{};
        }
    }
}

// MaxPool(3,2,1) + ReLU backward of the fused stem, fused with the BN0 backward sums.  Block (sample b,
// cout half hf) walks the pooled rows: rows i and i + 1 of the gated pooled gradient (0 where the window
// maximum was <= 0) and of the taps sit in a two-slot LDS ring, row i + 2 is loaded into registers while
// band i is produced.  A thread owns 2 x 2 input pixels (rows 2 i, 2 i + 1, columns 2 m, 2 m + 1) of a
// cout: the only windows that can select them are (i, m), (i, m + 1), (i + 1, m), (i + 1, m + 1), each
// through one fixed tap, added in window order (the reference's accumulation order).  dz0 is written as
// bf16 (its only consumer, the weight gradient, rounds dy to bf16 anyway).  The BN0 backward sums run
// over the windows as their rows are staged: sum dz0 = sum of the gated gradient, sum dz0 * xhat = sum
// of gated * xhat(y0 at the tap) -- the per-pixel sums regrouped.  Partials per (cout, sample).
constexpr int SPB_T = 256;
constexpr int SPB_NI = 16;  // staged items per thread and row: 32 * OW <= 16 * 256 (OW <= 128)

// one pooled row of the half: gradient items (c, j) from the NCHW planes (+ the second addend), tap / y0
// items (j = t >> 5, c = t & 31) from the pooled NHWC runs.  Every load is unconditional (items out of
// range read element 0 and are replaced afterwards), so a row's loads are all in flight together.
template <bool TWO>
__device__ __forceinline__ void spb_load_row(int row, int OH, int OW, int OHW, int n, int C, int hf, int c_0, int j_0,
                                             int cq, int cr, const float* __restrict__ dp, const float* __restrict__ dp2,
                                             const float* __restrict__ yp, const uint8_t* __restrict__ ap,
                                             float (&dv)[SPB_NI], float (&yv)[SPB_NI], int (&av)[SPB_NI]) {
    const bool rok = row < OH;
    int c = c_0, j = j_0;
#pragma unroll
    for (int u = 0; u < SPB_NI; ++u) {
        const int t = u * SPB_T + (int)threadIdx.x;
        const bool ok = t < n && rok;
        const int jj = t >> 5, cc = t & 31;
        const int od = ok ? c * OHW + row * OW + j : 0;
        const int on = ok ? (row * OW + jj) * C + 32 * hf + cc : 0;
        float d = dp[od];
        if (TWO) d += dp2[od];
        const float y = yp[on];
        const int ab = ap[on];
        dv[u] = ok ? d : 0.f;
        yv[u] = ok ? y : 0.f;
        av[u] = ok ? ab : 255;
        c += cq;
        j += cr;
        if (j >= OW) { j -= OW; ++c; }
    }
}

__global__ __launch_bounds__(SPB_T) void stem_pool_bwd_kernel(StemArgs a) {
    extern __shared__ __attribute__((aligned(16))) float sm[];
    const int b = blockIdx.x >> 1, hf = blockIdx.x & 1, C = a.cout;
    const int H = a.H, W = a.W, OH = a.OH, OW = a.OW, OHW = OH * OW, n = 32 * OW;
    // LDS rows of OWP = OW + 2 columns: the two sentinel columns (tap 255, gradient 0) stand for the
    // windows past the right edge, so the band loop reads its six windows unconditionally
    const int OWP = OW + 2, np_ = 32 * OWP;
    float* gl = sm;                                                // [2][32][OWP] gated gradient
    uint8_t* al = reinterpret_cast<uint8_t*>(sm + 2 * np_);        // [2][32][OWP] taps
    float* ysl = reinterpret_cast<float*>(al + ((2 * np_ + 15) & ~15));  // [32][OWP] y0 at the tap (sums)
    for (int t = threadIdx.x; t < 2 * 32 * 2; t += SPB_T) {        // sentinels of both slots
        const int sl = t >> 6, cc = (t >> 1) & 31, e = t & 1;
        gl[sl * np_ + cc * OWP + OW + e] = 0.f;
        al[sl * np_ + cc * OWP + OW + e] = 255;
    }
    __shared__ float kz[32], kw4[32];
    if (threadIdx.x < 32) {
        const float4 k = a.cf[32 * hf + threadIdx.x];
        kz[threadIdx.x] = k.z;
        kw4[threadIdx.x] = k.w;
    }
    const float* dpb = a.dpool + ((int64_t)b * C + 32 * hf) * OHW;   // NCHW planes of the half
    const float* dpb2 = a.dpool2 ? a.dpool2 + ((int64_t)b * C + 32 * hf) * OHW : dpb;
    const float* ypb = a.pool_ysel + (int64_t)b * OHW * C;            // pooled NHWC of the sample
    const uint8_t* apb = a.pool_arg + (int64_t)b * OHW * C;
    const bool two = a.dpool2 != nullptr;
    float dv[SPB_NI], yv[SPB_NI];
    int av[SPB_NI];
    // item t = u * 256 + tid as (c, j) = (t / OW, t % OW), advanced per u without divisions
    const int cq = SPB_T / OW, cr = SPB_T - cq * OW;
    const int c_0 = (int)threadIdx.x / OW, j_0 = (int)threadIdx.x - c_0 * OW;
#define PCX_SPB_LOAD(ROW)                                                                                    \
    do {                                                                                                     \
        if (two) spb_load_row<true>(ROW, OH, OW, OHW, n, C, hf, c_0, j_0, cq, cr, dpb, dpb2, ypb, apb, dv, yv, av);  \
        else spb_load_row<false>(ROW, OH, OW, OHW, n, C, hf, c_0, j_0, cq, cr, dpb, dpb2, ypb, apb, dv, yv, av); \
    } while (0)
    // taps and y0 first (NHWC items), a barrier, the gradient gated by its tap (NCHW items), a barrier,
    // then the BN0 sums of the row: thread t sums channel t >> 3 over columns t & 7, t & 7 + 8, ...
    double sg = 0.0, sx = 0.0;
    const int sc_c = threadIdx.x >> 3, sc_j = threadIdx.x & 7;
    auto store_row = [&](int slot) {
        float* g = gl + slot * np_;
        uint8_t* ap = al + slot * np_;
#pragma unroll
        for (int u = 0; u < SPB_NI; ++u) {
            const int t = u * SPB_T + (int)threadIdx.x;
            if (t < n) {
                const int jj = t >> 5, cc = t & 31;
                ap[cc * OWP + jj] = (uint8_t)av[u];
                ysl[cc * OWP + jj] = yv[u];
            }
        }
        __syncthreads();
        {
            int c = c_0, j = j_0;
#pragma unroll
            for (int u = 0; u < SPB_NI; ++u) {
                const int t = u * SPB_T + (int)threadIdx.x;
                if (t < n) g[c * OWP + j] = ap[c * OWP + j] != 255 ? dv[u] : 0.f;
                c += cq;
                j += cr;
                if (j >= OW) { j -= OW; ++c; }
            }
        }
        __syncthreads();
        const float kzc = kz[sc_c], kwc = kw4[sc_c];
        float tg = 0.f, tx = 0.f;  // (a row's dozen terms in float32, the running sums in float64)
        for (int j = sc_j; j < OW; j += 8) {
            const float gv = g[sc_c * OWP + j];
            tg += gv;
            tx = fmaf(gv, (ysl[sc_c * OWP + j] - kzc) * kwc, tx);
        }
        sg += (double)tg;
        sx += (double)tx;
    };
    __syncthreads();
    PCX_SPB_LOAD(0);
    store_row(0);
    PCX_SPB_LOAD(1);
    __syncthreads();
    store_row(1);
    // band item: channel c, 4-column group q -> pixels (2 i + dr, 4 q + dc), dr < 2, dc < 4; the
    // windows (i + wi, 2 q + wj), wi < 2, wj < 3, reach pixel (2 wi - 1 + kh, 2 wj - 1 + kw) through tap
    // kh 3 + kw; contributions are added in window (row-major) order
    const int MQ = (W + 3) >> 2;
    const int mq = SPB_T / MQ, mr = SPB_T - mq * MQ;
    uint16_t* const zb = a.dz16 + ((int64_t)b * C + 32 * hf) * H * W;  // the half's 32 planes (32-bit offsets)
    for (int i = 0; i < OH; ++i) {
        PCX_SPB_LOAD(i + 2);  // in flight under the band
        __syncthreads();  // rows i, i + 1 staged
        const float* g0 = gl + (i & 1) * np_;
        const float* g1 = gl + ((i + 1) & 1) * np_;
        const uint8_t* a0 = al + (i & 1) * np_;
        const uint8_t* a1 = al + ((i + 1) & 1) * np_;
        const bool r1ok = 2 * i + 1 < H;
        int c = (int)threadIdx.x / MQ, q = (int)threadIdx.x - c * MQ;
        for (int t = threadIdx.x; t < 32 * MQ; t += SPB_T, c += mq, q += mr) {
            if (q >= MQ) { q -= MQ; ++c; }
            const int o = c * OWP + 2 * q;
            int tp[2][3];
            float dd[2][3];
#pragma unroll
            for (int wj = 0; wj < 3; ++wj) {
                tp[0][wj] = a0[o + wj];
                tp[1][wj] = a1[o + wj];
                dd[0][wj] = g0[o + wj];
                dd[1][wj] = g1[o + wj];
            }
            float px[2][4] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
#pragma unroll
            for (int wi = 0; wi < 2; ++wi)
#pragma unroll
                for (int wj = 0; wj < 3; ++wj)
#pragma unroll
                    for (int dr = 0; dr < 2; ++dr)
#pragma unroll
                        for (int dc = 0; dc < 4; ++dc) {
                            const int kh = dr + 1 - 2 * wi, kw = dc + 1 - 2 * wj;
                            if (kh < 0 || kh > 2 || kw < 0 || kw > 2) continue;
                            if (tp[wi][wj] == kh * 3 + kw) px[dr][dc] += dd[wi][wj];
                        }
            const int col = 4 * q;
            uint16_t* zr = zb + (c * H + 2 * i) * W + col;
            if ((W & 3) == 0) {
#pragma unroll
                for (int dr = 0; dr < 2; ++dr) {
                    if (dr == 1 && !r1ok) break;
                    uint2 v;
                    v.x = (unsigned)__builtin_bit_cast(uint16_t, (__bf16)px[dr][0]) |
                          ((unsigned)__builtin_bit_cast(uint16_t, (__bf16)px[dr][1]) << 16);
                    v.y = (unsigned)__builtin_bit_cast(uint16_t, (__bf16)px[dr][2]) |
                          ((unsigned)__builtin_bit_cast(uint16_t, (__bf16)px[dr][3]) << 16);
                    *reinterpret_cast<uint2*>(zr + dr * W) = v;
                }
            } else {
#pragma unroll
                for (int dr = 0; dr < 2; ++dr)
#pragma unroll
                    for (int dc = 0; dc < 4; ++dc)
                        if ((dr == 0 || r1ok) && col + dc < W) zr[dr * W + dc] = __builtin_bit_cast(uint16_t, (__bf16)px[dr][dc]);
            }
        }
        __syncthreads();  // band done: slot i & 1 is free
        store_row(i & 1);  // row i + 2 (past the last row: taps 255, gradient 0)
    }
    // the 8 threads of a channel: fixed butterfly order; partials [C][B] (one slice per sample)
#pragma unroll
    for (int o = 1; o < 8; o <<= 1) {
        sg += __shfl_xor(sg, o, 64);
        sx += __shfl_xor(sx, o, 64);
    }
#undef PCX_SPB_LOAD
    if (sc_j == 0) {
        a.p_g[(int64_t)(32 * hf + sc_c) * a.B + b] = (float)sg;
        a.p_x[(int64_t)(32 * hf + sc_c) * a.B + b] = (float)sx;
    }
}

// Weight gradient from dz0 with y0 recomputed (the fused stem).  Block = a slice of samples; wave
// (mt, wt): couts 32 mt .. + 31, every other 32-pixel tile of the sample's virtual pixels (rows
// padded to WV = W rounded up to 8).  Per tile the recomputation runs transposed, C[pixel][cout] =
// im2col x W^T, so that lane (cout l32, half h) holds y0 of pixels acc_row(r, h): runs of 4
// consecutive pixels, which is also where it loads dz0 (16-byte loads) and forms dy = BN backward
// (stem_wgrad_mfma_kernel's expression, rounded to bf16) in registers.  Those 16 dy values are the A
// operand of the gradient GEMM dW[cout][tap] = sum_p dy[cout][p] x[p + tap] directly -- K-step ks
// takes registers 8 ks .. + 7, i.e. pixels 16 ks + 4 h + {0..3, 8..11} -- and the B operand (x at
// the tap offsets, fp32 LDS as stem_wgrad_mfma_kernel stages it) is read at those same pixels.  No
// transposition, no dy tile in LDS.
__global__ __launch_bounds__(256) void stem_wgrad_rc_kernel(StemArgs a) {
    extern __shared__ __attribute__((aligned(16))) float xs_f[];  // two bf16 copies of (H + 8) rows of the sample
    __bf16* xs = reinterpret_cast<__bf16*>(xs_f);
    __shared__ float red[2][32][64];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, h = lane >> 5, l32 = lane & 31;
    const int mt = wave >> 1, wt = wave & 1;
    const int H = a.H, W = a.W, HW = H * W, RW2 = st_rw2(W), CP = st_cp2(H + 8, W), WV = (W + 7) & ~7, HWV = H * WV;
    const int slice = blockIdx.x;
    const int b0 = slice * a.rows_per_blk, b1 = min(a.B, b0 + a.rows_per_blk);
    const int co = 32 * mt + l32;
    float A1, A2, A3;
    {
        const float4 k = a.cf_dy[co];
        A1 = k.x;
        A2 = -k.x * k.z;
        A3 = k.x * (k.w * k.z - k.y);
    }
    st_bf16x8 Wt[4];  // B operand of the recomputation: W^T[tap][cout], taps dh = 2 s + h, dw = j
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int dh = 2 * s + h, dw = j;
            Wt[s][j] = (__bf16)((dh < ST_K && dw < ST_K) ? a.w[co * ST_T + dh * ST_K + dw] : 0.f);
        }
    int boff[2];
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) {
        const int t = 32 * nt + l32, dh = t >> 3, dw = t & 7;
        boff[nt] = dh * RW2 + dw;
    }
    f32x16 acc[2] = {f32x16{0.f}, f32x16{0.f}};
    st2_zero(xs, H + 8, W);
    const int ntile = (HWV + 31) >> 5;
    for (int b = b0; b < b1; ++b) {
        __syncthreads();
        st2_stage(a.x + (int64_t)b * HW, H, W, xs, H + 8);
        __syncthreads();
        // dz0 (bf16) of the sample: one wave-uniform resource, the lane's cout plane in the offset
        const auto rs_g = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(a.dz16 + (int64_t)b * a.cout * HW), (short)0,
                                                            a.cout * HW * 2, 0x00020000);
        const uint16_t* gp = a.dz16 + ((int64_t)b * a.cout + co) * HW;
        // the lane's four dz0 runs of tile tt (W % 4 == 0: 8-byte loads), issued one tile ahead
        auto load_g = [&](int tt, uint2 (&gv)[4]) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int pq = tt * 32 + 8 * q + 4 * h;
                const int hh = pq / WV, ww = pq - hh * WV;
                const bool full = tt < ntile && hh < H && ww + 4 <= W;
                gv[q] = __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(
                                                      rs_g, full ? (co * HW + hh * W + ww) * 2 : 0x7fff0000, 0, 0));
            }
        };
        uint2 gnx[4];
        if ((W & 3) == 0) load_g(wt, gnx);
        for (int tt = wt; tt < ntile; tt += 2) {
            const int p0 = tt * 32;
            uint2 gcur[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) gcur[q] = gnx[q];
            if ((W & 3) == 0) load_g(tt + 2, gnx);  // in flight under this tile's MFMAs
            // y0 of pixel p0 + l32 (A operand: im2col row, taps 8 h .. 8 h + 7 of each K-step)
            f32x16 y;
            {
                const int p = min(p0 + l32, HWV - 1);
                const int hh = p / WV, ww = p - hh * WV;
                const int o = (hh + h) * RW2 + ww + 1;
                y = f32x16{0.f};
#pragma unroll
                for (int s = 0; s < 4; ++s)
                    y = __builtin_amdgcn_mfma_f32_32x32x16_bf16(st2_ld8(xs, CP, o + 2 * s * RW2), Wt[s], y, 0, 0, 0);
            }
            // the lane's four pixel runs q: p0 + 8 q + 4 h .. + 3 (one padded row each)
            int xoff[4];
            st_bf16x8 dy[2];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int pq = p0 + 8 * q + 4 * h;
                const int hh = pq / WV, ww = pq - hh * WV;
                const int nv = hh < H ? min(4, W - ww) : 0;  // real pixels of the run (<= 0: padding)
                xoff[q] = min(hh, H - 1) * RW2 + ww + 1;
                float g[4];
                if ((W & 3) == 0) {
                    const uint2 t = gcur[q];
                    g[0] = __uint_as_float(t.x << 16); g[1] = __uint_as_float(t.x & 0xffff0000u);
                    g[2] = __uint_as_float(t.y << 16); g[3] = __uint_as_float(t.y & 0xffff0000u);
                } else {
#pragma unroll
                    for (int e = 0; e < 4; ++e) g[e] = e < nv ? __uint_as_float((unsigned)gp[hh * W + ww + e] << 16) : 0.f;
                }
#pragma unroll
                for (int e = 0; e < 4; ++e)
                    dy[q >> 1][4 * (q & 1) + e] = (__bf16)(e < nv ? fmaf(A1, g[e], fmaf(A2, y[4 * q + e], A3)) : 0.f);
            }
#pragma unroll
            for (int ks = 0; ks < 2; ++ks)
#pragma unroll
                for (int nt = 0; nt < 2; ++nt) {
                    st_u32x4 bv;
                    const st_u32x2 lo = st2_ld4(xs, CP, xoff[2 * ks] + boff[nt]);
                    const st_u32x2 hi = st2_ld4(xs, CP, xoff[2 * ks + 1] + boff[nt]);
                    bv.x = lo.x; bv.y = lo.y; bv.z = hi.x; bv.w = hi.y;
                    acc[nt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(dy[ks], __builtin_bit_cast(st_bf16x8, bv), acc[nt], 0, 0, 0);
                }
        }
    }
    if (wt == 1) {
#pragma unroll
        for (int nt = 0; nt < 2; ++nt)
#pragma unroll
            for (int r = 0; r < 16; ++r) red[mt][acc_row(r, h)][32 * nt + l32] = acc[nt][r];
    }
    __syncthreads();
    if (wt == 0) {
#pragma unroll
        for (int nt = 0; nt < 2; ++nt)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int t = 32 * nt + l32, dh = t >> 3, dw = t & 7;
                if (dh < ST_K && dw < ST_K) {
                    const int c = 32 * mt + acc_row(r, h);
                    a.part[((int64_t)slice * a.cout + c) * ST_T + dh * ST_K + dw] = acc[nt][r] + red[mt][acc_row(r, h)][t];
                }
            }
    }
}

// bf16 precision, cout = 64: the stem weight gradient as a bf16 MFMA GEMM,
// dW[cout][tap] = sum over pixels dy[cout][p] x[p + tap] (K = pixels), per block a slice of samples.
// Wave w owns couts 32 (w >> 1) .. + 31 and every other 64-pixel chunk (w & 1).  dy = bf16(a dz + b y + c)
// (the BN backward, as stem_wgrad_kernel<true> rounds it) is loaded pixel-contiguous (16-byte loads),
// transposed through the wave's LDS tile [32 couts][64 pixels] and read back as the MFMA A operand
// (8 pixels per lane); B = x of the staged sample at the 8 x 8 tap grid (dh = t >> 3, dw = t & 7 for
// tap column t; dh or dw = 7 columns are dropped), 8 consecutive pixels of one image row per lane half.
// The pixel (K) index runs over rows padded to WV = W rounded up to 8 (padding columns carry dy = 0).
__global__ __launch_bounds__(256) void stem_wgrad_mfma_kernel(StemArgs a) {
    extern __shared__ __attribute__((aligned(16))) float xs[];  // (H + 8) rows of the sample
    __shared__ __attribute__((aligned(16))) __bf16 dyt[4][32][64 + 8];  // per wave (row pad: 16 bytes)
    __shared__ float red[2][32][64];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, h = lane >> 5, l32 = lane & 31;
    const int mt = wave >> 1, wt = wave & 1;
    const int H = a.H, W = a.W, HW = H * W, RW = st_rw(W), WV = (W + 7) & ~7, HWV = H * WV;
    const int slice = blockIdx.x;
    const int b0 = slice * a.rows_per_blk, b1 = min(a.B, b0 + a.rows_per_blk);
    // BN-backward coefficients of the 4 couts this lane loads per row group (lane = 16 pixel quads x 4 couts)
    const int q = lane & 15, cg = lane >> 4;  // pixel quad, cout sub-row
    float A1[8], A2[8], A3[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const float4 k = a.cf_dy[32 * mt + 4 * i + cg];
        A1[i] = k.x;
        A2[i] = -k.x * k.z;
        A3[i] = k.x * (k.w * k.z - k.y);
    }
    // B offsets of this lane's two tap columns (N-tiles nt = 0, 1: tap t = 32 nt + l32)
    int boff[2];
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) {
        const int t = 32 * nt + l32, dh = t >> 3, dw = t & 7;
        boff[nt] = dh * RW + dw;
    }
    f32x16 acc[2] = {f32x16{0.f}, f32x16{0.f}};
    for (int i = threadIdx.x; i < (H + 8) * RW; i += 256) xs[i] = 0.f;
    const int nchunk = (HWV + 63) >> 6;
    for (int b = b0; b < b1; ++b) {
        __syncthreads();
        st_stage<true>(a.x + (int64_t)b * HW, H, W, xs);
        __syncthreads();
        const int64_t pb = ((int64_t)b * a.cout + 32 * mt) * HW;
        for (int ch = wt; ch < nchunk; ch += 2) {
            const int c0 = ch * 64;
            // dy tile: lane (q, cg) loads virtual pixels c0 + 4q .. + 3 (one padded row) of couts 4i + cg
            const int pq = c0 + 4 * q;
            const int qr = pq / WV, qc = pq - qr * WV;
            const bool pv = qr < H;
            const int nv = pv ? min(4, W - qc) : 0;  // real pixels of the quad (<= 0: padding)
            const int64_t po = (int64_t)qr * W + qc;
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const int64_t o = pb + (int64_t)(4 * i + cg) * HW;
                float zz[4], yy[4];
                if ((W & 3) == 0 && nv == 4) {
                    const float4 z = ld4(a.dz + o + po), y = ld4(a.y + o + po);
                    zz[0] = z.x; zz[1] = z.y; zz[2] = z.z; zz[3] = z.w;
                    yy[0] = y.x; yy[1] = y.y; yy[2] = y.z; yy[3] = y.w;
                } else {
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        zz[e] = e < nv ? a.dz[o + po + e] : 0.f;
                        yy[e] = e < nv ? a.y[o + po + e] : 0.f;
                    }
                }
                __bf16* d = &dyt[wave][4 * i + cg][4 * q];
#pragma unroll
                for (int e = 0; e < 4; ++e) d[e] = (__bf16)(e < nv ? fmaf(A1[i], zz[e], fmaf(A2[i], yy[e], A3[i])) : 0.f);
            }
            __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the wave's LDS writes done (wave-private tile)
            __builtin_amdgcn_wave_barrier();
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                const st_bf16x8 Av = *reinterpret_cast<const st_bf16x8*>(&dyt[wave][l32][16 * s + 8 * h]);
                // this lane half's 8 virtual pixels (one padded row; past the image: dy = 0 there)
                const int p = min(c0 + 16 * s + 8 * h, HWV - 8);
                const int hh = p / WV, ww = p - hh * WV;
                const float* xb = xs + hh * RW + ww + 1;
#pragma unroll
                for (int nt = 0; nt < 2; ++nt) {
                    st_bf16x8 Bv;
#pragma unroll
                    for (int j = 0; j < 8; ++j) Bv[j] = (__bf16)xb[boff[nt] + j];
                    acc[nt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(Av, Bv, acc[nt], 0, 0, 0);
                }
            }
            __builtin_amdgcn_wave_barrier();  // (the next chunk rewrites the tile after these reads)
            __builtin_amdgcn_s_waitcnt(0xc07f);
        }
    }
    // the two waves of a cout half: fixed-order sum through LDS, then the 49 real taps to the slice
    if (wt == 1) {
#pragma unroll
        for (int nt = 0; nt < 2; ++nt)
#pragma unroll
            for (int r = 0; r < 16; ++r) red[mt][acc_row(r, h)][32 * nt + l32] = acc[nt][r];
    }
    __syncthreads();
    if (wt == 0) {
#pragma unroll
        for (int nt = 0; nt < 2; ++nt)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int t = 32 * nt + l32, dh = t >> 3, dw = t & 7;
                if (dh < ST_K && dw < ST_K) {
                    const int co = 32 * mt + acc_row(r, h);
                    a.part[((int64_t)slice * a.cout + co) * ST_T + dh * ST_K + dw] =
                        acc[nt][r] + red[mt][acc_row(r, h)][t];
                }
            }
    }
}

// float32 precision, cout = 64: the stem weight gradient on fp32 MFMA (v_mfma_f32_32x32x2_f32),
// dW[cout][tap] = sum_p dy[cout][p] x[p + tap], with stem_wgrad_mfma_kernel's waves, slices and tap
// grid.  Per 16-pixel chunk (virtual pixels over rows padded to WV = W rounded up to 8), lane (cout
// l32, half h) loads its 8 pixels p0 + 8 h .. + 7 of dz0 and y0 (16-byte loads, one chunk ahead),
// forms dy = BN backward in float32 and feeds them as the A operand of 8 K-steps (K-step ks: pixel
// p0 + 8 h + ks in lane half h); B = x at tap column 32 nt + l32 of the same pixels, 8 consecutive
// floats of one LDS row.  Products and sums in float32; only the summation order differs from
// stem_wgrad_kernel<false>.
__global__ __launch_bounds__(256) void stem_wgrad_f32_kernel(StemArgs a) {
    extern __shared__ __attribute__((aligned(16))) float xs[];  // (H + 8) rows of the sample
    __shared__ float red[2][32][64];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, h = lane >> 5, l32 = lane & 31;
    const int mt = wave >> 1, wt = wave & 1;
    const int H = a.H, W = a.W, HW = H * W, RW = st_rw(W), WV = (W + 7) & ~7, HWV = H * WV;
    const int slice = blockIdx.x;
    const int b0 = slice * a.rows_per_blk, b1 = min(a.B, b0 + a.rows_per_blk);
    const int co = 32 * mt + l32;
    float A1, A2, A3;
    {
        const float4 k = a.cf_dy[co];  // dy = a (dz - mb - (y - mean) mgi)
        A1 = k.x;
        A2 = -k.x * k.z;
        A3 = k.x * (k.w * k.z - k.y);
    }
    int boff[2];
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) {
        const int t = 32 * nt + l32, dh = t >> 3, dw = t & 7;
        boff[nt] = dh * RW + dw;
    }
    f32x16 acc[2] = {f32x16{0.f}, f32x16{0.f}};
    for (int i = threadIdx.x; i < (H + 8) * RW; i += 256) xs[i] = 0.f;
    const int nchunk = (HWV + 15) >> 4;
    for (int b = b0; b < b1; ++b) {
        __syncthreads();
        st_stage<false>(a.x + (int64_t)b * HW, H, W, xs);
        __syncthreads();
        const float* zb = a.dz + ((int64_t)b * a.cout + co) * HW;
        const float* yb = a.y + ((int64_t)b * a.cout + co) * HW;
        // the lane's run of chunk ch: 8 pixels of one padded row (nv real ones, <= 0: padding)
        auto load = [&](int ch, float (&z)[8], float (&y)[8]) {
            const int p = ch * 16 + 8 * h;
            const int hh = p / WV, ww = p - hh * WV;
            const int nv = (ch < nchunk && hh < H) ? min(8, W - ww) : 0;
            const int o = min(hh, H - 1) * W + ww;
            if ((W & 3) == 0) {  // nv is 0, 4 or 8
#pragma unroll
                for (int q = 0; q < 2; ++q) {
                    const bool v = nv >= 4 * q + 4;
                    const float4 tz = v ? ld4(zb + o + 4 * q) : make_float4(0.f, 0.f, 0.f, 0.f);
                    const float4 ty = v ? ld4(yb + o + 4 * q) : make_float4(0.f, 0.f, 0.f, 0.f);
                    z[4 * q] = tz.x; z[4 * q + 1] = tz.y; z[4 * q + 2] = tz.z; z[4 * q + 3] = tz.w;
                    y[4 * q] = ty.x; y[4 * q + 1] = ty.y; y[4 * q + 2] = ty.z; y[4 * q + 3] = ty.w;
                }
            } else {
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    z[e] = e < nv ? zb[o + e] : 0.f;
                    y[e] = e < nv ? yb[o + e] : 0.f;
                }
            }
            return nv;
        };
        float zn[8], yn[8];
        int nvn = load(wt, zn, yn);
        for (int ch = wt; ch < nchunk; ch += 2) {
            float dy[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) dy[e] = e < nvn ? fmaf(A1, zn[e], fmaf(A2, yn[e], A3)) : 0.f;
            nvn = load(ch + 2, zn, yn);  // in flight under this chunk's MFMAs
            const int p = min(ch * 16 + 8 * h, HWV - 8);
            const int hh = p / WV, ww = p - hh * WV;
            const float* xb = xs + hh * RW + ww + 1;
#pragma unroll
            for (int ks = 0; ks < 8; ++ks)
#pragma unroll
                for (int nt = 0; nt < 2; ++nt)
                    acc[nt] = __builtin_amdgcn_mfma_f32_32x32x2f32(dy[ks], xb[boff[nt] + ks], acc[nt], 0, 0, 0);
        }
    }
    // the two waves of a cout half: fixed-order sum through LDS, then the 49 real taps to the slice
    if (wt == 1) {
#pragma unroll
        for (int nt = 0; nt < 2; ++nt)
#pragma unroll
            for (int r = 0; r < 16; ++r) red[mt][acc_row(r, h)][32 * nt + l32] = acc[nt][r];
    }
    __syncthreads();
    if (wt == 0) {
#pragma unroll
        for (int nt = 0; nt < 2; ++nt)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int t = 32 * nt + l32, dh = t >> 3, dw = t & 7;
                if (dh < ST_K && dw < ST_K) {
                    const int c = 32 * mt + acc_row(r, h);
                    a.part[((int64_t)slice * a.cout + c) * ST_T + dh * ST_K + dw] = acc[nt][r] + red[mt][acc_row(r, h)][t];
                }
            }
    }
}

template <bool BF>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3))) void stem_wgrad_kernel(StemArgs a) {
    extern __shared__ __attribute__((aligned(16))) float xs[];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int H = a.H, W = a.W, HW = H * W, RW = st_rw(W);
    const int nq = (W + 3) >> 2, ntask = H * nq;
    const int slice = blockIdx.y;
    const int b0 = slice * a.rows_per_blk, b1 = min(a.B, b0 + a.rows_per_blk);  // samples of the slice
    const int cg = (blockIdx.x * 4 + wave) * ST_WCPW;
    const bool live = cg < a.cout;  // (a.cout % ST_WCPW == 0)
    float acc[ST_WCPW][ST_T];
    float A1[ST_WCPW], A2[ST_WCPW], A3[ST_WCPW];
#pragma unroll
    for (int j = 0; j < ST_WCPW; ++j) {
        const float4 k = a.cf_dy[live ? cg + j : 0];  // dy = a (dz - mb - (y - mean) mgi)
        A1[j] = k.x;
        A2[j] = -k.x * k.z;
        A3[j] = k.x * (k.w * k.z - k.y);
#pragma unroll
        for (int t = 0; t < ST_T; ++t) acc[j][t] = 0.f;
    }
    st_zero(H, W, xs);
    for (int b = b0; b < b1; ++b) {
        __syncthreads();
        st_stage<BF>(a.x + (int64_t)b * HW, H, W, xs);
        __syncthreads();
        if (!live) continue;
        const float* dzb = a.dz + ((int64_t)b * a.cout + cg) * HW;
        const float* yb = a.y + ((int64_t)b * a.cout + cg) * HW;
        // (dz, y) of the lane's next task are in flight while the current one accumulates
        float4 cz[ST_WCPW], cy[ST_WCPW];
        auto fetch = [&](int t, float4 (&z)[ST_WCPW], float4 (&y)[ST_WCPW]) {
            const int hh = t / nq, w0 = 4 * (t - hh * nq);
#pragma unroll
            for (int j = 0; j < ST_WCPW; ++j) {
                const int o = j * HW + hh * W + w0;
                if ((W & 3) == 0) {
                    z[j] = ld4(dzb + o);
                    y[j] = ld4(yb + o);
                } else {
                    z[j].x = dzb[o];
                    y[j].x = yb[o];
                    z[j].y = w0 + 1 < W ? dzb[o + 1] : 0.f;
                    y[j].y = w0 + 1 < W ? yb[o + 1] : 0.f;
                    z[j].z = w0 + 2 < W ? dzb[o + 2] : 0.f;
                    y[j].z = w0 + 2 < W ? yb[o + 2] : 0.f;
                    z[j].w = w0 + 3 < W ? dzb[o + 3] : 0.f;
                    y[j].w = w0 + 3 < W ? yb[o + 3] : 0.f;
                }
            }
        };
        if (lane < ntask) fetch(lane, cz, cy);
        for (int t = lane; t < ntask; t += 64) {
            const int hh = t / nq, w0 = 4 * (t - hh * nq);
            float dy[ST_WCPW][4];
#pragma unroll
            for (int j = 0; j < ST_WCPW; ++j) {
                const float dz[4] = {cz[j].x, cz[j].y, cz[j].z, cz[j].w};
                const float yy[4] = {cy[j].x, cy[j].y, cy[j].z, cy[j].w};
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    float d = fmaf(A1[j], dz[e], fmaf(A2[j], yy[e], A3[j]));
                    if ((W & 3) != 0 && w0 + e >= W) d = 0.f;
                    dy[j][e] = BF ? bf16r(d) : d;
                }
            }
            if (t + 64 < ntask) fetch(t + 64, cz, cy);
            // one window row at a time: 12 registers of input instead of 84
#pragma unroll
            for (int dh = 0; dh < ST_K; ++dh) {
                const float* r = xs + (hh + dh) * RW + w0;
                float v[12];
#pragma unroll
                for (int q = 0; q < 3; ++q) {
                    const float4 t4 = *reinterpret_cast<const float4*>(r + 4 * q);
                    v[4 * q] = t4.x; v[4 * q + 1] = t4.y; v[4 * q + 2] = t4.z; v[4 * q + 3] = t4.w;
                }
#pragma unroll
                for (int j = 0; j < ST_WCPW; ++j)
#pragma unroll
                    for (int k = 0; k < ST_K; ++k)
#pragma unroll
                        for (int e = 0; e < 4; ++e)
                            acc[j][dh * ST_K + k] = fmaf(dy[j][e], v[e + 1 + k], acc[j][dh * ST_K + k]);
            }
        }
    }
    if (!live) return;
#pragma unroll
    for (int j = 0; j < ST_WCPW; ++j)
#pragma unroll
        for (int t = 0; t < ST_T; ++t) {
            const float v = wave_sum(acc[j][t]);
            if (lane == 0) a.part[((int64_t)slice * a.cout + cg + j) * ST_T + t] = v;
        }
}

__global__ void round_bf16_kernel(const float* __restrict__ in, float* __restrict__ out, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = bf16r(in[i]);
}

// out[e] = sum_k part[k][e]: a block owns 32 consecutive outputs; its 8 thread groups sum slices
// g, g + 8, ... (coalesced 128-byte rows), then the 8 group sums are added in a fixed order
// (deterministic; the previous one-thread-per-output form left most of the chip idle for the
// small weight tensors: 36 blocks for a 32 x 32 x 9 gradient)
__global__ __launch_bounds__(256) void sum_slices_kernel(const float* __restrict__ part, int nslice, int64_t n,
                                                         float* __restrict__ out) {
    __shared__ float red[8][33];
    const int o = threadIdx.x & 31, g = threadIdx.x >> 5;
    const int64_t e = (int64_t)blockIdx.x * 32 + o;
    float s = 0.f;
    if (e < n) {
        int k = g;
        for (; k + 24 < nslice; k += 32) {
            const float a0 = part[(int64_t)k * n + e], a1 = part[(int64_t)(k + 8) * n + e];
            const float a2 = part[(int64_t)(k + 16) * n + e], a3 = part[(int64_t)(k + 24) * n + e];
            s += a0;
            s += a1;
            s += a2;
            s += a3;
        }
        for (; k < nslice; k += 8) s += part[(int64_t)k * n + e];
    }
    red[g][o] = s;
    __syncthreads();
    if (g == 0 && e < n) {
        float t = red[0][o];
#pragma unroll
        for (int q = 1; q < 8; ++q) t += red[q][o];
        out[e] = t;
    }
}

__global__ void pack_fwd_kernel(const float* __restrict__ w, float* __restrict__ wp, int cout, int cin) {
    int e = blockIdx.x * blockDim.x + threadIdx.x;  // e over [cout][cin][9]
    if (e >= cout * cin * 9) return;
    int n = e / (cin * 9), rem = e - n * cin * 9, c = rem / 9, t = rem - c * 9;
    wp[((int64_t)t * cin + c) * cout + n] = w[e];
}

__global__ void pack_dgrad_kernel(const float* __restrict__ w, float* __restrict__ wp, int cout, int cin) {
    int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= cout * cin * 9) return;
    int n = e / (cin * 9), rem = e - n * cin * 9, c = rem / 9, t = rem - c * 9;
    // dgrad GEMM: input channels = n (dy), output channels = c (dx), tap flipped
    wp[((int64_t)(8 - t) * cout + n) * cin + c] = w[e];
}

}  // namespace

// ====================================================================== host launchers
size_t conv3x3_nblk(int B, int H, int W, int cout) {
    int wm, wn;
    tile_shape(cout, &wm, &wn);
    int64_t M = (int64_t)B * H * W;
    return (size_t)ceil_div(M, 4 * wn * 32);
}


// forward: blocks walk samples b = block, block + nblk, ...; weight gradient: slices of samples
int stem_nblk(int B, int H, int* rows_per_blk) {
    (void)H;
    *rows_per_blk = 1;
    return std::min(B, 2048);
}

int stem_wgrad_nslice(int B, int H, int* rows_per_slice, bool mfma) {
    (void)H;
    const int sps = std::max(1, B / (mfma ? 1024 : 256));  // samples per slice (MFMA form: a block per slice)
    *rows_per_slice = sps;
    return ceil_div(B, sps);
}

static size_t stem_smem(int H, int W) { return (size_t)(H + 6) * st_rw(W) * 4; }

int launch_stem_fwd(StemArgs a, int bf16, float* wround, hipStream_t s) {
    PCX_CHECK_ARG(a.cout == 8 || a.cout == 16 || a.cout % 64 == 0 && a.cout <= 64,
                  "stem: cout %d unsupported (8, 16, 64)", a.cout);
    PCX_CHECK_ARG((int64_t)a.B * a.cout * a.H * a.W < ((int64_t)1 << 40) && stem_smem(a.H, a.W) <= 160 * 1024,
                  "stem: %dx%d input too large", a.H, a.W);
    if (bf16) {  // the GEMM's bf16 operand rounding, applied to the weights once
        const int n = a.cout * ST_T;
        round_bf16_kernel<<<ceil_div(n, 256), 256, 0, s>>>(a.w, wround, n);
        PCX_LAUNCH_CHECK("round_bf16_kernel");
        a.w = wround;
    }
    const size_t sm = stem_smem(a.H, a.W);
    if (bf16 && a.cout == 64 && (size_t)st_cp2(a.H + 7, a.W) * 4 <= 160 * 1024) {  // bf16 MFMA form
        const size_t smm = (size_t)st_cp2(a.H + 7, a.W) * 4;
        (void)hipFuncSetAttribute((const void*)stem_fwd_mfma_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)smm);
        stem_fwd_mfma_kernel<<<a.nblk, 256, smm, s>>>(a);
        PCX_LAUNCH_CHECK("stem_fwd_mfma_kernel");
        return PCX_OK;
    }
    PCX_CHECK_ARG(a.out, "stem: statistics-only pass needs the bf16 MFMA form");
    if (!bf16 && a.cout == 64 && (size_t)(a.H + 8) * st_rw(a.W) * 4 <= 128 * 1024) {  // fp32 MFMA form
        const size_t smm = (size_t)(a.H + 8) * st_rw(a.W) * 4;
        (void)hipFuncSetAttribute((const void*)stem_fwd_f32_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)smm);
        stem_fwd_f32_kernel<<<a.nblk, 256, smm, s>>>(a);
        PCX_LAUNCH_CHECK("stem_fwd_f32_kernel");
        return PCX_OK;
    }
#define PCX_STEM_F(B_, C_)                                                                          \
    if ((bf16 != 0) == B_ && a.cout == 4 * C_) {                                                    \
        (void)hipFuncSetAttribute((const void*)stem_fwd_kernel<B_, C_>,                              \
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)sm);             \
        stem_fwd_kernel<B_, C_><<<a.nblk, 256, sm, s>>>(a);                                         \
    }
    PCX_STEM_F(false, 16) PCX_STEM_F(true, 16) PCX_STEM_F(false, 4) PCX_STEM_F(true, 4)
    PCX_STEM_F(false, 2) PCX_STEM_F(true, 2)
#undef PCX_STEM_F
    PCX_LAUNCH_CHECK("stem_fwd_kernel");
    return PCX_OK;
}

bool stem_wgrad_mfma_ok(int cout, int H, int W) {  // (the bf16 and the fp32 MFMA forms)
    return cout == 64 && (size_t)(H + 8) * st_rw(W) * 4 + 48 * 1024 <= 160 * 1024;
}

static size_t stem_pool_smem(int H, int W) {
    (void)W;
    return (size_t)4 * sp_copy(H) * 2;
}

bool stem_fused_ok(int cout, int H, int W) {
    return cout == 64 && W <= 256 && stem_pool_smem(H, W) <= 80 * 1024 &&
           (size_t)st_cp2(H + 8, W) * 4 + 16 * 1024 <= 160 * 1024 &&
           maxpool3_bwd_prep_fits(H, W, (H - 1) / 2 + 1, (W - 1) / 2 + 1);
}

int launch_stem_pool(StemArgs a, hipStream_t s) {
    PCX_CHECK_ARG(stem_fused_ok(a.cout, a.H, a.W), "stem_pool: cout %d at %dx%d unsupported", a.cout, a.H, a.W);
    PCX_CHECK_ARG(a.OH == (a.H - 1) / 2 + 1 && a.OW == (a.W - 1) / 2 + 1, "stem_pool: output %dx%d for %dx%d", a.OH,
                  a.OW, a.H, a.W);
    PCX_CHECK_ARG(a.cf && a.pool_arg && a.pool_ysel, "stem_pool: missing output");
    PCX_CHECK_ARG((int64_t)2 * a.B * sp_ncb(a.OW) < ((int64_t)1 << 31), "stem_pool: batch %d too large", a.B);
    const size_t sm = stem_pool_smem(a.H, a.W);
    (void)hipFuncSetAttribute((const void*)stem_pool_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sm);
    stem_pool_kernel<<<(unsigned)(a.B * sp_ncb(a.OW)), 128, sm, s>>>(a);
    PCX_LAUNCH_CHECK("stem_pool_kernel");
    return PCX_OK;
}

int launch_stem_pool_bwd(StemArgs a, int* nslice, hipStream_t s) {
    PCX_CHECK_ARG(stem_fused_ok(a.cout, a.H, a.W), "stem_pool_bwd: cout %d at %dx%d unsupported", a.cout, a.H, a.W);
    PCX_CHECK_ARG(a.OH == (a.H - 1) / 2 + 1 && a.OW == (a.W - 1) / 2 + 1, "stem_pool_bwd: output %dx%d for %dx%d", a.OH,
                  a.OW, a.H, a.W);
    PCX_CHECK_ARG(a.dpool && a.pool_arg && a.pool_ysel && a.cf && a.dz16 && a.p_g && a.p_x,
                  "stem_pool_bwd: missing argument");
    PCX_CHECK_ARG(a.cout == 64 && a.OW <= 128 && (int64_t)2 * a.B < ((int64_t)1 << 31), "stem_pool_bwd: shape");
    *nslice = a.B;  // partials [cout][B]
    const int np_ = 32 * (a.OW + 2);
    const size_t lds = (size_t)2 * np_ * 4 + ((2 * np_ + 15) & ~15) + (size_t)np_ * 4;
    stem_pool_bwd_kernel<<<(unsigned)(2 * a.B), SPB_T, lds, s>>>(a);
    PCX_LAUNCH_CHECK("stem_pool_bwd_kernel");
    return PCX_OK;
}

int launch_stem_wgrad_rc(StemArgs a, hipStream_t s) {
    PCX_CHECK_ARG(stem_fused_ok(a.cout, a.H, a.W), "stem_wgrad_rc: cout %d at %dx%d unsupported", a.cout, a.H, a.W);
    PCX_CHECK_ARG(a.dz16 && a.cf_dy && a.part && a.nblk >= 1 && (int64_t)a.nblk * a.rows_per_blk >= a.B,
                  "stem_wgrad_rc: bad arguments");
    const size_t sm = (size_t)st_cp2(a.H + 8, a.W) * 4;
    (void)hipFuncSetAttribute((const void*)stem_wgrad_rc_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sm);
    stem_wgrad_rc_kernel<<<(unsigned)a.nblk, 256, sm, s>>>(a);
    PCX_LAUNCH_CHECK("stem_wgrad_rc_kernel");
    return PCX_OK;
}

int launch_stem_wgrad(StemArgs a, int bf16, hipStream_t s) {
    PCX_CHECK_ARG(a.cout % ST_WCPW == 0, "stem: cout %d must be even", a.cout);
    PCX_CHECK_ARG(stem_smem(a.H, a.W) <= 160 * 1024, "stem: %dx%d input too large", a.H, a.W);
    if (bf16 && stem_wgrad_mfma_ok(a.cout, a.H, a.W)) {  // bf16 MFMA form: one block per slice
        const size_t smm = (size_t)(a.H + 8) * st_rw(a.W) * 4;
        (void)hipFuncSetAttribute((const void*)stem_wgrad_mfma_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)smm);
        stem_wgrad_mfma_kernel<<<(unsigned)a.nblk, 256, smm, s>>>(a);
        PCX_LAUNCH_CHECK("stem_wgrad_mfma_kernel");
        return PCX_OK;
    }
    if (!bf16 && stem_wgrad_mfma_ok(a.cout, a.H, a.W)) {  // fp32 MFMA form: one block per slice
        const size_t smm = (size_t)(a.H + 8) * st_rw(a.W) * 4;
        (void)hipFuncSetAttribute((const void*)stem_wgrad_f32_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)smm);
        stem_wgrad_f32_kernel<<<(unsigned)a.nblk, 256, smm, s>>>(a);
        PCX_LAUNCH_CHECK("stem_wgrad_f32_kernel");
        return PCX_OK;
    }
    const size_t sm = stem_smem(a.H, a.W);
    dim3 grid((unsigned)ceil_div(a.cout, 4 * ST_WCPW), (unsigned)a.nblk);
    if (bf16) {
        (void)hipFuncSetAttribute((const void*)stem_wgrad_kernel<true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sm);
        stem_wgrad_kernel<true><<<grid, 256, sm, s>>>(a);
    } else {
        (void)hipFuncSetAttribute((const void*)stem_wgrad_kernel<false>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sm);
        stem_wgrad_kernel<false><<<grid, 256, sm, s>>>(a);
    }
    PCX_LAUNCH_CHECK("stem_wgrad_kernel");
    return PCX_OK;
}

int conv1_nblk(int B, int H, int* rows_per_blk) {
    int64_t nrows = (int64_t)B * H;
    int rpb = (int)std::max<int64_t>(1, nrows / 2048);
    *rows_per_blk = rpb;
    return ceil_div(nrows, rpb);
}

int launch_conv1_fwd(Conv1Args a, hipStream_t s) {
    PCX_CHECK_ARG(a.cout % (4 * C1F_CPW) == 0, "conv1: cout %d must be a multiple of 16", a.cout);
    PCX_CHECK_ARG((int64_t)a.B * a.H < ((int64_t)1 << 31), "conv1: too many rows");
    if (a.W % 4 == 0)
        conv1_fwd_kernel<true><<<a.nblk, 256, 0, s>>>(a);
    else
        conv1_fwd_kernel<false><<<a.nblk, 256, 0, s>>>(a);
    PCX_LAUNCH_CHECK("conv1_fwd_kernel");
    return PCX_OK;
}

// the LDS-DMA form: 32 output channels, y recomputed, rows of whole 16-byte quads that one wave's DMA covers
static bool wgrad1_dma_ok(int W, int cout) { return cout == 32 && W % 4 == 0 && W >= 4 && W <= 252; }

int wgrad1_nslice(int B, int H, int W, int cout, int* rows_per_slice) {
    const int64_t nrows = (int64_t)B * H;
    // LDS-DMA form: two resident blocks per CU (2 x 78 KB of LDS), each streaming its rows; else ~5 slices
    // per CU (the register kernel holds 5 waves per SIMD: one round of resident blocks)
    const int want = (wgrad1_dma_ok(W, cout) ? 2 : 5) * num_cus();
    *rows_per_slice = (int)std::max<int64_t>(1, (nrows + want - 1) / want);
    return ceil_div(nrows, *rows_per_slice);
}

int launch_wgrad1(Wgrad1Args a, hipStream_t s) {
    PCX_CHECK_ARG(a.cout % (4 * C1W_CPW) == 0, "wgrad1: cout must be a multiple of %d", 4 * C1W_CPW);
    PCX_CHECK_ARG((int64_t)a.B * a.H < ((int64_t)1 << 31), "wgrad1: too many rows");
    PCX_CHECK_ARG(a.y || a.w, "wgrad1: needs the conv output y or the weights to recompute it");
    PCX_CHECK_ARG(a.nslice == ceil_div((int64_t)a.B * a.H, a.rows_per_slice), "wgrad1: %d slices of %d rows",
                  a.nslice, a.rows_per_slice);
    const bool rc = a.y == nullptr;
    if (rc && wgrad1_dma_ok(a.W, a.cout) && (int64_t)32 * a.H * a.W * 4 < ((int64_t)1 << 31)) {
        const size_t lds = (size_t)2 * W1D_BUF * 4;
        (void)hipFuncSetAttribute((const void*)wgrad1_dma_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        wgrad1_dma_kernel<<<a.nslice, 256, lds, s>>>(a);
        PCX_LAUNCH_CHECK("wgrad1_dma_kernel");
        return PCX_OK;
    }
    if (a.W % 4 == 0) {
        if (rc) wgrad1_kernel<true, true><<<a.nslice, 256, 0, s>>>(a);
        else wgrad1_kernel<true, false><<<a.nslice, 256, 0, s>>>(a);
    } else {
        if (rc) wgrad1_kernel<false, true><<<a.nslice, 256, 0, s>>>(a);
        else wgrad1_kernel<false, false><<<a.nslice, 256, 0, s>>>(a);
    }
    PCX_LAUNCH_CHECK("wgrad1_kernel");
    return PCX_OK;
}

int launch_sum_slices(const float* part, int nslice, int64_t n, float* out, hipStream_t s) {
    sum_slices_kernel<<<ceil_div(n, 32), 256, 0, s>>>(part, nslice, n, out);
    PCX_LAUNCH_CHECK("sum_slices_kernel");
    return PCX_OK;
}

int launch_pack_fwd(const float* w, float* wp, int cout, int cin, hipStream_t s) {
    int n = cout * cin * 9;
    pack_fwd_kernel<<<ceil_div(n, 256), 256, 0, s>>>(w, wp, cout, cin);
    PCX_LAUNCH_CHECK("pack_fwd_kernel");
    return PCX_OK;
}

int launch_pack_dgrad(const float* w, float* wp, int cout, int cin, hipStream_t s) {
    int n = cout * cin * 9;
    pack_dgrad_kernel<<<ceil_div(n, 256), 256, 0, s>>>(w, wp, cout, cin);
    PCX_LAUNCH_CHECK("pack_dgrad_kernel");
    return PCX_OK;
}

}  // namespace pcx
