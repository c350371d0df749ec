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

// ------------------------------------------------------------------ Cin = 1 first conv
constexpr int C1_CPW = 8;  // output channels per wave

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
    for (int cg = wave * C1_CPW; cg < a.cout; cg += 4 * C1_CPW) {
        float wt[C1_CPW][9];
#pragma unroll
        for (int j = 0; j < C1_CPW; ++j)
#pragma unroll
            for (int t = 0; t < 9; ++t) wt[j][t] = a.w[(cg + j) * 9 + t];
        // shift for the one-pass variance: the output at the block's first pixel
        float K[C1_CPW];
        {
            const int b = r0 / a.H, hh = r0 - b * a.H;
            float xr[3][6];
            c1_window<false>(a.x + (int64_t)b * HW, a.H, a.W, hh, 0, xr);
#pragma unroll
            for (int j = 0; j < C1_CPW; ++j) {
                float v = 0.f;
#pragma unroll
                for (int t = 0; t < 9; ++t) v = fmaf(wt[j][t], xr[t / 3][1 + t % 3 - 1], v);
                K[j] = v;
            }
        }
        float s1[C1_CPW], s2[C1_CPW];
#pragma unroll
        for (int j = 0; j < C1_CPW; ++j) s1[j] = s2[j] = 0.f;
        for (int t = lane; t < ntask; t += 64) {
            const int rr = t / nq, q = t - rr * nq;
            const int gr = r0 + rr, b = gr / a.H, hh = gr - b * a.H;
            const int w0 = 4 * q;
            float xr[3][6];
            c1_window<FULL>(a.x + (int64_t)b * HW, a.H, a.W, hh, w0, xr);
            float* ob = a.out + ((int64_t)b * a.cout + cg) * HW + (int64_t)hh * a.W + w0;
#pragma unroll
            for (int j = 0; j < C1_CPW; ++j) {
                float v[4];
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    float acc = 0.f;
#pragma unroll
                    for (int tp = 0; tp < 9; ++tp) acc = fmaf(wt[j][tp], xr[tp / 3][e + tp % 3], acc);
                    v[e] = acc;
                }
                if (FULL) {
                    st4(ob + (int64_t)j * HW, make_float4(v[0], v[1], v[2], v[3]));
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
        for (int j = 0; j < C1_CPW; ++j) {
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
// HBM-read-bound (dz and y are read once).  Partials per slice.
template <bool FULL>
__global__ __launch_bounds__(256) void wgrad1_kernel(Wgrad1Args a) {
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int HW = a.H * a.W;
    const int nrows = a.B * a.H;
    const int r0 = blockIdx.x * a.rows_per_slice;
    const int r1 = min(nrows, r0 + a.rows_per_slice);
    const int nq = (a.W + 3) >> 2;
    const int ntask = (r1 - r0) * nq;
    for (int cg = wave * C1_CPW; cg < a.cout; cg += 4 * C1_CPW) {
        float acc[C1_CPW][9];
        float A1[C1_CPW], A2[C1_CPW], A3[C1_CPW];
#pragma unroll
        for (int j = 0; j < C1_CPW; ++j) {
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
            for (int j = 0; j < C1_CPW; ++j) {
                float dz[4], yy[4];
                if (FULL) {
                    const float4 u = ld4(a.dz + o + (int64_t)j * HW), v = ld4(a.y + o + (int64_t)j * HW);
                    dz[0] = u.x; dz[1] = u.y; dz[2] = u.z; dz[3] = u.w;
                    yy[0] = v.x; yy[1] = v.y; yy[2] = v.z; yy[3] = v.w;
                }
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    if (!FULL) {
                        const bool ok = w0 + e < a.W;
                        dz[e] = ok ? a.dz[o + (int64_t)j * HW + e] : 0.f;
                        yy[e] = ok ? a.y[o + (int64_t)j * HW + e] : 0.f;
                    }
                    float dy = fmaf(A1[j], dz[e], fmaf(A2[j], yy[e], A3[j]));
                    if (!FULL && w0 + e >= a.W) dy = 0.f;
#pragma unroll
                    for (int tp = 0; tp < 9; ++tp) acc[j][tp] = fmaf(dy, xr[tp / 3][e + tp % 3], acc[j][tp]);
                }
            }
        }
#pragma unroll
        for (int j = 0; j < C1_CPW; ++j)
#pragma unroll
            for (int t = 0; t < 9; ++t) {
                float v = wave_sum(acc[j][t]);
                if (lane == 0) a.part[((int64_t)blockIdx.x * a.cout + cg + j) * 9 + t] = v;
            }
    }
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


int conv1_nblk(int B, int H, int* rows_per_blk) {
    int64_t nrows = (int64_t)B * H;
    int rpb = (int)std::max<int64_t>(1, nrows / 2048);
    *rows_per_blk = rpb;
    return ceil_div(nrows, rpb);
}

int launch_conv1_fwd(Conv1Args a, hipStream_t s) {
    PCX_CHECK_ARG(a.cout % (4 * C1_CPW) == 0, "conv1: cout %d must be a multiple of 32", a.cout);
    PCX_CHECK_ARG((int64_t)a.B * a.H < ((int64_t)1 << 31), "conv1: too many rows");
    if (a.W % 4 == 0)
        conv1_fwd_kernel<true><<<a.nblk, 256, 0, s>>>(a);
    else
        conv1_fwd_kernel<false><<<a.nblk, 256, 0, s>>>(a);
    PCX_LAUNCH_CHECK("conv1_fwd_kernel");
    return PCX_OK;
}

int launch_wgrad1(Wgrad1Args a, hipStream_t s) {
    PCX_CHECK_ARG(a.cout % (4 * C1_CPW) == 0, "wgrad1: cout must be a multiple of 32");
    PCX_CHECK_ARG((int64_t)a.B * a.H < ((int64_t)1 << 31), "wgrad1: too many rows");
    if (a.W % 4 == 0)
        wgrad1_kernel<true><<<a.nslice, 256, 0, s>>>(a);
    else
        wgrad1_kernel<false><<<a.nslice, 256, 0, s>>>(a);
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
