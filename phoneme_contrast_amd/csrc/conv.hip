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

__global__ __launch_bounds__(256) void conv1_fwd_kernel(Conv1Args a) {
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t HW = (int64_t)a.H * a.W;
    const int64_t nrows = (int64_t)a.B * a.H;
    const int64_t r0 = (int64_t)blockIdx.x * a.rows_per_blk;
    const int64_t r1 = min(nrows, r0 + a.rows_per_blk);
    for (int cg = wave * C1_CPW; cg < a.cout; cg += 4 * C1_CPW) {
        float wt[C1_CPW][9];
#pragma unroll
        for (int j = 0; j < C1_CPW; ++j)
#pragma unroll
            for (int t = 0; t < 9; ++t) wt[j][t] = a.w[(cg + j) * 9 + t];
        // shift for the one-pass variance: the output at the block's first pixel
        float K[C1_CPW];
        {
            int b = (int)(r0 / a.H), hh = (int)(r0 - (int64_t)b * a.H);
            float x9[9];
#pragma unroll
            for (int t = 0; t < 9; ++t) {
                int y = hh + t / 3 - 1, x = t % 3 - 1;
                x9[t] = (y >= 0 && y < a.H && x >= 0) ? a.x[(int64_t)b * HW + (int64_t)y * a.W + x] : 0.f;
            }
#pragma unroll
            for (int j = 0; j < C1_CPW; ++j) {
                float v = 0.f;
#pragma unroll
                for (int t = 0; t < 9; ++t) v = fmaf(wt[j][t], x9[t], v);
                K[j] = v;
            }
        }
        float s1[C1_CPW], s2[C1_CPW];
#pragma unroll
        for (int j = 0; j < C1_CPW; ++j) s1[j] = s2[j] = 0.f;
        for (int64_t gr = r0; gr < r1; ++gr) {
            const int b = (int)(gr / a.H), hh = (int)(gr - (int64_t)b * a.H);
            const float* xb = a.x + (int64_t)b * HW;
            for (int w = lane; w < a.W; w += 64) {
                float x9[9];
#pragma unroll
                for (int t = 0; t < 9; ++t) {
                    int y = hh + t / 3 - 1, x = w + t % 3 - 1;
                    x9[t] = (y >= 0 && y < a.H && x >= 0 && x < a.W) ? xb[(int64_t)y * a.W + x] : 0.f;
                }
#pragma unroll
                for (int j = 0; j < C1_CPW; ++j) {
                    float v = 0.f;
#pragma unroll
                    for (int t = 0; t < 9; ++t) v = fmaf(wt[j][t], x9[t], v);
                    a.out[((int64_t)b * a.cout + cg + j) * HW + (int64_t)hh * a.W + w] = v;
                    float d = v - K[j];
                    s1[j] += d;
                    s2[j] = fmaf(d, d, s2[j]);
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
__global__ __launch_bounds__(256) void wgrad1_kernel(Wgrad1Args a) {
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t HW = (int64_t)a.H * a.W;
    const int64_t nrows = (int64_t)a.B * a.H;
    const int64_t r0 = (int64_t)blockIdx.x * a.rows_per_slice;
    const int64_t r1 = min(nrows, r0 + a.rows_per_slice);
    for (int cg = wave * C1_CPW; cg < a.cout; cg += 4 * C1_CPW) {
        float acc[C1_CPW][9];
        float4 cf[C1_CPW];
#pragma unroll
        for (int j = 0; j < C1_CPW; ++j) {
            cf[j] = a.cf_dy[cg + j];
#pragma unroll
            for (int t = 0; t < 9; ++t) acc[j][t] = 0.f;
        }
        for (int64_t gr = r0; gr < r1; ++gr) {
            const int b = (int)(gr / a.H), hh = (int)(gr - (int64_t)b * a.H);
            const float* xb = a.x + (int64_t)b * HW;
            for (int w = lane; w < a.W; w += 64) {
                float x9[9];
#pragma unroll
                for (int t = 0; t < 9; ++t) {
                    int y = hh + t / 3 - 1, x = w + t % 3 - 1;
                    x9[t] = (y >= 0 && y < a.H && x >= 0 && x < a.W) ? xb[(int64_t)y * a.W + x] : 0.f;
                }
#pragma unroll
                for (int j = 0; j < C1_CPW; ++j) {
                    int64_t o = ((int64_t)b * a.cout + cg + j) * HW + (int64_t)hh * a.W + w;
                    float dy = cf[j].x * (a.dz[o] - cf[j].y - (a.y[o] - cf[j].w) * cf[j].z);
#pragma unroll
                    for (int t = 0; t < 9; ++t) acc[j][t] = fmaf(dy, x9[t], acc[j][t]);
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
    conv1_fwd_kernel<<<a.nblk, 256, 0, s>>>(a);
    PCX_LAUNCH_CHECK("conv1_fwd_kernel");
    return PCX_OK;
}

int launch_wgrad1(Wgrad1Args a, hipStream_t s) {
    PCX_CHECK_ARG(a.cout % (4 * C1_CPW) == 0, "wgrad1: cout must be a multiple of 32");
    wgrad1_kernel<<<a.nslice, 256, 0, s>>>(a);
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
