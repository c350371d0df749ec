// Shared epilogue of the 3x3 conv kernels (conv.hip, conv_dma.hip): stores / BN statistics
// (forward) or ReLU / MaxPool / Dropout backward + BN-backward sums (data gradient).
#pragma once
#include "kernels.h"

namespace pcx {

__device__ __forceinline__ float conv_sum32(float v) {  // reduce within each 32-lane half
#pragma unroll
    for (int o = 16; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// Transposed butterfly: v[r] (r < 16) summed over the 32 lanes of each half-wave in 16 shuffles
// (instead of 16 x 5).  Lane l of a half returns the total of r = (l >> 1) & 15.  `sel` gets the
// same lane-bit selection applied to a half-uniform array (no shuffles): sel = u[(l >> 1) & 15].
__device__ __forceinline__ float xsum16(const float (&v)[16], int l32) {
    // (named scalars at every level: selects between elements of a local array became one dynamically indexed
    // load, which kept the array in scratch -- 16 stores and an indexed scratch load per call: round 6)
    const bool b4 = l32 & 16, b3 = l32 & 8, b2 = l32 & 4, b1 = l32 & 2;
#define PCX_X8(j) const float w8_##j = (b4 ? v[j + 8] : v[j]) + __shfl_xor(b4 ? v[j] : v[j + 8], 16, 64);
    PCX_X8(0) PCX_X8(1) PCX_X8(2) PCX_X8(3) PCX_X8(4) PCX_X8(5) PCX_X8(6) PCX_X8(7)
#undef PCX_X8
    const float w4_0 = (b3 ? w8_4 : w8_0) + __shfl_xor(b3 ? w8_0 : w8_4, 8, 64);
    const float w4_1 = (b3 ? w8_5 : w8_1) + __shfl_xor(b3 ? w8_1 : w8_5, 8, 64);
    const float w4_2 = (b3 ? w8_6 : w8_2) + __shfl_xor(b3 ? w8_2 : w8_6, 8, 64);
    const float w4_3 = (b3 ? w8_7 : w8_3) + __shfl_xor(b3 ? w8_3 : w8_7, 8, 64);
    const float w2_0 = (b2 ? w4_2 : w4_0) + __shfl_xor(b2 ? w4_0 : w4_2, 4, 64);
    const float w2_1 = (b2 ? w4_3 : w4_1) + __shfl_xor(b2 ? w4_1 : w4_3, 4, 64);
    const float w1 = (b1 ? w2_1 : w2_0) + __shfl_xor(b1 ? w2_0 : w2_1, 2, 64);
    return w1 + __shfl_xor(w1, 1, 64);
}
// select u[(l32 >> 1) & 15] with the butterfly's lane bits (named scalars, elements made opaque: as xsum16)
__device__ __forceinline__ float xsel16(const float (&u)[16], int l32) {
    const bool b4 = l32 & 16, b3 = l32 & 8, b2 = l32 & 4, b1 = l32 & 2;
#define PCX_S8(j)                                  \
    float lo_##j = u[j], hi_##j = u[j + 8];        \
    asm("" : "+v"(lo_##j), "+v"(hi_##j));          \
    const float w8_##j = b4 ? hi_##j : lo_##j;
    PCX_S8(0) PCX_S8(1) PCX_S8(2) PCX_S8(3) PCX_S8(4) PCX_S8(5) PCX_S8(6) PCX_S8(7)
#undef PCX_S8
    const float w4_0 = b3 ? w8_4 : w8_0, w4_1 = b3 ? w8_5 : w8_1, w4_2 = b3 ? w8_6 : w8_2, w4_3 = b3 ? w8_7 : w8_3;
    const float w2_0 = b2 ? w4_2 : w4_0, w2_1 = b2 ? w4_3 : w4_1;
    return b1 ? w2_1 : w2_0;
}
__device__ __forceinline__ float readlane_f(float v, int l) {
    return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), l));
}

template <int WM, int WN, int EPI>
__device__ __forceinline__ void conv_epilogue(const ConvArgs& a, f32x16 (&acc)[WM][WN], float* red,
                                              int tile, int n0, int64_t m0, int64_t Mtot, int64_t HW,
                                              int wave, int tid, const bool (&valid)[WN],
                                              const int (&pb)[WN], const int (&pp)[WN]) {
    constexpr int COUT_T = 32 * WM;
    const int lane = tid & 63, h = lane >> 5, l32 = lane & 31;
    const int cnt_w = (int)max((int64_t)0, min((int64_t)WN * 32, Mtot - (m0 + wave * WN * 32)));
    if (EPI == EPI_FWD) {
        // store y; per (wave, channel) Chan statistics shifted by the channel's first pixel of the
        // half-wave (K, read with v_readlane), reduced with the transposed butterfly
        float* ob[WN];
#pragma unroll
        for (int ni = 0; ni < WN; ++ni) ob[ni] = a.out + ((int64_t)pb[ni] * a.cout + n0 + 4 * h) * HW + pp[ni];
#pragma unroll
        for (int mi = 0; mi < WM; ++mi) {
            float kv[16], s1[16], s2[16];
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const float k0 = readlane_f(acc[mi][0][r], 0), k1 = readlane_f(acc[mi][0][r], 32);
                kv[r] = h ? k1 : k0;
                const int64_t co = (int64_t)(mi * 32 + (r & 3) + 8 * (r >> 2)) * HW;
                s1[r] = 0.f;
                s2[r] = 0.f;
#pragma unroll
                for (int ni = 0; ni < WN; ++ni) {
                    const float v = acc[mi][ni][r];
                    if (valid[ni]) {
                        ob[ni][co] = v;
                        const float d = v - kv[r];
                        s1[r] += d;
                        s2[r] = fmaf(d, d, s2[r]);
                    }
                }
            }
            const float t1 = xsum16(s1, l32), t2 = xsum16(s2, l32), K = xsel16(kv, l32);
            if (!(l32 & 1)) {
                const float n = (float)cnt_w;
                const float mean = cnt_w ? K + t1 / n : 0.f;
                const float m2 = cnt_w ? fmaxf(t2 - t1 * t1 / n, 0.f) : 0.f;
                float* d = red + (wave * COUT_T + mi * 32 + acc_row(l32 >> 1, h)) * 3;
                d[0] = n; d[1] = mean; d[2] = m2;
            }
        }
        __syncthreads();
        if (tid < COUT_T) {
            float n = 0.f, mean = 0.f, m2 = 0.f;
#pragma unroll
            for (int w = 0; w < 4; ++w) {
                const float* d = red + (w * COUT_T + tid) * 3;
                if (d[0] > 0.f) {
                    float nt = n + d[0];
                    float delta = d[1] - mean;
                    mean += delta * d[0] / nt;
                    m2 += d[2] + delta * delta * n * d[0] / nt;
                    n = nt;
                }
            }
            a.part0[(int64_t)(n0 + tid) * a.nblk + tile] = n * mean;
            a.part1[(int64_t)(n0 + tid) * a.nblk + tile] = m2;
            if (tid == 0 && n0 == 0) a.partn[tile] = n;
        }
    } else if (EPI == EPI_BWD_STORE) {
        // plain data gradient (cnn_deep routes its stride-1 3x3 convs here): store or accumulate
#pragma unroll
        for (int ni = 0; ni < WN; ++ni) {
            if (!valid[ni]) continue;
            float* op = a.out + ((int64_t)pb[ni] * a.cout + n0 + 4 * h) * HW + pp[ni];
#pragma unroll
            for (int mi = 0; mi < WM; ++mi)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    float* o = op + (int64_t)(mi * 32 + (r & 3) + 8 * (r >> 2)) * HW;
                    *o = a.accumulate ? *o + acc[mi][ni][r] : acc[mi][ni][r];
                }
        }
    } else {
        // backward epilogues: sums of dz and dz*xhat per channel.  The global loads of RB
        // accumulator rows are issued as one batch before any of their stores: the compiler must
        // assume a store may alias a later load, so row-by-row code paid one full memory round
        // trip per accumulator row.  Invalid pixels were clamped to the last valid one by the
        // caller, so every batched address is in bounds.
#ifndef PCX_EPI_RB_RELU
#define PCX_EPI_RB_RELU 4
#endif
#ifndef PCX_EPI_RB_POOL
#define PCX_EPI_RB_POOL 2
#endif
        constexpr int RB = (EPI == EPI_BWD_RELU) ? PCX_EPI_RB_RELU : PCX_EPI_RB_POOL;
        // per-channel coefficients staged in LDS once (the accumulator loop is free of them)
        float4* cfl = reinterpret_cast<float4*>(red + 4 * COUT_T * 3);
        if (tid < COUT_T) cfl[tid] = a.cf_out[n0 + tid];
        __syncthreads();
        int64_t base[WN];
#pragma unroll
        for (int ni = 0; ni < WN; ++ni) {
            if (EPI == EPI_BWD_RELU) {
                base[ni] = ((int64_t)pb[ni] * a.cout + n0) * HW + pp[ni];
            } else {
                const int hp = pp[ni] / a.W, wp = pp[ni] - hp * a.W;
                base[ni] = ((int64_t)pb[ni] * a.cout + n0) * a.Hs * a.Ws + (int64_t)(2 * hp) * a.Ws + 2 * wp;
            }
        }
        const int chs = (EPI == EPI_BWD_RELU) ? (int)HW : a.Hs * a.Ws;  // channel-plane stride
#pragma unroll
        for (int mi = 0; mi < WM; ++mi) {
            float sz[16], sx[16];
#pragma unroll
            for (int rb = 0; rb < 16; rb += RB) {
                constexpr int NY = (EPI == EPI_BWD_RELU) ? 1 : 4;
                float yv[RB][WN][NY], dv[RB][WN];
#pragma unroll
                for (int j = 0; j < RB; ++j) {
                    const int chl = mi * 32 + acc_row(rb + j, h);
#pragma unroll
                    for (int ni = 0; ni < WN; ++ni) {
                        const float* yp = a.yprev + base[ni] + (int64_t)chl * chs;
                        yv[j][ni][0] = yp[0];
                        if (EPI == EPI_BWD_POOL) {
                            yv[j][ni][1] = yp[1];
                            yv[j][ni][2] = yp[a.Ws];
                            yv[j][ni][3] = yp[a.Ws + 1];
                            dv[j][ni] = a.drop_out ? a.drop_out[(int64_t)pb[ni] * a.cout + n0 + chl] : 1.f;
                        }
                    }
                }
#pragma unroll
                for (int j = 0; j < RB; ++j) {
                const int r = rb + j;
                const int chl = mi * 32 + acc_row(r, h);
                const float4 cf = cfl[chl];
                float sdz = 0.f, sdx = 0.f;
#pragma unroll
                for (int ni = 0; ni < WN; ++ni) {
                    if (!valid[ni]) continue;
                    const float g = acc[mi][ni][r];
                    float* op = a.out + base[ni] + (int64_t)chl * chs;
                    if (EPI == EPI_BWD_RELU) {
                        const float y = yv[j][ni][0];
                        float dz = (fmaf(y, cf.x, cf.y) > 0.f) ? g : 0.f;
                        op[0] = dz;
                        sdz += dz;
                        sdx = fmaf(dz, (y - cf.z) * cf.w, sdx);
                    } else {  // EPI_BWD_POOL
                        const float gd = g * dv[j][ni];
                        const float y0 = yv[j][ni][0], y1 = yv[j][ni][1], y2 = yv[j][ni][2], y3 = yv[j][ni][3];
                        float r0 = fmaxf(fmaf(y0, cf.x, cf.y), 0.f), r1 = fmaxf(fmaf(y1, cf.x, cf.y), 0.f);
                        float r2 = fmaxf(fmaf(y2, cf.x, cf.y), 0.f), r3 = fmaxf(fmaf(y3, cf.x, cf.y), 0.f);
                        // first maximum in window scan order, as torch's max_pool2d
                        int arg = 0;
                        float best = r0, ya = y0;
                        if (r1 > best) { best = r1; arg = 1; ya = y1; }
                        if (r2 > best) { best = r2; arg = 2; ya = y2; }
                        if (r3 > best) { best = r3; arg = 3; ya = y3; }
                        float d = best > 0.f ? gd : 0.f;
                        op[0] = arg == 0 ? d : 0.f;
                        op[1] = arg == 1 ? d : 0.f;
                        op[a.Ws] = arg == 2 ? d : 0.f;
                        op[a.Ws + 1] = arg == 3 ? d : 0.f;
                        sdz += d;
                        sdx = fmaf(d, (ya - cf.z) * cf.w, sdx);
                    }
                }
                sz[r] = sdz;
                sx[r] = sdx;
                }
            }
            const float tz = xsum16(sz, l32), tx = xsum16(sx, l32);
            if (!(l32 & 1)) {
                float* d = red + (wave * COUT_T + mi * 32 + acc_row(l32 >> 1, h)) * 2;
                d[0] = tz; d[1] = tx;
            }
        }
        __syncthreads();
        if (tid < COUT_T) {
            float s0 = 0.f, s1 = 0.f;
#pragma unroll
            for (int w = 0; w < 4; ++w) {
                s0 += red[(w * COUT_T + tid) * 2];
                s1 += red[(w * COUT_T + tid) * 2 + 1];
            }
            a.part0[(int64_t)(n0 + tid) * a.nblk + tile] = s0;
            a.part1[(int64_t)(n0 + tid) * a.nblk + tile] = s1;
        }
    }
}

}  // namespace pcx
