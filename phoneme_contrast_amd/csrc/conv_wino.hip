// 3x3 / stride 1 / pad 1 convolution (forward and data gradient) as Winograd F(2x2, 3x3) on fp32
// MFMA (v_mfma_f32_16x16x4_f32).  Same contract as conv3x3_dma (ConvArgs, prologues, epilogues),
// 16 multiplies per 2x2 output tile instead of 36: 4/9 of the direct conv's MFMA work, all of it
// in exact fp32 (the transforms are additions; the weight transform is evaluated in float64).
//
//   Y = A^T [ U (.) V ] A,   U = G g G^T (weights, once per call),   V = B^T d B (4x4 input patch)
//
// Per Winograd element xi (16 of them) the tile contraction is a GEMM over input channels:
// M_xi[cout][tile] = sum_c U_xi[cout][c] V_xi[c][tile].  MFMA orientation: A = U (16 couts x 4
// channels), B = V (4 channels x 16 tiles), so lane l owns the (channel l >> 4, tile l & 15)
// patch: it reads the 4x4 patch from LDS, applies the producer's BN + ReLU, transforms it in
// registers and feeds the 16 values to 16 MFMAs (x 2 cout sub-tiles).  The accumulators of lane l
// hold, for every xi, the same (cout, tile) positions, so the output transform is also per lane.
//
// Layout / staging (MI355X-first):
//  * persistent workgroups (two per CU) walk units = (64 consecutive tiles of one sample in row-major
//    tile order, 32 output channels); consecutive units (neighbouring rows, the other channel groups
//    of the same tiles) run on one XCD, so the halo rows they share come from that XCD's L2 -- taken
//    in order from a per-XCD work queue (ConvArgs::queue, round 4) so that the workgroups do not drift
//    apart over a launch; narrow images (W < 31) use units of 64 consecutive tiles of the whole batch
//    (SP: a wave's 16 tiles in up to 4 row segments of one or more samples);
//  * wave w owns tiles 16 w .. 16 w + 15 of the unit: one or two row segments of one or two tile
//    rows.  Its LDS slot holds, per input channel, the 4 input rows of those segments side by side
//    (<= 36 columns), so every patch of the wave is a 4 x 4 window of one slot at a per-lane column;
//  * the slot of a K-chunk (CK channels) is copied HBM/L2 -> LDS by buffer_load_dword ... lds with
//    per-lane offsets computed once per unit (the channel is the buffer base), double buffered
//    across chunks and units (the next unit's first chunk lands during this unit's last chunk and
//    epilogue); out-of-image positions carry an out-of-range offset and copy a 0 (BN+ReLU operands
//    of border waves are zeroed again after the prologue by per-row / per-column factors);
//  * slot plane stride = 32 mod 64 floats: the 32 lanes of a ds_read_b64 group (16 consecutive
//    tiles x 2 channels) cover the 64 banks once;
//  * transformed weights U are packed [cout / 32][cin][4][32][4] (xi = 4 q + e innermost), one
//    contiguous run per K-chunk: dwordx4 DMA, conflict-free ds_read_b128 A operands;
//  * epilogue: the 16 lanes of a row hold 16 consecutive tiles, so output rows are stored (and the
//    producer's y / pooled windows loaded) as 128- / 256-byte runs.
#include <cstdlib>
#include <type_traits>

#include "conv_epilogue.h"
#include "pk_f32.h"

namespace pcx {
namespace {

typedef __attribute__((address_space(3))) void lds_void;

typedef float f2 __attribute__((ext_vector_type(2)));

// n / d for 0 <= n < 2^22 with inv = 1 / d (float): one correction step makes it exact
__device__ __forceinline__ int wdiv(int n, int d, float inv) {
    int q = (int)((float)n * inv);
    const int r = n - q * d;
    q += r >= d ? 1 : 0;
    q -= r < 0 ? 1 : 0;
    return q;
}

__device__ __forceinline__ f32x4 mfma16(float a, float b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// global -> LDS copy (saddr form): global = uniform base + per-lane byte offset, LDS = M0 + lane * 4 * VEC
template <int VEC>
__device__ __forceinline__ void wdma(const float* sbase, unsigned voff, unsigned lds_byte_addr) {
    const unsigned m0 = __builtin_amdgcn_readfirstlane(lds_byte_addr);
    if constexpr (VEC == 4)
        asm volatile("s_nop 0\n\tglobal_load_lds_dwordx4 %0, %1" :: "v"(voff), "s"(sbase), "{m0}"(m0) : "memory");
    else
        asm volatile("s_nop 0\n\tglobal_load_lds_dword %0, %1" :: "v"(voff), "s"(sbase), "{m0}"(m0) : "memory");
}

__device__ __forceinline__ const float* wuniform(const float* p) {
    const uint64_t v = (uint64_t)(uintptr_t)p;
    const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)v);
    const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(v >> 32));
    return (const float*)(uintptr_t)(((uint64_t)hi << 32) | lo);
}

// per-wave staging slot: CK channel planes of 4 rows x WSW columns (two row segments: the wave's
// 16 tiles in row-major order span at most two tile rows), plane stride WSP = 32 mod 64 floats
constexpr int WSW = 36, WSP = 160;

// LDS DMA of one dword per lane from a buffer resource (out-of-range offsets write 0);
// LDS destination = M0 + 4 * lane.
__device__ __forceinline__ void bdma(__amdgpu_buffer_rsrc_t r, unsigned voff, unsigned lds_byte_addr) {
    const unsigned m0 = __builtin_amdgcn_readfirstlane(lds_byte_addr);
    asm volatile("s_nop 0\n\tbuffer_load_dword %0, %1, 0 offen lds" :: "v"(voff), "s"(r), "{m0}"(m0) : "memory");
}

// LDS DMA of 16 bytes per lane (the source may be any 4-byte aligned address: measured,
// profiles/r4_probe_dma_align.txt); LDS destination = M0 + 16 * lane.  Past num_records the range
// check is per dword (profiles/r4_probe_dma_oob.txt).
__device__ __forceinline__ void bdma4(__amdgpu_buffer_rsrc_t r, unsigned voff, unsigned lds_byte_addr) {
    const unsigned m0 = __builtin_amdgcn_readfirstlane(lds_byte_addr);
    asm volatile("s_nop 0\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds" :: "v"(voff), "s"(r), "{m0}"(m0) : "memory");
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t wrsrc(const float* base, int bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), (short)0, bytes, 0x00020000);
}

// sum over the 16 lanes of a row (lanes sharing l >> 4)
__device__ __forceinline__ float row16_sum(float v) {
    v += __shfl_xor(v, 1, 64);
    v += __shfl_xor(v, 2, 64);
    v += __shfl_xor(v, 4, 64);
    v += __shfl_xor(v, 8, 64);
    return v;
}
// transposed butterfly: v[j] (j < 8) summed over the 16 lanes of a row in 8 shuffles; lane n
// returns the total of j = (n >> 1) & 7
// (every element passes an empty asm first: a select between two loads of a local array was otherwise turned
// into one dynamically indexed load, which kept the array in scratch -- a store per element and a scratch load
// per unit in the forward epilogue)
__device__ __forceinline__ float opq(float x) {
    asm("" : "+v"(x));
    return x;
}
__device__ __forceinline__ float row16_xsum8(const float (&v)[8], int n) {
    const bool b3 = n & 8, b2 = n & 4, b1 = n & 2;
    const float a0 = (b3 ? v[4] : v[0]) + __shfl_xor(b3 ? v[0] : v[4], 8, 64);
    const float a1 = (b3 ? v[5] : v[1]) + __shfl_xor(b3 ? v[1] : v[5], 8, 64);
    const float a2 = (b3 ? v[6] : v[2]) + __shfl_xor(b3 ? v[2] : v[6], 8, 64);
    const float a3 = (b3 ? v[7] : v[3]) + __shfl_xor(b3 ? v[3] : v[7], 8, 64);
    const float c0 = (b2 ? a2 : a0) + __shfl_xor(b2 ? a0 : a2, 4, 64);
    const float c1 = (b2 ? a3 : a1) + __shfl_xor(b2 ? a1 : a3, 4, 64);
    const float w1 = (b1 ? c1 : c0) + __shfl_xor(b1 ? c0 : c1, 2, 64);
    return w1 + __shfl_xor(w1, 1, 64);
}

// select v[(n >> 1) & 7] with the butterfly's lane bits (no shuffles)
__device__ __forceinline__ float row16_xsel8(const float (&v)[8], int n) {
    const bool b3 = n & 8, b2 = n & 4, b1 = n & 2;
    float w[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) w[j] = opq(v[j]);
    const float a0 = b3 ? w[4] : w[0], a1 = b3 ? w[5] : w[1], a2 = b3 ? w[6] : w[2], a3 = b3 ? w[7] : w[3];
    const float c0 = b2 ? a2 : a0, c1 = b2 ? a3 : a1;
    return b1 ? c1 : c0;
}


// Branch-free epilogue stores (round 5): a guarded global store (`if (ok) p[i] = v`) compiles to an exec-mask
// branch per store -- 16 to 64 per unit, ~11-40 % of the conv's time in the epilogue knock-outs
// (profiles/r5_wino_knockouts.txt).  Instead every store is a buffer store relative to the wave's first
// output plane: lanes keep byte offsets, an element outside the image gets an offset past num_records (the
// hardware drops the store), the channel's plane offset rides in soffset.
constexpr unsigned WOOB = 0x80000000u;  // masked element offset (> every num_records used)
// epilogue stores stream (cache policy nt on gfx950; round 6): every output tensor is GBs, read by the next kernel
constexpr int WST = PCX_AB_NO_NT_STORES ? 0 : 2;
typedef unsigned u32x2w __attribute__((ext_vector_type(2)));
typedef unsigned u32x4w __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void bst1(__amdgpu_buffer_rsrc_t r, unsigned vo, int so, float x) {
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, x), r, vo, so, WST);
}
__device__ __forceinline__ void bst2(__amdgpu_buffer_rsrc_t r, unsigned vo, int so, float x, float y) {
    __builtin_amdgcn_raw_buffer_store_b64(u32x2w{__builtin_bit_cast(unsigned, x), __builtin_bit_cast(unsigned, y)}, r,
                                          vo, so, WST);
}
__device__ __forceinline__ void bst4(__amdgpu_buffer_rsrc_t r, unsigned vo, int so, float x, float y, float z, float w) {
    __builtin_amdgcn_raw_buffer_store_b128(u32x4w{__builtin_bit_cast(unsigned, x), __builtin_bit_cast(unsigned, y),
                                                  __builtin_bit_cast(unsigned, z), __builtin_bit_cast(unsigned, w)},
                                           r, vo, so, WST);
}
__device__ __forceinline__ float2 bld2(__amdgpu_buffer_rsrc_t r, unsigned vo, int so) {
    const u32x2w t = __builtin_amdgcn_raw_buffer_load_b64(r, vo, so, 0);
    const unsigned t0 = t.x, t1 = t.y;  // (named copies: no bit_cast of a vector-lane lvalue)
    return make_float2(__builtin_bit_cast(float, t0), __builtin_bit_cast(float, t1));
}
__device__ __forceinline__ float bld1(__amdgpu_buffer_rsrc_t r, unsigned vo, int so) {
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, vo, so, 0));
}

// True in the last of the block's 4 waves to call it for this unit (an LDS counter at red + 514, reset by that
// wave): the wave's scratch writes are complete before it counts itself in.
__device__ __forceinline__ bool last_wave(float* red, int lane) {
    int* cnt = reinterpret_cast<int*>(red + 514);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    int v = 0;
    if (lane == 0) v = atomicAdd(cnt, 1);
    v = __builtin_amdgcn_readfirstlane(v);
    if (v != 3) return false;
    if (lane == 0) *cnt = 0;
    return true;
}

// Epilogue of one unit.  Lane (n, kq) holds output channels n0 + 16 mi + 4 kq + i (j = 4 mi + i < 8)
// of its tile (outputs y[j][e] at (2 tr + (e >> 1), 2 tc + (e & 1))).  The 16 lanes of a row hold
// 16 consecutive tiles of one or two tile rows, so a store of one output row is a 128-byte run.
// red: 512 floats of LDS private to the epilogue.
template <int EPI, bool V4, bool POOL>
__device__ __forceinline__ void wino_epilogue(const ConvArgs& a, const float (&y)[8][4], float* red, const float4* cfl, int b,
                                              int tb, int n0, int tr, int tc, bool tvalid, int wave, int tid) {
    const int lane = tid & 63, n = lane & 15, kq = lane >> 4;
    const int HW = a.H * a.W;
    const int h0 = 2 * tr, w0 = 2 * tc;
    const bool okr1 = h0 + 1 < a.H, okc1 = w0 + 1 < a.W;
    const bool vec = (a.W & 1) == 0;  // output pairs (h, w0..w0+1) are 8-byte aligned and complete
    bool ok[4];
    ok[0] = tvalid;
    ok[1] = tvalid && okc1;
    ok[2] = tvalid && okr1;
    ok[3] = ok[1] && okr1;
    const int pix0 = h0 * a.W + w0;
    const int poff[4] = {0, 1, a.W, a.W + 1};
    const int jsel = (n >> 1) & 7;                               // channel this lane reduces
    const int cosel = 16 * (jsel >> 2) + 4 * kq + (jsel & 3);
    // store bases: the wave's first sample bw (lane 0 holds the wave's first tile; host-checked 32-bit offsets)
    const int bw = __builtin_amdgcn_readfirstlane(b);
    const int lpl = (b - bw) * a.cout + 4 * kq;  // the lane's channel-4kq plane relative to the wave's first
    auto wrs = [&](const void* base, int hw, int esz) {  // tensor [B][cout][hw] of esz-byte elements
        const int64_t rest = ((int64_t)(a.B - bw) * a.cout - n0) * hw * esz;
        const int nrec = rest <= 0 ? 0 : (int)(rest < 0x7ffffff0 ? rest : 0x7ffffff0);
        const float* p = reinterpret_cast<const float*>(static_cast<const char*>(base) +
                                                        ((int64_t)bw * a.cout + n0) * hw * esz);
        return wrsrc(wuniform(p), __builtin_amdgcn_readfirstlane(nrec));
    };
    // channel j's plane offset (bytes, uniform)
    auto chs = [&](int j, int hwb) { return __builtin_amdgcn_readfirstlane((16 * (j >> 2) + (j & 3)) * hwb); };
    unsigned oe[4];  // conv-resolution byte offsets of the lane's 4 outputs (channel 4 kq), masked
#pragma unroll
    for (int e = 0; e < 4; ++e) oe[e] = ok[e] ? 4u * (unsigned)(lpl * HW + pix0 + poff[e]) : WOOB;
    if (EPI == EPI_FWD) {
        // store y; per channel Chan statistics of the block: each wave sums about a shift K (the
        // channel's first output in its row of lanes), reduced with the transposed butterfly
        const __amdgpu_buffer_rsrc_t rs = wrs(a.out, HW, 4);
        float cnt = 0.f;
#pragma unroll
        for (int e = 0; e < 4; ++e) cnt += ok[e] ? 1.f : 0.f;
        // (round 6: the shifted sums packed over channel pairs j, j + 1 -- the register pairs the packed output
        // transform produced -- with the validity as a 0 / 1 factor: 15 packed instructions per two channels
        // instead of 32 scalar ones; the outputs of invalid tiles are finite)
        const PkK pk = pk_consts();
        float s1[8], s2[8], kv[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int so = chs(j, 4 * HW);
            const float* v = y[j];
            if (vec) {
                bst2(rs, oe[0], so, v[0], v[1]);
                bst2(rs, oe[2], so, v[2], v[3]);
            } else {
#pragma unroll
                for (int e = 0; e < 4; ++e) bst1(rs, oe[e], so, v[e]);
            }
            kv[j] = __shfl(v[0], lane & 48, 64);
        }
#pragma unroll
        for (int j = 0; j < 8; j += 2) {
            const pk_f2 kk = {kv[j], kv[j + 1]};
            pk_f2 t = {0.f, 0.f}, q = {0.f, 0.f};
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const float m = ok[e] ? 1.f : 0.f;
                const pk_f2 d = pk_sub(pk, pk_f2{y[j][e], y[j + 1][e]}, kk) * pk_f2{m, m};
                t = e ? t + d : d;
                q = e ? __builtin_elementwise_fma(d, d, q) : d * d;
            }
            s1[j] = t.x; s1[j + 1] = t.y;
            s2[j] = q.x; s2[j + 1] = q.y;
        }
        const float T1 = row16_xsum8(s1, n), T2 = row16_xsum8(s2, n);
        const float K = row16_xsel8(kv, n);
        cnt = row16_sum(cnt);
        if (!(n & 1)) {
            float* d = red + (wave * 32 + cosel) * 3;
            d[0] = T1; d[1] = T2; d[2] = K;
        }
        if (lane == 0) red[384 + wave] = cnt;  // valid outputs of the wave (all channels alike)
        if constexpr (POOL) {
            // (round 6) the consumer block's 2x2 max-pool selection, made here: a tile IS a pooling window (H, W
            // even, host-checked).  relu(s y + t) with s = gamma invstd is monotone in y with the sign of gamma,
            // so the window's first maximum of relu(BN(y)) -- torch max_pool2d's rule, bn_relu_pool_kernel's --
            // is the first maximum of y (gamma > 0), the first minimum (gamma < 0), or the first element (gamma
            // 0: all equal), wherever that maximum is positive; where it is not, the pooled value and every
            // gradient through it are 0 whichever element is recorded.  Writes y at the selected element and
            // its index at the pooled resolution (ysel / parg: the backward's EPI_BWD_POOLSEL inputs); the
            // pooled activation is then one light pass over ysel (pool_act_kernel) instead of bn_relu_pool's
            // full-resolution read of y.  sgn: the LDS table of sign(gamma) per output channel.
            const float* sgn = reinterpret_cast<const float*>(cfl);
            const int HWp = (a.H >> 1) * (a.W >> 1);
            const __amdgpu_buffer_rsrc_t rsy = wrs(a.pool_ysel, HWp, 4), rsa = wrs(a.pool_arg, HWp, 1);
            const unsigned pe = (unsigned)(lpl * HWp + tr * (a.W >> 1) + tc);
            const unsigned oy = tvalid ? 4u * pe : WOOB, oa = tvalid ? pe : WOOB;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const float sg = sgn[n0 + 16 * (j >> 2) + 4 * kq + (j & 3)];
                float best = y[j][0] * sg, ys = y[j][0];
                unsigned arg = 0;
#pragma unroll
                for (int e = 1; e < 4; ++e) {
                    const float z = y[j][e] * sg;
                    const bool gt = z > best;
                    best = gt ? z : best;
                    ys = gt ? y[j][e] : ys;
                    arg = gt ? (unsigned)e : arg;
                }
                bst1(rsy, oy, chs(j, 4 * HWp), ys);
                __builtin_amdgcn_raw_buffer_store_b8((unsigned char)arg, rsa, oa, chs(j, HWp), 0);
            }
        }
        // the last of the block's 4 waves to get here merges the 4 waves' statistics (round 6: no block barrier;
        // a __syncthreads here cost 3-6 % of the forward convs, profiles/r6_wino_epilogue_barrier.txt).  The
        // scratch is safe to reuse: every wave passes the next unit's first chunk barrier only after this merge.
        if (last_wave(red, lane)) {
            const int c = lane;
            float nn = 0.f, mean = 0.f, m2 = 0.f;
#pragma unroll
            for (int w = 0; w < 4; ++w) {
                const float nw = red[384 + w];
                if (nw > 0.f) {
                    const float* d = red + (w * 32 + c) * 3;
                    const float rw = __builtin_amdgcn_rcpf(nw);  // 1-ulp reciprocals (statistics)
                    const float mw = d[2] + d[0] * rw, m2w = fmaxf(d[1] - d[0] * d[0] * rw, 0.f);
                    const float nt = nn + nw, delta = mw - mean, f = nw * __builtin_amdgcn_rcpf(nt);
                    mean += delta * f;
                    m2 += m2w + delta * delta * nn * f;
                    nn = nt;
                }
            }
            if (c < 32) {
                a.part0[(int64_t)(n0 + c) * a.nblk + tb] = nn * mean;
                a.part1[(int64_t)(n0 + c) * a.nblk + tb] = m2;
                if (c == 0 && n0 == 0) a.partn[tb] = nn;
            }
        }
    } else if (EPI == EPI_BWD_STORE) {
        const __amdgpu_buffer_rsrc_t rs = wrs(a.out, HW, 4);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int so = chs(j, 4 * HW);
            const float* v = y[j];
            if (vec) {
#pragma unroll
                for (int rr = 0; rr < 2; ++rr) {
                    float2 t = make_float2(v[2 * rr], v[2 * rr + 1]);
                    if (a.accumulate) {  // (masked loads read 0)
                        const float2 p = bld2(rs, oe[2 * rr], so);
                        t.x += p.x;
                        t.y += p.y;
                    }
                    bst2(rs, oe[2 * rr], so, t.x, t.y);
                }
            } else {
#pragma unroll
                for (int e = 0; e < 4; ++e) bst1(rs, oe[e], so, a.accumulate ? bld1(rs, oe[e], so) + v[e] : v[e]);
            }
        }
    } else {
        // data-gradient epilogues: dz through ReLU (and MaxPool / Dropout2d) of the producer, and the
        // producer BN's backward sums (dz, dz * xhat) per channel
        float sz[8], sx[8];
        if (EPI == EPI_BWD_RELU) {
            // all loads first (masked elements read 0), then the arithmetic and the stores: one memory
            // round trip per unit instead of one per channel
            const __amdgpu_buffer_rsrc_t ry = wrs(a.yprev, HW, 4);
            float4 cf[8];
            float yy[8][4];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int co = 16 * (j >> 2) + 4 * kq + (j & 3);
                const int so = chs(j, 4 * HW);
                cf[j] = cfl[n0 + co];
                if (vec) {
                    const float2 p0 = bld2(ry, oe[0], so), p1 = bld2(ry, oe[2], so);
                    yy[j][0] = p0.x; yy[j][1] = p0.y; yy[j][2] = p1.x; yy[j][3] = p1.y;
                } else {
#pragma unroll
                    for (int e = 0; e < 4; ++e) yy[j][e] = bld1(ry, oe[e], so);
                }
            }
            const __amdgpu_buffer_rsrc_t rs = wrs(a.out, HW, 4);
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int so = chs(j, 4 * HW);
                float dz[4], s_z = 0.f, s_x = 0.f;
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    dz[e] = (ok[e] && fmaf(yy[j][e], cf[j].x, cf[j].y) > 0.f) ? y[j][e] : 0.f;
                    s_z += dz[e];
                    s_x = fmaf(dz[e], (yy[j][e] - cf[j].z) * cf[j].w, s_x);
                }
                if (vec) {
                    bst2(rs, oe[0], so, dz[0], dz[1]);
                    bst2(rs, oe[2], so, dz[2], dz[3]);
                } else {
#pragma unroll
                    for (int e = 0; e < 4; ++e) bst1(rs, oe[e], so, dz[e]);
                }
                sz[j] = s_z;
                sx[j] = s_x;
            }
        } else if (EPI == EPI_BWD_POOLSEL || EPI == EPI_BWD_POOLSELP) {
            constexpr bool PO = EPI == EPI_BWD_POOLSELP;
            // the pooled data gradient from the forward's recorded selection: y at each window's selected
            // element and its index (bn_relu_pool_kernel), read at the conv's (pooled) resolution -- a
            // quarter of the full-resolution window reads; dz written at Hs x Ws as EPI_BWD_POOL does
            const int HWs = a.Hs * a.Ws;
            const __amdgpu_buffer_rsrc_t ry = wrs(a.ysel, HW, 4), ra = wrs(a.parg, HW, 1);
            const __amdgpu_buffer_rsrc_t ro = wrs(PO ? static_cast<const void*>(a.dpool) : a.out, PO ? HW : HWs, 4);
            unsigned ob[4], os[4];  // parg byte offsets; full-resolution window offsets (row r0, column c0)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                ob[e] = ok[e] ? (unsigned)(lpl * HW + pix0 + poff[e]) : WOOB;
                os[e] = ok[e] ? 4u * (unsigned)(lpl * HWs + (2 * h0 + 2 * (e >> 1)) * a.Ws + 2 * w0 + 2 * (e & 1)) : WOOB;
            }
#pragma unroll
            for (int half = 0; half < 2; ++half) {
                // four channels' loads together (one round trip per batch; registers)
                float ys[4][4], dv[4];
                unsigned ag[4];
                float4 cf[4];
#pragma unroll
                for (int jj = 0; jj < 4; ++jj) {
                    const int j = 4 * half + jj;
                    const int co = 16 * (j >> 2) + 4 * kq + (j & 3);
                    const int so = chs(j, 4 * HW), sb = chs(j, HW);
                    cf[jj] = cfl[n0 + co];
                    dv[jj] = a.drop_out ? a.drop_out[(int64_t)b * a.cout + n0 + co] : 1.f;
                    if (vec) {
                        const float2 p0 = bld2(ry, oe[0], so), p1 = bld2(ry, oe[2], so);
                        ys[jj][0] = p0.x; ys[jj][1] = p0.y; ys[jj][2] = p1.x; ys[jj][3] = p1.y;
                        ag[jj] = (unsigned)__builtin_amdgcn_raw_buffer_load_b16(ra, ob[0], sb, 0) |
                                 ((unsigned)__builtin_amdgcn_raw_buffer_load_b16(ra, ob[2], sb, 0) << 16);
                    } else {
                        ag[jj] = 0;
#pragma unroll
                        for (int e = 0; e < 4; ++e) {
                            ys[jj][e] = bld1(ry, oe[e], so);
                            ag[jj] |= (unsigned)__builtin_amdgcn_raw_buffer_load_b8(ra, ob[e], sb, 0) << (8 * e);
                        }
                    }
                }
#pragma unroll
                for (int jj = 0; jj < 4; ++jj) {
                    const int j = 4 * half + jj;
                    const float4 k = cf[jj];
                    float dzw[4][4], dde[4];
                    float s_z = 0.f, s_x = 0.f;
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        const int r0 = 2 * (e >> 1), c0 = 2 * (e & 1);
                        const float ya = ys[jj][e];
                        // the window's maximum of relu(BN) is positive iff the selected element's BN output is
                        const float dd = (ok[e] && fmaf(ya, k.x, k.y) > 0.f) ? y[j][e] * dv[jj] : 0.f;
                        dde[e] = dd;
                        if constexpr (!PO) {
                            const unsigned arg = (ag[jj] >> (8 * e)) & 3u;
                            dzw[r0][c0] = arg == 0 ? dd : 0.f;
                            dzw[r0][c0 + 1] = arg == 1 ? dd : 0.f;
                            dzw[r0 + 1][c0] = arg == 2 ? dd : 0.f;
                            dzw[r0 + 1][c0 + 1] = arg == 3 ? dd : 0.f;
                        }
                        s_z += dd;
                        s_x = fmaf(dd, (ya - k.z) * k.w, s_x);
                    }
                    if constexpr (PO) {
                        // EPI_BWD_POOLSELP: the consumer rebuilds the windows from parg -- the routed
                        // gradient at the pooled resolution only (a quarter of the full-resolution writes)
                        const int so = chs(j, 4 * HW);
                        if (vec) {
                            bst2(ro, oe[0], so, dde[0], dde[1]);
                            bst2(ro, oe[2], so, dde[2], dde[3]);
                        } else {
#pragma unroll
                            for (int e = 0; e < 4; ++e) bst1(ro, oe[e], so, dde[e]);
                        }
                    } else {
                        const int so = chs(j, 4 * HWs);
                        if constexpr (V4) {  // (H, W even: ok[e] == tvalid; the window rows are 16-byte runs)
#pragma unroll
                            for (int r = 0; r < 4; ++r)
                                bst4(ro, os[0] + (r == 0 ? 0u : 4u * (unsigned)(r * a.Ws)), so, dzw[r][0], dzw[r][1],
                                     dzw[r][2], dzw[r][3]);
                        } else {
#pragma unroll
                            for (int e = 0; e < 4; ++e) {  // (dword stores: odd Ws leaves rows 4-byte aligned)
                                const int r0 = 2 * (e >> 1), c0 = 2 * (e & 1);
                                const unsigned o1 = os[e] + 4u * (unsigned)a.Ws;
                                bst1(ro, os[e], so, dzw[r0][c0]);
                                bst1(ro, os[e] + 4u, so, dzw[r0][c0 + 1]);
                                bst1(ro, o1, so, dzw[r0 + 1][c0]);
                                bst1(ro, o1 + 4u, so, dzw[r0 + 1][c0 + 1]);
                            }
                        }
                    }
                    sz[j] = s_z;
                    sx[j] = s_x;
                }
            }
        } else {  // EPI_BWD_POOL: the conv runs at the pooled resolution; dz lives at Hs x Ws
            const int HWs = a.Hs * a.Ws;
            constexpr int PB = V4 ? 1 : 2;  // channels per batch of window loads (registers)
            const int soff0 = tvalid ? (2 * h0) * a.Ws + 2 * w0 : 0;  // loads clamped in bounds
            const float* yb = a.yprev + ((int64_t)b * a.cout + n0) * HWs + soff0;
            const __amdgpu_buffer_rsrc_t ro = wrs(a.out, HWs, 4);
            unsigned os[4];  // full-resolution window offsets (row r0, column c0), masked
#pragma unroll
            for (int e = 0; e < 4; ++e)
                os[e] = ok[e] ? 4u * (unsigned)(lpl * HWs + (2 * h0 + 2 * (e >> 1)) * a.Ws + 2 * w0 + 2 * (e & 1)) : WOOB;
#pragma unroll
            for (int half = 0; half < 8 / PB; ++half) {
                // PB channels' windows loaded together (one round trip per batch; registers)
                float win[PB][4][4];
                float4 cf[PB];
                float dv[PB];
#pragma unroll
                for (int jj = 0; jj < PB; ++jj) {
                    const int j = PB * half + jj;
                    const int co = 16 * (j >> 2) + 4 * kq + (j & 3);
                    cf[jj] = cfl[n0 + co];
                    dv[jj] = a.drop_out ? a.drop_out[(int64_t)b * a.cout + n0 + co] : 1.f;
                    const float* yp = yb + (int64_t)co * HWs;
                    if (V4) {  // host-checked: H, W even, Ws % 4 == 0: a tile's window is four 16-byte rows
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            const float4 t = ld4(yp + r * a.Ws);
                            win[jj][r][0] = t.x; win[jj][r][1] = t.y; win[jj][r][2] = t.z; win[jj][r][3] = t.w;
                        }
                    } else {
#pragma unroll
                        for (int e = 0; e < 4; ++e) {
                            const int r0 = 2 * (e >> 1), c0 = 2 * (e & 1);
                            const float* q = yp + (ok[e] ? r0 * a.Ws + c0 : 0);
                            const int dc = ok[e] ? 1 : 0, dr = ok[e] ? a.Ws : 0;
                            win[jj][r0][c0] = q[0];
                            win[jj][r0][c0 + 1] = q[dc];
                            win[jj][r0 + 1][c0] = q[dr];
                            win[jj][r0 + 1][c0 + 1] = q[dr + dc];
                        }
                    }
                }
#pragma unroll
                for (int jj = 0; jj < PB; ++jj) {
                    const int j = PB * half + jj;
                    float dzw[4][4];
                    float s_z = 0.f, s_x = 0.f;
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        const int r0 = 2 * (e >> 1), c0 = 2 * (e & 1);
                        const float y0 = win[jj][r0][c0], y1 = win[jj][r0][c0 + 1];
                        const float y2 = win[jj][r0 + 1][c0], y3 = win[jj][r0 + 1][c0 + 1];
                        const float4 k = cf[jj];
                        const float q0 = fmaxf(fmaf(y0, k.x, k.y), 0.f), q1 = fmaxf(fmaf(y1, k.x, k.y), 0.f);
                        const float q2 = fmaxf(fmaf(y2, k.x, k.y), 0.f), q3 = fmaxf(fmaf(y3, k.x, k.y), 0.f);
                        // first maximum in window scan order, as torch's max_pool2d
                        int arg = 0;
                        float best = q0, ya = y0;
                        if (q1 > best) { best = q1; arg = 1; ya = y1; }
                        if (q2 > best) { best = q2; arg = 2; ya = y2; }
                        if (q3 > best) { best = q3; arg = 3; ya = y3; }
                        const float dd = (ok[e] && best > 0.f) ? y[j][e] * dv[jj] : 0.f;
                        dzw[r0][c0] = arg == 0 ? dd : 0.f;
                        dzw[r0][c0 + 1] = arg == 1 ? dd : 0.f;
                        dzw[r0 + 1][c0] = arg == 2 ? dd : 0.f;
                        dzw[r0 + 1][c0 + 1] = arg == 3 ? dd : 0.f;
                        s_z += dd;
                        s_x = fmaf(dd, (ya - k.z) * k.w, s_x);
                    }
                    const int so = chs(j, 4 * HWs);
                    if (V4) {
#pragma unroll
                        for (int r = 0; r < 4; ++r)
                            bst4(ro, os[0] + (r == 0 ? 0u : 4u * (unsigned)(r * a.Ws)), so, dzw[r][0], dzw[r][1],
                                 dzw[r][2], dzw[r][3]);
                    } else {
#pragma unroll
                        for (int e = 0; e < 4; ++e) {
                            const int r0 = 2 * (e >> 1), c0 = 2 * (e & 1);
                            const unsigned o1 = os[e] + 4u * (unsigned)a.Ws;
                            bst1(ro, os[e], so, dzw[r0][c0]);
                            bst1(ro, os[e] + 4u, so, dzw[r0][c0 + 1]);
                            bst1(ro, o1, so, dzw[r0 + 1][c0]);
                            bst1(ro, o1 + 4u, so, dzw[r0 + 1][c0 + 1]);
                        }
                    }
                    sz[j] = s_z;
                    sx[j] = s_x;
                }
                __builtin_amdgcn_sched_barrier(0);  // keep the pairs' loads apart (registers)
            }
        }
        const float tz = row16_xsum8(sz, n), tx = row16_xsum8(sx, n);
        if (!(n & 1)) {
            red[(wave * 32 + cosel) * 2] = tz;
            red[(wave * 32 + cosel) * 2 + 1] = tx;
        }
        if (last_wave(red, lane)) {  // (as the forward: the last wave sums, no block barrier)
            const int c = lane & 31;
            float s0 = 0.f, s1 = 0.f;
#pragma unroll
            for (int w = 0; w < 4; ++w) {
                s0 += red[(w * 32 + c) * 2];
                s1 += red[(w * 32 + c) * 2 + 1];
            }
            if (lane < 32) {
                a.part0[(int64_t)(n0 + c) * a.nblk + tb] = s0;
                a.part1[(int64_t)(n0 + c) * a.nblk + tb] = s1;
            }
        }
    }
}

// (WINO_KO bits, analysis builds only: 1 no operand copies, 2 no epilogue, 4 no chunk sync, 8 no BN + ReLU)
// Persistent: each workgroup walks units u = it * G + (XCD-contiguous slot); unit = (64-tile block tb
// of one sample, 32-channel output group cg).  The first K-chunk of the next unit is copied while the
// last chunk of the current one is multiplied and during its epilogue.
// X4 (round 4): the operand slot is copied by 16-byte DMAs -- 5 per chunk of 8 channels instead of 24
// dword copies; a slot row is 40 floats (segment B starts on a 16-byte granule), the 4-byte-aligned
// sources of the granules straddle the image's left / right edges, and the out-of-image columns they
// bring in (the neighbouring rows' values) are zeroed by selects in the border waves, for every prologue.
// Needs 4 readable bytes before a.src (ConvArgs::src_guard: the plans carve a guard at the workspace start).
template <int PRO, int EPI, int CK, bool V4, bool X4, bool SP = false, bool POOL = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void conv_wino_kernel(ConvArgs a, WinoGeo g) {
    static_assert(!POOL || (EPI == EPI_FWD && !SP), "pooled selection: forward epilogue, per-sample units");
    static_assert(!X4 || CK == 8, "16-byte staging covers whole 8-channel chunks");
    static_assert(!SP || X4, "spanning units stage by 16-byte copies");
    constexpr int WROW = X4 ? 40 : WSW;       // slot row width (floats)
    constexpr int NCP = X4 ? 5 : 3;           // copy offsets per lane
    constexpr int WSLOT = CK * WSP + 32;      // floats of one wave's slot (+ the last plane's overflow)
    constexpr int INF = 4 * WSLOT;            // input floats per buffer
    constexpr int BUFF = INF + CK * 512;      // + transformed weights of the chunk
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int tid = threadIdx.x, lane = tid & 63, n = lane & 15, kq = lane >> 4;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int HW = a.H * a.W;
    const PkK pk = pk_consts();
    float* cft = smem + 2 * BUFF;             // [cin] float2 {s, t}
    float* red = cft + 2 * a.cin;             // epilogue scratch (512 floats + the queue slots and the counter)
    // data-gradient epilogues: the producer BN's coefficients per output channel, read from LDS (round 6: eight
    // 16-byte global loads per unit and lane, with their 64-bit address arithmetic, exposed at the unit's end)
    constexpr bool CFL = EPI != EPI_FWD && EPI != EPI_BWD_STORE;
    float4* cfl = reinterpret_cast<float4*>(red + 516);
    if (CFL)
        for (int c = tid; c < a.cout; c += 256) cfl[c] = a.cf_out[c];
    if (POOL)  // the pooled selection's sign(gamma) per output channel, in the same LDS slot
        for (int c = tid; c < a.cout; c += 256) {
            const float gm = a.pool_gamma[c];
            reinterpret_cast<float*>(cfl)[c] = gm > 0.f ? 1.f : gm < 0.f ? -1.f : 0.f;
        }
    const unsigned lds0 = (unsigned)(uintptr_t)(lds_void*)smem;
    if (PRO != PRO_RAW)
        for (int c = tid; c < a.cin; c += 256) {
            const float4 f = a.cf_in[c];
            cft[2 * c] = f.x;
            cft[2 * c + 1] = f.y;
        }
    if (tid == 0) reinterpret_cast<int*>(red + 514)[0] = 0;  // the epilogue's last-wave counter
    const int nunits = (SP ? g.nblk : a.B * g.BPS) * g.ncg;
    const int G = gridDim.x;
    // XCD-contiguous slot of this workgroup inside a round (dispatch is round-robin over the 8 XCDs)
    const int slot = ((G & 7) || g.naive_slots) ? (int)blockIdx.x : (int)(blockIdx.x & 7) * (G >> 3) + (int)(blockIdx.x >> 3);
    // Unit queue (a.queue): the static order u = it G + slot lets the workgroups drift apart over the
    // ~250 rounds of a B = 4096 launch, and the halo rows two neighbouring units share then miss the XCD's
    // L2 (L2-miss bytes 2.1x the input at B = 4096 against 1.3x at B = 512: profiles/r4_wino_l2_order.txt).
    // With the queue each XCD's workgroups take the units of one contiguous eighth of the launch in
    // order from that XCD's counter (then help the other XCDs), so neighbours are in flight together.
    const int nq = (a.queue && !(G & 7)) ? 8 : 1;
    int* qsl = reinterpret_cast<int*>(red + 512);  // [2]: the next unit, by unit parity
    // (queue q covers units [q nunits / nq, (q + 1) nunits / nq): nq is 1 or 8 and nunits < 2^22 (host-checked),
    // so a shift, not the 64-bit division the compiler emitted for `/ nq` -- ~150 scalar instructions per grab)
    const int lq = nq == 8 ? 3 : 0;
    auto grab = [&]() -> int {  // lane 0 of wave 0 only
        const int x0 = nq == 8 ? (int)(blockIdx.x & 7) : 0;
        for (int k = 0; k < nq; ++k) {
            const int q = (x0 + k) & (nq - 1);
            const int lo = (q * nunits) >> lq, len = (((q + 1) * nunits) >> lq) - lo;
            const int v = atomicAdd(a.queue + 32 * q, 1);
            if (v < len) return lo + v;
        }
        return nunits;
    };

    struct Unit { int b, tb, cg, tw, tr_a, tc_a; };
    // (wave-uniform divisions by float reciprocals: a few VALU instead of ~30 per integer division)
    auto unit_of = [&](int u) {
        Unit x;
        x.tb = wdiv(u, g.ncg, g.inv_ncg);
        x.cg = u - x.tb * g.ncg;
        if constexpr (SP) {  // tw = the wave's first tile in the batch-wide tile order
            x.tw = x.tb * 64 + wave * 16;
            x.b = wdiv(x.tw, g.NTS, g.inv_NTS);
            const int rem = x.tw - x.b * g.NTS;
            x.tr_a = wdiv(rem, g.TC, g.inv_TC);
            x.tc_a = rem - x.tr_a * g.TC;
        } else {
            x.b = wdiv(x.tb, g.BPS, g.inv_BPS);
            x.tw = (x.tb - x.b * g.BPS) * 64 + wave * 16;  // the wave's first tile (within its sample)
            x.tr_a = wdiv(x.tw, g.TC, g.inv_TC);
            x.tc_a = x.tw - x.tr_a * g.TC;
        }
        return x;
    };
    // SP: the wave's 16 tiles as up to 4 row segments (rows of one or more samples) placed side by side
    // in the slot row, each on its own 16-byte granule: segment s = tiles st[s] .. st[s] + len[s] - 1 of
    // the wave, image row pair tr[s] of sample b[s], slot column p[s]; rows past the batch get len 0
    struct Segs { int st[4], len[4], p[4], b[4], tr[4]; };
    auto segs_of = [&](const Unit& x) {
        Segs S;
        int j = 0, pc = 0, b = x.b, tr = x.tr_a, tc = x.tc_a;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int len = min(16 - j, g.TC - tc);
            const int lv = b < a.B ? len : 0;
            S.st[q] = j; S.len[q] = lv; S.p[q] = pc; S.b[q] = b; S.tr[q] = tr;
            pc += lv > 0 ? ((2 * lv + 2 + 3) & ~3) : 0;
            j += len;
            tc = 0;
            if (++tr == g.TR) { tr = 0; ++b; }
        }
        return S;
    };
    // Copies: per channel plane three 64-lane dword copies cover slot positions 0..191: 0..143 are
    // the 4 rows x WSW columns, 144..191 (out-of-range offsets: zeros) run into the next plane's
    // first 32 positions, which that plane's copies, issued later by the same wave, overwrite (a
    // wave's loads land in issue order); the last plane runs into the slot's 32-float tail.  Lane
    // offsets depend on the unit only (the channel is the buffer base); out-of-image positions get
    // an out-of-range offset, which copies a 0.  (No exec masking next to in-flight MFMAs.)
    unsigned voff[NCP];
    auto plan_copies = [&](const Unit& x) {
        if constexpr (SP) {
            // granule gi = 64 j + lane: plane gi / 40, row (gi % 40) / 10, slot column 4 (gi % 10) -> segment by
            // slot column; offsets relative to a.src + (b cin + c0) HW - 1 (b = the unit's first sample)
            const Segs S = segs_of(x);
#pragma unroll
            for (int j = 0; j < NCP; ++j) {
                const int gi = 64 * j + lane, pl = gi / 40, gg = gi - pl * 40, r = gg / 10, sc = 4 * (gg - r * 10);
                int q = 0;
#pragma unroll
                for (int t = 1; t < 4; ++t) q += (S.len[t] > 0 && sc >= S.p[t]) ? 1 : 0;
                int len = S.len[0], p0 = S.p[0], bq = S.b[0], trq = S.tr[0];
#pragma unroll
                for (int t = 1; t < 4; ++t)
                    if (q == t) { len = S.len[t]; p0 = S.p[t]; bq = S.b[t]; trq = S.tr[t]; }
                const int cs = sc - p0, grow = 2 * trq - 1 + r, gcol = (q == 0 ? 2 * x.tc_a - 1 : -1) + cs;
                const bool ok = len > 0 && cs < 2 * len + 2 && (unsigned)grow < (unsigned)a.H;
                voff[j] = ok ? 4u * (unsigned)((bq - x.b) * a.cin * HW + pl * HW + grow * a.W + gcol + 1) : 0x80000000u;
            }
            return;
        }
        const int len_a = min(16, g.TC - x.tc_a);
        const int segw = 2 * len_a + 2;
        const int rb0 = 2 * x.tr_a - 1, rb1 = 2 * x.tr_a + 1;
        const int cb0 = 2 * x.tc_a - 1, cb1 = -segw - 1;
        if constexpr (X4) {
            // granule gi = 64 j + lane of the chunk: plane gi / 40, row (gi % 40) / 10, slot column 4 (gi % 10);
            // offsets relative to a.src + (b cin + c0) HW - 1 (the granule of image column -1 starts in range)
            // (branch-free: with short-circuit && the compiler put the offset multiply under exec-mask branches,
            // ~50 instructions per copy offset and unit; here every term is evaluated and one select picks)
            const int SB = (segw + 3) & ~3, segwB = 2 * (16 - len_a) + 2;
            const bool twoseg = len_a < 16;
#pragma unroll
            for (int j = 0; j < NCP; ++j) {
                const int gi = 64 * j + lane, pl = gi / 40, gg = gi - pl * 40, r = gg / 10, sc = 4 * (gg - r * 10);
                const bool sB = sc >= SB;
                const int grow = r + (sB ? rb1 : rb0), gcol = sB ? sc - SB - 1 : cb0 + sc;
                const bool colok = sB ? (twoseg & (sc - SB < segwB)) : (sc < segw);
                const bool ok = ((unsigned)grow < (unsigned)a.H) & colok;
                const unsigned off = 4u * (unsigned)(pl * HW + grow * a.W + gcol + 1);
                voff[j] = ok ? off : 0x80000000u;
            }
            return;
        }
#pragma unroll
        for (int p = 0; p < 3; ++p) {
            const int pos = 64 * p + lane;
            const int r = pos / WSW, cc = pos - r * WSW;
            const bool s1 = cc >= segw;
            const int grow = r + (s1 ? rb1 : rb0), gcol = cc + (s1 ? cb1 : cb0);
            const bool ok = (unsigned)grow < (unsigned)a.H && (unsigned)gcol < (unsigned)a.W;
            voff[p] = (pos < 4 * WSW && ok) ? 4u * (unsigned)(grow * a.W + gcol) : 0x80000000u;
        }
    };
    // part p of NP: channel planes [p CK / NP, (p + 1) CK / NP) and the matching share of the weight
    // copies (the copies of a chunk are spread over its K-steps: the TA takes a dword copy's 64
    // addresses at a few per clock, and a burst of them stalls the issuing wave in order)
    auto issue = [&](const Unit& x, int c0, int buf, int part, int np) {
#if defined(WINO_KO) && (WINO_KO & 1)  // analysis builds only (tools/wino_ko.sh): no operand copies
        return;
#endif
        const float* sb = a.src + ((int64_t)x.b * a.cin + c0) * HW;
        const unsigned sl = lds0 + 4u * (unsigned)(buf * BUFF + wave * WSLOT);
        if constexpr (X4) {  // 5 granule copies per chunk: parts of 3 + 2
            // (SP: the following samples' planes too, up to the end of the batch)
            // (a wave past the batch has every offset out of range: num_records 1 keeps them so)
            int nrec = CK * HW + 1;
            if constexpr (SP) {
                const int64_t rest = (int64_t)(a.B - x.b) * a.cin * HW - (int64_t)c0 * HW + 1;
                nrec = rest < 1 ? 1 : rest > 0x1ffffff0 ? 0x1ffffff0 : (int)rest;
            }
            const __amdgpu_buffer_rsrc_t r = wrsrc(sb - 1, 4 * nrec);
            const int j0 = part == 0 ? 0 : 3, j1 = np == 1 ? NCP : (part == 0 ? 3 : NCP);
#pragma unroll
            for (int j = 0; j < NCP; ++j)
                if (j >= j0 && j < j1) bdma4(r, voff[j], sl + 1024u * (unsigned)j);
        }
        const int cpp = X4 ? 0 : CK / np;
#pragma unroll
        for (int ci = 0; ci < cpp; ++ci) {
            const int cl = part * cpp + ci;
            const __amdgpu_buffer_rsrc_t r = wrsrc(sb + (int64_t)cl * HW, 4 * HW);
            bdma(r, voff[0], sl + 4u * (unsigned)(cl * WSP));
            bdma(r, voff[1], sl + 4u * (unsigned)(cl * WSP + 64));
            bdma(r, voff[2], sl + 4u * (unsigned)(cl * WSP + 128));
        }
        const float* sw = wuniform(a.wpack + ((int64_t)x.cg * a.cin + c0) * 512);
        const unsigned wl = lds0 + 4u * (unsigned)(buf * BUFF + INF);
        const int wpp = (CK / 2) / np;
#pragma unroll
        for (int jj = 0; jj < wpp; ++jj) {
            const int j = part * wpp + jj;
            wdma<4>(sw, 4u * (unsigned)(j * 1024 + tid * 4), wl + 4u * (unsigned)(j * 1024 + wave * 256));
        }
    };

    const int nchunk = a.cin / CK;
    int u = slot;
    if (a.queue) {
        if (tid == 0) qsl[0] = grab();
        __syncthreads();
        u = __builtin_amdgcn_readfirstlane(qsl[0]);
    }
    int par = 0;  // unit parity (queue slot of the next unit: qsl[par ^ 1])
    Unit cur = unit_of(u < nunits ? u : 0);
    if (u < nunits) {
        plan_copies(cur);
        issue(cur, 0, 0, 0, 1);
    }
    int kk = 0;  // chunks issued so far (buffer = kk & 1)
    while (u < nunits) {
        // next unit: static, or taken from the queue now (its atomic returns while this unit's first
        // chunks run) and published to the block through LDS in the last chunk
        int un = u + G;
        int qv = 0;
        if (a.queue && tid == 0) qv = grab();
        Unit nxt = unit_of(un < nunits ? un : u);
        // this lane's tile of the current unit
        int tr, tc, pbase, lb = cur.b;
        bool tvalid;
        if constexpr (SP) {
            const Segs S = segs_of(cur);
            int q = 0;
#pragma unroll
            for (int t = 1; t < 4; ++t) q += (S.len[t] > 0 && n >= S.st[t]) ? 1 : 0;
            int st = S.st[0], p0 = S.p[0], bq = S.b[0], trq = S.tr[0];
#pragma unroll
            for (int t = 1; t < 4; ++t)
                if (q == t) { st = S.st[t]; p0 = S.p[t]; bq = S.b[t]; trq = S.tr[t]; }
            tr = trq;
            tc = (q == 0 ? cur.tc_a : 0) + n - st;
            lb = bq;
            tvalid = cur.tw + n < g.NTOT;
            pbase = wave * WSLOT + kq * WSP + p0 + 2 * (n - st);
        } else {
            const int len_a = min(16, g.TC - cur.tc_a);
            const bool seg1 = n >= len_a;
            tr = seg1 ? cur.tr_a + 1 : cur.tr_a;
            tc = seg1 ? n - len_a : cur.tc_a + n;
            tvalid = cur.tw + n < g.NTS;
            // (X4: segment B starts at the granule after segment A's segw columns)
            const int bshift = X4 ? (((2 * len_a + 2 + 3) & ~3) - (2 * len_a + 2)) : 0;
            pbase = wave * WSLOT + kq * WSP + (seg1 ? 2 * n + 2 + bshift : 2 * n);
        }
        // BN+ReLU operands: out-of-image patch rows / columns must be 0 after the prologue (the copy
        // wrote raw 0s there); a factor per patch row / column, applied only in waves that touch the
        // image border
        float fr0 = 1.f, fr2 = 1.f, fr3 = 1.f, fc0 = 1.f, fc2 = 1.f, fc3 = 1.f;
        bool border = false;
        if (PRO != PRO_RAW || X4) {
            fr0 = tr > 0 ? 1.f : 0.f;
            fr2 = 2 * tr + 1 < a.H ? 1.f : 0.f;
            fr3 = 2 * tr + 2 < a.H ? 1.f : 0.f;
            fc0 = tc > 0 ? 1.f : 0.f;
            fc2 = 2 * tc + 1 < a.W ? 1.f : 0.f;
            fc3 = 2 * tc + 2 < a.W ? 1.f : 0.f;
            // (X4 under PRO_RAW: out-of-image rows are zero-copied; only the columns need zeroing)
            const float f = (PRO == PRO_RAW ? 1.f : fr0 * fr2 * fr3) * fc0 * fc2 * fc3;
            border = __builtin_amdgcn_readfirstlane((int)(__ballot(f == 0.f) != 0)) != 0;
        }
        f32x4 acc[16][2];  // the unit's first K-step starts the sums from 0 (no zeroing pass)
        auto kloop = [&](auto btag) {
            constexpr bool BRD = decltype(btag)::value;
            // zero-start first K-step (not on the border copy / the pooled epilogue: registers)
            constexpr bool PEEL = !BRD && EPI != EPI_BWD_POOL;
            // one K-step (4 input channels) on operands in LDS
            auto kstep = [&](const float* bi, const float* bw, int s, int c0, auto ftag) {
                constexpr bool FIRST = decltype(ftag)::value;
                    const int cl = 4 * s + kq;
                f2 P[4][2];  // patch row r, columns 2 k, 2 k + 1
                const float* pp = bi + pbase + 4 * s * WSP;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    P[r][0] = *reinterpret_cast<const f2*>(pp + r * WROW);
                    P[r][1] = *reinterpret_cast<const f2*>(pp + r * WROW + 2);
                }
                f32x4 av[2][4];
#pragma unroll
                for (int mi = 0; mi < 2; ++mi)
#pragma unroll
                    for (int q = 0; q < 4; ++q)
                        av[mi][q] = *reinterpret_cast<const f32x4*>(bw + (((cl * 4 + q) * 32) + 16 * mi + n) * 4);
                const f2 st = PRO != PRO_RAW ? *reinterpret_cast<const f2*>(cft + 2 * (c0 + cl)) : f2{1.f, 0.f};
                // every LDS read of the K-step is issued before its arithmetic (one exposed latency per K-step,
                // covered by the SIMD's other wave, instead of the scheduler's waits between MFMAs: -1 to -3 %,
                // profiles/r5_wino_sched.txt)
                __builtin_amdgcn_sched_barrier(0);
#if defined(WINO_KO) && (WINO_KO & 8)  // analysis builds only: no BN + ReLU prologue arithmetic
                if (false) {
#else
                if (PRO != PRO_RAW) {
#endif
#pragma unroll
                    for (int r = 0; r < 4; ++r)
#pragma unroll
                        for (int k = 0; k < 2; ++k) P[r][k] = pk_bnrelu(P[r][k], st);
                    if constexpr (BRD && !X4) {
#pragma unroll
                        for (int k = 0; k < 2; ++k) {
                            P[0][k] *= fr0;
                            P[2][k] *= fr2;
                            P[3][k] *= fr3;
                        }
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            P[r][0].x *= fc0;
                            P[r][1].x *= fc2;
                            P[r][1].y *= fc3;
                        }
                    }
                }
                if constexpr (BRD && X4) {
                    // the 16-byte copies bring the neighbouring rows' values into the out-of-image columns
                    // (and, under BN + ReLU, relu(t) into the zero-copied rows): selects, not products (the
                    // value before a tensor's first plane is the workspace's unwritten slack)
                    if constexpr (PRO != PRO_RAW) {
#pragma unroll
                        for (int k = 0; k < 2; ++k) {
                            P[0][k] = fr0 != 0.f ? P[0][k] : f2{0.f, 0.f};
                            P[2][k] = fr2 != 0.f ? P[2][k] : f2{0.f, 0.f};
                            P[3][k] = fr3 != 0.f ? P[3][k] : f2{0.f, 0.f};
                        }
                    }
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        P[r][0].x = fc0 != 0.f ? P[r][0].x : 0.f;
                        P[r][1].x = fc2 != 0.f ? P[r][1].x : 0.f;
                        P[r][1].y = fc3 != 0.f ? P[r][1].y : 0.f;
                    }
                }
                // V = B^T d B (rows first, then columns): 32 additions as 16 packed
                float v[16];
                pk_input_transform(pk, P, v);
#pragma unroll
                for (int x = 0; x < 16; ++x)
#pragma unroll
                    for (int mi = 0; mi < 2; ++mi) acc[x][mi] = mfma16(av[mi][x >> 2][x & 3], v[x], FIRST ? f32x4{0.f, 0.f, 0.f, 0.f} : acc[x][mi]);
            };
            auto chunk = [&](int k, auto ftag) {
                const int c0 = k * CK;
                if (a.queue && tid == 0 && k + 1 == nchunk) qsl[par ^ 1] = qv;
#if !(defined(WINO_KO) && (WINO_KO & 4))  // analysis builds only: no chunk synchronisation
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __syncthreads();  // chunk kk visible; chunk kk-1 fully consumed
#endif
                // the next chunk (of this unit, or the next unit's first), copied part by part
                // ahead of this chunk's K-steps
                const bool more = k + 1 < nchunk;
                if (!more && a.queue) {
                    un = __builtin_amdgcn_readfirstlane(qsl[par ^ 1]);
                    nxt = unit_of(un < nunits ? un : u);
                }
                const bool pre = more || un < nunits;
                if (!more && pre) plan_copies(nxt);
                const Unit& tgt = more ? cur : nxt;
                const int tc0 = more ? c0 + CK : 0, tbuf = (kk + 1) & 1;
                const float* bi = smem + (kk & 1) * BUFF;
                const float* bw = bi + INF;
                if (pre) issue(tgt, tc0, tbuf, 0, CK / 4);
                kstep(bi, bw, 0, c0, ftag);
#pragma unroll
                for (int s = 1; s < CK / 4; ++s) {
                    if (pre) issue(tgt, tc0, tbuf, s, CK / 4);
                    kstep(bi, bw, s, c0, std::false_type{});
                }
                ++kk;
            };
            // chunk 0 peeled: its first K-step starts the sums from 0 (PEEL), so no copies of the
            // accumulators are needed between a zeroing and a summing loop entry
            if constexpr (PEEL) {
                chunk(0, std::true_type{});
                for (int k = 1; k < nchunk; ++k) chunk(k, std::false_type{});
            } else {
                for (int k = 0; k < nchunk; ++k) chunk(k, std::false_type{});
            }
        };
        if (border || EPI == EPI_BWD_POOL) {
#pragma unroll
            for (int x = 0; x < 16; ++x) {
                acc[x][0] = f32x4{0.f, 0.f, 0.f, 0.f};
                acc[x][1] = f32x4{0.f, 0.f, 0.f, 0.f};
            }
            if (border) kloop(std::true_type{});
            else kloop(std::false_type{});
        }
        else kloop(std::false_type{});

        // ---- output transform Y = A^T M A: y[j][e] = output (2 tr + (e >> 1), 2 tc + (e & 1)) of
        // channel j = 4 mi + i
        // (packed over channel pairs i, i + 1: 24 additions per channel as 12 packed, same order: pk_f32.h)
        float y[8][4];
#pragma unroll
        for (int mi = 0; mi < 2; ++mi)
#pragma unroll
            for (int ih = 0; ih < 2; ++ih) {
                auto A = [&](int x) -> f2 {
                    return ih ? __builtin_shufflevector(acc[x][mi], acc[x][mi], 2, 3)
                              : __builtin_shufflevector(acc[x][mi], acc[x][mi], 0, 1);
                };
                f2 s0[4], s1[4];
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    s0[c] = A(c) + A(4 + c) + A(8 + c);
                    s1[c] = pk_sub(pk, pk_sub(pk, A(4 + c), A(8 + c)), A(12 + c));
                }
                const f2 y0 = s0[0] + s0[1] + s0[2];
                const f2 y1 = pk_sub(pk, pk_sub(pk, s0[1], s0[2]), s0[3]);
                const f2 y2 = s1[0] + s1[1] + s1[2];
                const f2 y3 = pk_sub(pk, pk_sub(pk, s1[1], s1[2]), s1[3]);
                const int j = 4 * mi + 2 * ih;
                y[j][0] = y0.x; y[j][1] = y1.x; y[j][2] = y2.x; y[j][3] = y3.x;
                y[j + 1][0] = y0.y; y[j + 1][1] = y1.y; y[j + 1][2] = y2.y; y[j + 1][3] = y3.y;
            }
#if defined(WINO_KO) && (WINO_KO & 2)  // analysis builds only: no epilogue (one guarded store keeps y live)
        {
            float t = 0.f;
#pragma unroll
            for (int j = 0; j < 8; ++j) t += y[j][0] + y[j][1] + y[j][2] + y[j][3];
            if (t == 1234.5f) a.out[tid] = t;
        }
#else
        wino_epilogue<EPI, V4, POOL>(a, y, red, cfl, lb, cur.tb, cur.cg * 32, tr, tc, tvalid, wave, tid);
#endif
        u = un;
        cur = nxt;
        par ^= 1;
    }
    // the last workgroup out leaves the queue zero for the next launch (every workgroup has taken its
    // last unit: its own counter and the others' are past their ranges)
    if (a.queue && tid == 0) {
        __threadfence();
        if (atomicAdd(a.queue + 32 * 8, 1) == G - 1) {
            for (int q = 0; q < 9; ++q) atomicExch(a.queue + 32 * q, 0);
        }
    }
}

// U = G g G^T per (GEMM output channel m, GEMM input channel k), evaluated in float64.
// flip: data-gradient GEMM of forward weights w[K][M][3][3] (g[m][k] = w[k][m] rotated 180 deg).
__device__ __forceinline__ void wino_pack_one(const float* __restrict__ w, float* __restrict__ u, int M, int K, int flip,
                                              int e);
__global__ void wino_pack_kernel(const float* __restrict__ w, float* __restrict__ u, int M, int K, int flip) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= M * K) return;
    wino_pack_one(w, u, M, K, flip, e);
}
// several packs in one launch (a network's layers: one launch per pass instead of one per layer)
__global__ void wino_pack_multi_kernel(WinoPackJobs j) {
    int e = blockIdx.x * blockDim.x + threadIdx.x;
    for (int i = 0; i < j.n; ++i) {
        const int n = j.M[i] * j.K[i];
        if (e < n) {
            wino_pack_one(j.w[i], j.u[i], j.M[i], j.K[i], j.flip[i], e);
            return;
        }
        e -= n;
    }
}
__device__ __forceinline__ void wino_pack_one(const float* __restrict__ w, float* __restrict__ u, int M, int K, int flip,
                                              int e) {
    const int m = e / K, k = e - m * K;
    double gg[3][3];
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c)
            gg[r][c] = flip ? (double)w[(((int64_t)k * M + m) * 3 + (2 - r)) * 3 + (2 - c)]
                            : (double)w[(((int64_t)m * K + k) * 3 + r) * 3 + c];
    double t[4][3];
    for (int c = 0; c < 3; ++c) {
        t[0][c] = gg[0][c];
        t[1][c] = 0.5 * (gg[0][c] + gg[1][c] + gg[2][c]);
        t[2][c] = 0.5 * (gg[0][c] - gg[1][c] + gg[2][c]);
        t[3][c] = gg[2][c];
    }
    const int cgi = m >> 5, ml = m & 31;
    float* dst = u + (((int64_t)cgi * K + k) * 4) * 128 + ml * 4;
    for (int q = 0; q < 4; ++q) {
        float4 o;
        o.x = (float)t[q][0];
        o.y = (float)(0.5 * (t[q][0] + t[q][1] + t[q][2]));
        o.z = (float)(0.5 * (t[q][0] - t[q][1] + t[q][2]));
        o.w = (float)t[q][2];
        *reinterpret_cast<float4*>(dst + q * 128) = o;
    }
}

}  // namespace

// ====================================================================== host side
static int wino_ck(int cin) { return cin % 8 == 0 ? 8 : 4; }

static WinoGeo wino_base(int B, int H, int W, int cout) {
    WinoGeo r{};
    r.TR = (H + 1) / 2;
    r.TC = (W + 1) / 2;
    r.NTS = r.TR * r.TC;
    r.BPS = ceil_div(r.NTS, 64);
    r.ncg = cout / 32;
    r.inv_ncg = 1.f / r.ncg;
    r.inv_BPS = 1.f / r.BPS;
    r.inv_TC = 1.f / r.TC;
    r.inv_NTS = 1.f / r.NTS;
    r.inv_TR = 1.f / r.TR;
    r.NTOT = B * r.NTS;
    r.nblk = B * r.BPS;
    return r;
}

bool wino_geometry(int B, int H, int W, int cin, int cout, WinoGeo* g) {
    if (cout % 32 || cin % 4 || H < 1 || W < 31) return false;  // 16 tiles of a wave span <= 2 tile rows
    const WinoGeo r = wino_base(B, H, W, cout);
    if ((int64_t)B * r.BPS * r.ncg >= ((int64_t)1 << 22)) return false;  // unit indices (float division)
    if ((int64_t)cin * H * W >= ((int64_t)1 << 30)) return false;
    if ((int64_t)wino_ck(cin) * H * W + 4 * W + 64 >= ((int64_t)1 << 24)) return false;  // packed copy offsets
    if (g) *g = r;
    return true;
}

bool wino_span_geometry(int B, int H, int W, int cin, int cout, WinoGeo* g) {
    if (cout % 32 || cin % 8 || H < 1 || W < 1 || W >= 31 || B < 1) return false;
    WinoGeo r = wino_base(B, H, W, cout);
    r.span = 1;
    if ((int64_t)B * r.NTS >= ((int64_t)1 << 22)) return false;  // batch-wide tile indices (float division)
    r.nblk = (int)ceil_div((int64_t)B * r.NTS, 64);
    if ((int64_t)r.nblk * r.ncg >= ((int64_t)1 << 22)) return false;
    if ((int64_t)4 * (4 * (int64_t)cin * H * W + 8 * H * W + 64) >= ((int64_t)1 << 30)) return false;  // copy offsets
    // every window of 16 consecutive tiles (it starts at any column of a row) must fit the slot row:
    // at most 4 row segments, each 2 len + 2 columns rounded up to a 16-byte granule, 40 columns in all
    for (int c0 = 0; c0 < r.TC; ++c0) {
        int j = 0, tc = c0, pc = 0, ns = 0;
        while (j < 16) {
            const int len = std::min(16 - j, r.TC - tc);
            pc += (2 * len + 2 + 3) & ~3;
            j += len;
            tc = 0;
            ++ns;
        }
        if (ns > 4 || pc > 40) return false;
    }
    if (g) *g = r;
    return true;
}

size_t wino_nblk(int B, int H, int W, int cin, int cout) {
    WinoGeo g;
    if (wino_geometry(B, H, W, cin, cout, &g) || wino_span_geometry(B, H, W, cin, cout, &g)) return (size_t)g.nblk;
    return 0;
}

int launch_wino_pack(const float* w, float* u, int M, int K, int flip, hipStream_t s) {
    PCX_CHECK_ARG(M % 32 == 0, "wino_pack: %d output channels (multiple of 32 required)", M);
    const int n = M * K;
    wino_pack_kernel<<<ceil_div(n, 256), 256, 0, s>>>(w, u, M, K, flip);
    PCX_LAUNCH_CHECK("wino_pack_kernel");
    return PCX_OK;
}

int launch_wino_pack_multi(const WinoPackJobs& j, hipStream_t s) {
    PCX_CHECK_ARG(j.n >= 0 && j.n <= WinoPackJobs::MAXJ, "wino_pack_multi: %d packs", j.n);
    int64_t n = 0;
    for (int i = 0; i < j.n; ++i) {
        PCX_CHECK_ARG(j.M[i] % 32 == 0, "wino_pack: %d output channels (multiple of 32 required)", j.M[i]);
        n += (int64_t)j.M[i] * j.K[i];
    }
    PCX_CHECK_ARG(n < ((int64_t)1 << 30), "wino_pack_multi: %lld weights", (long long)n);
    if (n == 0) return PCX_OK;
    wino_pack_multi_kernel<<<ceil_div(n, 256), 256, 0, s>>>(j);
    PCX_LAUNCH_CHECK("wino_pack_multi_kernel");
    return PCX_OK;
}

int launch_conv3x3_wino(int pro, int epi, ConvArgs a, hipStream_t s) {
    WinoGeo g;
    const bool sp = !wino_geometry(a.B, a.H, a.W, a.cin, a.cout, &g);
    PCX_CHECK_ARG(!sp || wino_span_geometry(a.B, a.H, a.W, a.cin, a.cout, &g),
                  "conv3x3_wino: unsupported shape (B %d, %dx%d, cin %d, cout %d)", a.B, a.H, a.W, a.cin, a.cout);
    PCX_CHECK_ARG(!sp || (pro == PRO_RAW && (epi == EPI_FWD || epi == EPI_BWD_STORE) && a.src_guard),
                  "conv3x3_wino: %dx%d images need PRO_RAW, EPI_FWD / EPI_BWD_STORE and src_guard", a.H, a.W);
    PCX_CHECK_ARG(a.nblk == g.nblk, "conv3x3_wino: partial buffer sized for %d tiles, need %d", a.nblk, g.nblk);
    {  // the epilogue's 32-bit buffer offsets span the samples of one wave's tiles x cout output planes
        const int64_t ns = sp ? (64 + g.NTS - 1) / g.NTS + 1 : 1;
        const int64_t hwo = std::max<int64_t>((int64_t)a.H * a.W, (epi == EPI_BWD_POOL || epi == EPI_BWD_POOLSEL)
                                                                      ? (int64_t)a.Hs * a.Ws : 0);
        PCX_CHECK_ARG(4 * ns * a.cout * hwo < 0x7ffffff0, "conv3x3_wino: %d x %lld outputs per sample exceed the "
                      "epilogue's 32-bit offsets", a.cout, (long long)hwo);
    }
    PCX_CHECK_ARG(pro == PRO_RAW || pro == PRO_BNRELU, "conv3x3_wino: prologue %d", pro);
    if (epi == EPI_BWD_POOL || epi == EPI_BWD_POOLSEL)
        PCX_CHECK_ARG(a.Hs >= 2 * a.H && a.Ws >= 2 * a.W, "conv3x3_wino: pooled source %dx%d for %dx%d", a.Hs, a.Ws,
                      a.H, a.W);
    PCX_CHECK_ARG((epi != EPI_BWD_POOLSEL && epi != EPI_BWD_POOLSELP) || (a.ysel && a.parg),
                  "conv3x3_wino: EPI_BWD_POOLSEL needs ysel and parg");
    PCX_CHECK_ARG(epi != EPI_BWD_POOLSELP || a.dpool, "conv3x3_wino: EPI_BWD_POOLSELP needs dpool");
    const int ck = wino_ck(a.cin);
    const size_t buff = (size_t)4 * (ck * WSP + 32) + (size_t)ck * 512;
    const bool pool = a.pool_ysel != nullptr;
    // + the epilogue's BN coefficients (float4 per channel) or the pooled selection's signs (float per channel)
    const bool cfl = epi != EPI_FWD && epi != EPI_BWD_STORE;
    const size_t smem = (2 * buff + 2 * (size_t)a.cin + 512 + 4 + (cfl ? 4 * (size_t)a.cout : pool ? (size_t)a.cout : 0)) * 4;
    PCX_CHECK_ARG(smem <= 160 * 1024, "conv3x3_wino: %zu B of LDS", smem);
    // persistent workgroups: two per CU (a multiple of 8, one XCD-contiguous run of units each round)
    const int64_t units = (int64_t)g.nblk * g.ncg;
    int64_t nwg = std::min<int64_t>(units, 2 * (int64_t)num_cus());
    if (nwg >= 8) nwg &= ~(int64_t)7;
    dim3 grid((unsigned)nwg);
    g.naive_slots = PCX_AB_WINO_SLOT;
    // pooled data gradient with 16-byte source rows
    const bool v4 = (epi == EPI_BWD_POOL || epi == EPI_BWD_POOLSEL) && (a.Ws & 3) == 0 && !(a.H & 1) && !(a.W & 1);
    // 16-byte operand copies where the caller guarantees 4 readable bytes before src (PCX_AB_NO_WINO_X4: dword copies)
    constexpr bool x4_env = !PCX_AB_NO_WINO_X4;
    // (not the pooled data gradient: its window registers already spill at 8-14 VGPRs; the two more
    // copy offsets of X4 made that 31-34)
    // measured at B = 4096 (profiles/r4_x4_time.txt): BN + ReLU forward and the data gradients gain
    // 3-6 %, the raw-input forward (L3 / L5: 32 -> 64, 64 -> 128) nothing or -2.5 %: dword copies there
    const bool x4 = ck == 8 && a.src_guard && x4_env && epi != EPI_BWD_POOL &&
                    (PCX_AB_WINO_X4_RAWFWD || !(pro == PRO_RAW && epi == EPI_FWD));
#define PCX_WINO_CASE(P_, E_, CK_, V4_, X4_)                                                            \
    if (pro == P_ && epi == E_ && ck == CK_ && v4 == V4_ && x4 == X4_) {                                \
        (void)hipFuncSetAttribute((const void*)conv_wino_kernel<P_, E_, CK_, V4_, X4_>,                 \
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);               \
        conv_wino_kernel<P_, E_, CK_, V4_, X4_><<<grid, 256, smem, s>>>(a, g);                          \
        PCX_LAUNCH_CHECK("conv_wino_kernel");                                                           \
        return PCX_OK;                                                                                  \
    }
    if (pool) {
        PCX_CHECK_ARG(!sp && epi == EPI_FWD && pro == PRO_BNRELU && ck == 8 && x4 && a.pool_arg && a.pool_gamma &&
                          !(a.H & 1) && !(a.W & 1),
                      "conv3x3_wino: pooled selection needs the BN + ReLU forward with 16-byte staging at even H, W");
        (void)hipFuncSetAttribute((const void*)conv_wino_kernel<PRO_BNRELU, EPI_FWD, 8, false, true, false, true>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
        conv_wino_kernel<PRO_BNRELU, EPI_FWD, 8, false, true, false, true><<<grid, 256, smem, s>>>(a, g);
        PCX_LAUNCH_CHECK("conv_wino_kernel (pooled selection)");
        return PCX_OK;
    }
    if (sp) {
        if (epi == EPI_FWD) {
            (void)hipFuncSetAttribute((const void*)conv_wino_kernel<PRO_RAW, EPI_FWD, 8, false, true, true>,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
            conv_wino_kernel<PRO_RAW, EPI_FWD, 8, false, true, true><<<grid, 256, smem, s>>>(a, g);
        } else {
            (void)hipFuncSetAttribute((const void*)conv_wino_kernel<PRO_RAW, EPI_BWD_STORE, 8, false, true, true>,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
            conv_wino_kernel<PRO_RAW, EPI_BWD_STORE, 8, false, true, true><<<grid, 256, smem, s>>>(a, g);
        }
        PCX_LAUNCH_CHECK("conv_wino_kernel (spanning units)");
        return PCX_OK;
    }
#define PCX_WINO_CK(P_, E_, V4_) PCX_WINO_CASE(P_, E_, 8, V4_, false) PCX_WINO_CASE(P_, E_, 4, V4_, false) \
    PCX_WINO_CASE(P_, E_, 8, V4_, true)
    PCX_WINO_CK(PRO_RAW, EPI_FWD, false)
    PCX_WINO_CK(PRO_BNRELU, EPI_FWD, false)
    PCX_WINO_CK(PRO_RAW, EPI_BWD_RELU, false)
    PCX_WINO_CASE(PRO_RAW, EPI_BWD_POOL, 8, false, false) PCX_WINO_CASE(PRO_RAW, EPI_BWD_POOL, 4, false, false)
    PCX_WINO_CASE(PRO_RAW, EPI_BWD_POOL, 8, true, false) PCX_WINO_CASE(PRO_RAW, EPI_BWD_POOL, 4, true, false)
    PCX_WINO_CK(PRO_RAW, EPI_BWD_POOLSEL, false)
    PCX_WINO_CK(PRO_RAW, EPI_BWD_POOLSEL, true)
    PCX_WINO_CASE(PRO_RAW, EPI_BWD_POOLSELP, 8, false, false) PCX_WINO_CASE(PRO_RAW, EPI_BWD_POOLSELP, 8, false, true)
    PCX_WINO_CASE(PRO_RAW, EPI_BWD_POOLSELP, 4, false, false)
    PCX_WINO_CK(PRO_RAW, EPI_BWD_STORE, false)
#undef PCX_WINO_CK
#undef PCX_WINO_CASE
    set_error("conv3x3_wino: unsupported combination (pro %d epi %d ck %d)", pro, epi, ck);
    return PCX_EINVAL;
}

}  // namespace pcx
