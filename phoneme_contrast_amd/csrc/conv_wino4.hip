// 3x3 / stride 1 / pad 1 convolution (forward and data gradient) as the 2-D Winograd transform
// F(4x3, 3x3) on fp32 MFMA (v_mfma_f32_16x16x4_f32): 4-row x 3-column output tiles, 6x5 input patches,
// 30 multiplies per 12 outputs (the direct conv: 108; conv_wino's F(2x2,3x3): 48).  Same contract as
// conv_wino.hip (ConvArgs, prologues, epilogues); all arithmetic fp32, the weight transform in float64.
//
//   Y = Ar^T [ U (.) V ] Ac,   U = Gr g Gc^T (6x5),   V = Br^T d Bc (6x5 patch)
//   rows:    F(4,3), points 0, +-1, +-2:  Br^T = [4 0 -5 0 1 0; 0 -4 -4 1 1 0; 0 4 -4 -1 1 0; 0 -2 -1 2 1 0;
//            0 2 -1 -2 1 0; 0 4 0 -5 0 1],  Gr = [1/4 0 0; -1/6 -1/6 -1/6; -1/6 1/6 -1/6; 1/24 1/12 1/6;
//            1/24 -1/12 1/6; 0 0 1],  Ar^T = [1 1 1 1 1 0; 0 1 -1 2 -2 0; 0 1 1 4 4 0; 0 1 -1 8 -8 1]
//   columns: F(3,3), points 0, 1, -1, 2:  Bc^T = [2 -1 -2 1 0; 0 -2 -1 1 0; 0 2 -3 1 0; 0 -1 0 1 0; 0 2 -1 -2 1],
//            Gc = [1/2 0 0; -1/2 -1/2 -1/2; -1/6 1/6 -1/6; 1/6 1/3 2/3; 0 0 1],  Ac^T = [1 1 1 1 0; 0 1 -1 2 0; 0 1 1 4 1]
//   (Lavin & Gray; float32 error of the pair measured in float64 simulation: ~1e-6 rms of |y|, F(2x2): 2e-7)
//
// Why this tile on MI355X: an fp32 MFMA runs on the same ALUs as the VALU (157.3 TF/s either way; a VALU
// instruction beside the MFMA stream costs 3-6 SIMD cycles: tools/mfma_mix.hip, profiles/r5_mfma_mix.txt),
// so the conv costs MFMA cycles + transform / prologue / epilogue VALU cycles.  A larger tile cuts MFMAs per
// output but transforms a larger patch, which only pays when each patch feeds 32 output channels: 2 x 30
// accumulator tiles = 240 registers, the AGPR file of ONE wave per SIMD (F(4x4) would need 288 and makes the
// compiler round-trip accumulators through VGPRs).  Per 12 outputs x 32 channels x 4 input channels the K
// step is 60 MFMAs + ~120 VALU (+60 for a BN + ReLU prologue): ~30 % fewer cycles per output than F(2x2).
//
// Layout / staging:
//  * 4 waves, one workgroup per CU (LDS ~87 KB), persistent over units = (64 consecutive tiles of the batch
//    in row-major tile order, 32 output channels) from the per-XCD queue (ConvArgs::queue) as conv_wino;
//    wave w owns tiles 16 w .. 16 w + 15: one or two row segments (tile columns >= 16), the second possibly
//    the first tile row of the next sample;
//  * K-chunk = 4 input channels = one K step, double buffered.  Wave slot: [4 channels][6 rows][60] + 8 pad
//    floats per channel (plane stride 368 = 48 mod 64: the lanes' 4-byte patch reads hit 64 banks), copied
//    by 6 buffer_load_dwordx4 ... lds per chunk (per-lane offsets per unit, 16-byte granules from any
//    4-byte-aligned source; out-of-image rows read 0, straddling columns are zeroed by selects in border
//    waves); the chunk's transformed weights [4][32][36] (30 used) by 18 global_load_lds_dwordx4;
//  * lane (tile n = l & 15, channel kq = l >> 4): 30 ds_read_b32 of its patch, BN + ReLU, 114-VALU
//    transform, 2 x 30 MFMAs (A = U: lane (cout n, channel kq), ds_read_b128 of 4 consecutive xi);
//  * epilogue per output channel (8 per lane): Ar^T M Ac (78 VALU), BN statistics / BN-backward sums as
//    conv_wino (transposed butterfly).
#include <cstdlib>
#include <type_traits>

#include "conv_epilogue.h"

namespace pcx {
namespace {

typedef __attribute__((address_space(3))) void lds_void;
typedef float f2v __attribute__((ext_vector_type(2)));

constexpr int W4_CK = 4;                          // channels per chunk (one K step)
constexpr int W4_ROW = 60;                        // slot row: 15 granules (two segments of 3 len + 2 columns)
constexpr int W4_RG = W4_ROW / 4;                 // 15
constexpr int W4_PLANE = 368;                     // 6 rows x 60 + 8 pad: plane stride = 48 mod 64
constexpr int W4_PG = W4_PLANE / 4;               // 92 granules per channel (90 data + 2 pad)
constexpr int W4_GRAN = W4_CK * W4_PG;            // 368 granules per wave and chunk
constexpr int W4_NCP = (W4_GRAN + 63) / 64;       // 6 input DMA instructions per wave and chunk
constexpr int W4_WSLOT = W4_NCP * 256;            // wave slot (floats): the last DMA's 16 surplus granules land here
constexpr int W4_INF = 4 * W4_WSLOT;              // input floats per buffer
constexpr int W4_XS = 36;                         // weight floats per (cin, cout): 30 xi + pad (stride 36: b128 reads conflict-free)
constexpr int W4_WF = W4_CK * 32 * W4_XS;         // weight floats per buffer: [channel][cout 32][36]
constexpr int W4_WDMA = W4_WF / 256;              // 18 weight DMA instructions per chunk (64 granules each)
constexpr int W4_BUFF = W4_INF + W4_WF;

__device__ __forceinline__ int w4div(int n, int d, float inv) {
    int q = (int)((float)n * inv);
    const int r = n - q * d;
    q += r >= d ? 1 : 0;
    q -= r < 0 ? 1 : 0;
    return q;
}

__device__ __forceinline__ f32x4 mfma16(float a, float b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ void w4_gdma(const float* sbase, unsigned voff, unsigned lds_byte_addr) {
    const unsigned m0 = __builtin_amdgcn_readfirstlane(lds_byte_addr);
    asm volatile("s_nop 0\n\tglobal_load_lds_dwordx4 %0, %1" :: "v"(voff), "s"(sbase), "{m0}"(m0) : "memory");
}

__device__ __forceinline__ void w4_bdma(__amdgpu_buffer_rsrc_t r, unsigned voff, unsigned lds_byte_addr) {
    const unsigned m0 = __builtin_amdgcn_readfirstlane(lds_byte_addr);
    asm volatile("s_nop 0\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds" :: "v"(voff), "s"(r), "{m0}"(m0) : "memory");
}

__device__ __forceinline__ const float* w4_uniform(const float* p) {
    const uint64_t v = (uint64_t)(uintptr_t)p;
    const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)v);
    const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(v >> 32));
    return (const float*)(uintptr_t)(((uint64_t)hi << 32) | lo);
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t w4_rsrc(const float* base, int bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), (short)0, bytes, 0x00020000);
}

// sums over the 16 lanes of a row (lanes sharing l >> 4)
__device__ __forceinline__ float w4_row16_sum(float v) {
    v += __shfl_xor(v, 1, 64);
    v += __shfl_xor(v, 2, 64);
    v += __shfl_xor(v, 4, 64);
    v += __shfl_xor(v, 8, 64);
    return v;
}
// transposed butterfly: v[j] (j < 8) summed over the 16 lanes of a row; lane n gets the total of j = (n >> 1) & 7
__device__ __forceinline__ float w4_xsum8(const float (&v)[8], int n) {
    const bool b3 = n & 8, b2 = n & 4, b1 = n & 2;
    float w4[4], w2[2];
#pragma unroll
    for (int j = 0; j < 4; ++j) w4[j] = (b3 ? v[j + 4] : v[j]) + __shfl_xor(b3 ? v[j] : v[j + 4], 8, 64);
#pragma unroll
    for (int j = 0; j < 2; ++j) w2[j] = (b2 ? w4[j + 2] : w4[j]) + __shfl_xor(b2 ? w4[j] : w4[j + 2], 4, 64);
    const float w1 = (b1 ? w2[1] : w2[0]) + __shfl_xor(b1 ? w2[0] : w2[1], 2, 64);
    return w1 + __shfl_xor(w1, 1, 64);
}
__device__ __forceinline__ float w4_xsel8(const float (&v)[8], int n) {
    const bool b3 = n & 8, b2 = n & 4, b1 = n & 2;
    float w4[4], w2[2];
#pragma unroll
    for (int j = 0; j < 4; ++j) w4[j] = b3 ? v[j + 4] : v[j];
#pragma unroll
    for (int j = 0; j < 2; ++j) w2[j] = b2 ? w4[j + 2] : w4[j];
    return b1 ? w2[1] : w2[0];
}

// 1-D input transform B^T d (12 VALU)
__device__ __forceinline__ void bt6(const float (&d)[6], float (&t)[6]) {
    const float a = fmaf(-4.f, d[2], d[4]), b = fmaf(-4.f, d[1], d[3]);
    const float c = d[4] - d[2], e = d[3] - d[1];
    t[0] = fmaf(4.f, d[0], fmaf(-5.f, d[2], d[4]));
    t[1] = a + b;
    t[2] = a - b;
    t[3] = fmaf(2.f, e, c);
    t[4] = fmaf(-2.f, e, c);
    t[5] = fmaf(4.f, d[1], fmaf(-5.f, d[3], d[5]));
}
// 1-D input transform Bc^T d of the column direction, F(3,3) (9 VALU)
__device__ __forceinline__ void bt5(const float (&d)[5], float (&t)[5]) {
    t[3] = d[3] - d[1];
    const float a = d[3] - d[2], b = d[1] - d[2], c = d[0] - d[2], e = d[4] - d[2];
    t[1] = fmaf(-2.f, d[1], a);
    t[2] = fmaf(2.f, b, a);
    t[0] = fmaf(2.f, c, t[3]);
    t[4] = fmaf(-2.f, t[3], e);
}
// 1-D output transform Ar^T m, F(4,3) (10 VALU)
__device__ __forceinline__ void at6(float m0, float m1, float m2, float m3, float m4, float m5, float (&o)[4]) {
    const float p = m1 + m2, q = m1 - m2, u = m3 + m4, w = m3 - m4;
    o[0] = (m0 + p) + u;
    o[1] = fmaf(2.f, w, q);
    o[2] = fmaf(4.f, u, p);
    o[3] = fmaf(8.f, w, q) + m5;
}
// 1-D output transform Ac^T m, F(3,3) (7 VALU)
__device__ __forceinline__ void at5(float m0, float m1, float m2, float m3, float m4, float (&o)[3]) {
    const float p = m1 + m2, q = m1 - m2;
    o[0] = (m0 + p) + m3;
    o[1] = fmaf(2.f, m3, q);
    o[2] = fmaf(4.f, m3, p) + m4;
}

// one accumulator element read out of its AGPR at the point of use (the compiler would otherwise copy all 240
// accumulators to VGPRs at the K loop's exit and spill); the caller drains the MFMA pipeline first (s_nop)
__device__ __forceinline__ float w4_accrd(float x) {
    float r;
    asm volatile("v_accvgpr_read_b32 %0, %1" : "=v"(r) : "a"(x));
    return r;
}


template <int PRO, int EPI>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void conv_wino4_kernel(ConvArgs a, Wino4Geo g) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int tid = threadIdx.x, lane = tid & 63, n = lane & 15, kq = lane >> 4;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int HW = a.H * a.W;
    float* cft = smem + 2 * W4_BUFF;  // [cin] float2 {s, t}
    float* red = cft + 2 * a.cin;     // epilogue scratch (512 floats) + the queue's 2 ints
    const unsigned lds0 = (unsigned)(uintptr_t)(lds_void*)smem;
    if (PRO != PRO_RAW)
        for (int c = tid; c < a.cin; c += 256) {
            const float4 f = a.cf_in[c];
            cft[2 * c] = f.x;
            cft[2 * c + 1] = f.y;
        }
    const int nunits = g.nblk * g.ncg;
    const int G = gridDim.x;
    const int slot = (G & 7) ? (int)blockIdx.x : (int)(blockIdx.x & 7) * (G >> 3) + (int)(blockIdx.x >> 3);
    const int nq = (a.queue && !(G & 7)) ? 8 : 1;
    int* qsl = reinterpret_cast<int*>(red + 512);
    auto grab = [&]() -> int {  // lane 0 of wave 0 only; (q nunits) < 2^25
        const int x0 = nq == 8 ? (int)(blockIdx.x & 7) : 0;
        for (int k = 0; k < nq; ++k) {
            const int q = (x0 + k) & (nq - 1);
            const int lo = nq == 8 ? (q * nunits) >> 3 : 0, hi = nq == 8 ? ((q + 1) * nunits) >> 3 : nunits;
            const int v = atomicAdd(a.queue + 32 * q, 1);
            if (v < hi - lo) return lo + v;
        }
        return nunits;
    };

    // unit = (64-tile block tb of the batch-wide tile order, 32-channel output group cg); the wave's 16 tiles:
    // segment A (sample ba, tile row tra, columns tca .. tca + lena - 1), segment B (sample bb, tile row trb,
    // columns 0 .. 15 - lena) when lena < 16 and bb < B
    struct Unit { int tb, cg, tw, ba, tra, tca, lena, bb, trb; };
    auto unit_of = [&](int u) {
        Unit x;
        x.tb = w4div(u, g.ncg, g.inv_ncg);
        x.cg = u - x.tb * g.ncg;
        x.tw = x.tb * 64 + wave * 16;
        x.ba = w4div(x.tw, g.NTS, g.inv_NTS);
        const int rem = x.tw - x.ba * g.NTS;
        x.tra = w4div(rem, g.TC, g.inv_TC);
        x.tca = rem - x.tra * g.TC;
        x.lena = min(16, g.TC - x.tca);
        const bool wrap = x.tra + 1 == g.TR;
        x.bb = wrap ? x.ba + 1 : x.ba;
        x.trb = wrap ? 0 : x.tra + 1;
        return x;
    };
    // slot granule gi = 64 j + lane: channel gi / 92, row (gi % 92) / 15, slot column 4 (gi % 15); granules
    // 0 .. nA - 1 hold segment A (image columns 3 tca - 1 ..), nA .. segment B (image columns -1 ..).
    // Offsets relative to src + (ba cin + c0) HW - 1.
    unsigned voff[W4_NCP];
    auto plan_copies = [&](const Unit& x) {
        const int nA = (3 * x.lena + 5) >> 2;
        const bool hasB = x.lena < 16 && x.bb < a.B;
        const int bofs = (x.bb - x.ba) * a.cin * HW;
#pragma unroll
        for (int j = 0; j < W4_NCP; ++j) {
            const int gi = 64 * j + lane;
            const int pl = gi / W4_PG, rem = gi - W4_PG * pl, r = rem / W4_RG, g15 = rem - W4_RG * r, sc = 4 * g15;
            const bool sB = g15 >= nA;
            const int grow = sB ? 4 * x.trb - 1 + r : 4 * x.tra - 1 + r;
            const int gcol = sB ? sc - 4 * nA - 1 : 3 * x.tca - 1 + sc;
            const bool ok = gi < W4_GRAN && r < 6 && (unsigned)grow < (unsigned)a.H && gcol < a.W && (!sB || hasB) &&
                            x.ba < a.B;
            voff[j] = ok ? 4u * (unsigned)((sB ? bofs : 0) + pl * HW + grow * a.W + gcol + 1) : 0x80000000u;
        }
    };
    auto issue = [&](const Unit& x, int c0, int buf) {
        const float* sb = w4_uniform(a.src + ((int64_t)x.ba * a.cin + c0) * HW - 1);
        // (the planes of this sample from c0 on and, for a segment B in the next sample, that sample's)
        // (a wave past the end of the batch, ba == B, gets num_records 1: every one of its offsets reads 0)
        const int64_t rest = (int64_t)(a.B - x.ba) * a.cin * HW - (int64_t)c0 * HW + 1;
        const int nrec = rest < 1 ? 1 : (int)min(rest, (int64_t)(a.cin + W4_CK) * HW + 1);
        const __amdgpu_buffer_rsrc_t r = w4_rsrc(sb, __builtin_amdgcn_readfirstlane(4 * nrec));
        const unsigned sl = lds0 + 4u * (unsigned)(buf * W4_BUFF + wave * W4_WSLOT);
#if !(defined(WINO4_KO) && (WINO4_KO & 1))  // analysis builds only (tools/wino4_kx.sh): no input copies
#pragma unroll
        for (int j = 0; j < W4_NCP; ++j) w4_bdma(r, voff[j], sl + 1024u * (unsigned)j);
#endif
        const float* sw = w4_uniform(a.wpack + ((int64_t)x.cg * a.cin + c0) * (32 * W4_XS));
        const unsigned wl = lds0 + 4u * (unsigned)(buf * W4_BUFF + W4_INF);
#if !(defined(WINO4_KO) && (WINO4_KO & 2))  // analysis builds only: no weight copies
#pragma unroll
        for (int j = 0; j < (W4_WDMA + 3) / 4; ++j) {
            const int jj = 4 * j + wave;
            if (jj < W4_WDMA) w4_gdma(sw, 16u * (unsigned)(64 * jj + lane), wl + 1024u * (unsigned)jj);
        }
#endif
    };

    const int nchunk = a.cin / W4_CK;
    int u = slot;
    if (a.queue) {
        if (tid == 0) qsl[0] = grab();
        __syncthreads();
        u = __builtin_amdgcn_readfirstlane(qsl[0]);
    }
    int par = 0;
    Unit cur = unit_of(u < nunits ? u : 0);
    if (u < nunits) {
        plan_copies(cur);
        issue(cur, 0, 0);
    }
    int kk = 0;
    while (u < nunits) {
        int un = u + G;
        int qv = 0;
        if (a.queue && tid == 0) qv = grab();
        Unit nxt = unit_of(un < nunits ? un : u);
        // this lane's tile
        const bool seg1 = n >= cur.lena;
        const bool tvalid = cur.tw + n < g.NTOT;
        const int b = tvalid ? (seg1 ? cur.bb : cur.ba) : 0;  // (lanes past the batch address sample 0, store nothing)
        const int tr = seg1 ? cur.trb : cur.tra;
        const int tc = seg1 ? n - cur.lena : cur.tca + n;
        const int nA = (3 * cur.lena + 5) >> 2;
        const int pbase = wave * W4_WSLOT + kq * W4_PLANE + (seg1 ? 4 * nA + 3 * (n - cur.lena) : 3 * n);
        // patch rows / columns inside the image (rows 4 tr - 1 + r, columns 3 tc - 1 + c)
        bool fr[6], fc[5];
#pragma unroll
        for (int q = 0; q < 6; ++q) fr[q] = (unsigned)(4 * tr - 1 + q) < (unsigned)a.H;
#pragma unroll
        for (int q = 0; q < 5; ++q) fc[q] = (unsigned)(3 * tc - 1 + q) < (unsigned)a.W;
        bool inside = true;
#pragma unroll
        for (int q = 0; q < 6; ++q) inside = inside && (PRO == PRO_RAW || fr[q]);
#pragma unroll
        for (int q = 0; q < 5; ++q) inside = inside && fc[q];
        const bool border = __builtin_amdgcn_readfirstlane((int)(__ballot(!inside) != 0)) != 0;

        f32x4 acc[30][2];
        {
            auto kstep = [&](const float* bi, const float* bw, int c0, auto ftag) {
                constexpr bool FIRST = decltype(ftag)::value;
                // every LDS operand of the step is requested up front (one exposed latency per step with one wave
                // per SIMD): the chunk's 16 weight quads, then the patch
                const float* wb = bw + (kq * 32 + n) * W4_XS;
                f32x4 W0[8], W1[8];
#pragma unroll
                for (int q = 0; q < 8; ++q) {
                    W0[q] = *reinterpret_cast<const f32x4*>(wb + 4 * q);
                    W1[q] = *reinterpret_cast<const f32x4*>(wb + 16 * W4_XS + 4 * q);
                }
                float d[6][5];
                const float* pp = bi + pbase;
#if defined(WINO4_KO) && (WINO4_KO & 8)  // analysis builds only: the patch as 8 aligned 16-byte reads (wrong values)
                {
                    const float* pq = bi + wave * W4_WSLOT + 4 * lane;
#pragma unroll
                    for (int k = 0; k < 8; ++k) {
                        const f32x4 t = *reinterpret_cast<const f32x4*>(pq + 256 * (k & 3) + 8 * (k >> 2));
#pragma unroll
                        for (int e = 0; e < 4; ++e)
                            if (4 * k + e < 30) d[(4 * k + e) / 5][(4 * k + e) % 5] = t[e];
                    }
                }
#else
#pragma unroll
                for (int r = 0; r < 6; ++r)
#pragma unroll
                    for (int c = 0; c < 5; ++c) d[r][c] = pp[r * W4_ROW + c];
#endif
                if (PRO != PRO_RAW) {
                    const f2v st = *reinterpret_cast<const f2v*>(cft + 2 * (c0 + kq));
#pragma unroll
                    for (int r = 0; r < 6; ++r)
#pragma unroll
                        for (int c = 0; c < 5; ++c) d[r][c] = fmaxf(fmaf(d[r][c], st.x, st.y), 0.f);
                }
                if (border) {  // (wave-uniform branch)
                    // out-of-image patch elements are 0 (the 16-byte copies bring the neighbouring rows' values into
                    // out-of-image columns; BN + ReLU turns zero-copied rows into relu(t))
#pragma unroll
                    for (int r = 0; r < 6; ++r)
#pragma unroll
                        for (int c = 0; c < 5; ++c) d[r][c] = ((PRO == PRO_RAW || fr[r]) && fc[c]) ? d[r][c] : 0.f;
                }
                // V = Br^T d Bc: columns (6-point) first, then each row (5-point) of V, whose xi = 5 r + c are
                // consumed by the MFMAs of every quad (4 consecutive xi) the row completes
                float e[6][5];
#pragma unroll
                for (int c = 0; c < 5; ++c) {
                    const float col[6] = {d[0][c], d[1][c], d[2][c], d[3][c], d[4][c], d[5][c]};
                    float t[6];
                    bt6(col, t);
#pragma unroll
                    for (int r = 0; r < 6; ++r) e[r][c] = t[r];
                }
                float v[32];
                v[30] = v[31] = 0.f;
#pragma unroll
                for (int r = 0; r < 6; ++r) {
                    float t[5];
                    bt5(e[r], t);
#pragma unroll
                    for (int c = 0; c < 5; ++c) v[5 * r + c] = t[c];
#pragma unroll
                    for (int q = 0; q < 8; ++q) {
                        const int last = min(4 * q + 3, 29);  // the quad's last real xi
                        if (last > 5 * r + 4 || (r > 0 && last <= 5 * r - 1)) continue;
                        const f32x4 w0 = W0[q], w1 = W1[q];
#pragma unroll
                        for (int e2 = 0; e2 < 4; ++e2) {
                            const int x = 4 * q + e2;
                            if (x >= 30) continue;
                            acc[x][0] = mfma16(w0[e2], v[x], FIRST ? f32x4{0.f, 0.f, 0.f, 0.f} : acc[x][0]);
                            acc[x][1] = mfma16(w1[e2], v[x], FIRST ? f32x4{0.f, 0.f, 0.f, 0.f} : acc[x][1]);
                        }
                    }
                }
            };
            auto chunk = [&](int k, auto ftag) {
                const int c0 = k * W4_CK;
                if (a.queue && tid == 0 && k + 1 == nchunk) qsl[par ^ 1] = qv;
#if !(defined(WINO4_KO) && (WINO4_KO & 4))  // analysis builds only: no wait for the chunk copies
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
                __syncthreads();  // chunk k visible to every wave; chunk k - 1 consumed
                const bool more = k + 1 < nchunk;
                if (!more && a.queue) {
                    un = __builtin_amdgcn_readfirstlane(qsl[par ^ 1]);
                    nxt = unit_of(un < nunits ? un : u);
                }
                const bool pre = more || un < nunits;
                if (!more && pre) plan_copies(nxt);
                if (pre) issue(more ? cur : nxt, more ? c0 + W4_CK : 0, (kk + 1) & 1);
                const float* bi = smem + (kk & 1) * W4_BUFF;
                kstep(bi, bi + W4_INF, c0, ftag);
                ++kk;
            };
            chunk(0, std::true_type{});
            for (int k = 1; k < nchunk; ++k) chunk(k, std::false_type{});
        }

        // ---- epilogue: per output channel j = 4 mi + i (cout n0 + 16 mi + 4 kq + i) of the lane's tile
        // (the accumulators are read by inline asm: wait out the last MFMAs' result latency first)
        asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
        const int n0 = cur.cg * 32;
        const int h0 = 4 * tr, w0 = 3 * tc;
        const int nrow = tvalid ? min(4, a.H - h0) : 0;
        const int ncol = tvalid ? min(3, a.W - w0) : 0;
        const bool full = nrow == 4 && ncol == 3;
        const int pix0 = tvalid ? h0 * a.W + w0 : 0;
        const int jsel = (n >> 1) & 7;
        const int cosel = 16 * (jsel >> 2) + 4 * kq + (jsel & 3);
        float s1[8], s2[8], kv[8];
        const float cntl = (float)(nrow * ncol);
        // branch-free stores and producer reads: buffer accesses relative to the wave's first plane (sample ba,
        // channel n0); an element outside the tile's image part gets an offset past num_records (store dropped,
        // load 0), the channel's plane offset rides in soffset
        const int64_t orest = ((int64_t)(a.B - cur.ba) * a.cout - n0) * HW;
        const int onrec = __builtin_amdgcn_readfirstlane(
            4 * (int)(orest < 0 ? 0 : min(orest, (int64_t)2 * a.cout * HW)));
        const int64_t obase = ((int64_t)cur.ba * a.cout + n0) * HW;
        const int lofs = ((b - cur.ba) * a.cout + 4 * kq) * HW + pix0;
        unsigned eoff[4][3];
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int c = 0; c < 3; ++c)
                eoff[r][c] = (full || (r < nrow && c < ncol)) ? 4u * (unsigned)(lofs + r * a.W + c) : 0x80000000u;
        const __amdgpu_buffer_rsrc_t rs_o =
            w4_rsrc(w4_uniform((EPI == EPI_FWD || EPI == EPI_BWD_RELU ? a.out : a.dpool) + obase), onrec);
        const __amdgpu_buffer_rsrc_t rs_y =
            w4_rsrc(w4_uniform((EPI == EPI_BWD_RELU ? a.yprev : EPI == EPI_FWD ? a.out : a.ysel) + obase), onrec);
#pragma unroll
        for (int mi = 0; mi < 2; ++mi)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                __builtin_amdgcn_sched_barrier(0);  // one channel at a time: its 30 accumulators leave the AGPRs here
                const int j = 4 * mi + i, co = 16 * mi + 4 * kq + i;
                const int soff = __builtin_amdgcn_readfirstlane(4 * (16 * mi + i) * HW);
                // (data gradient: the producer's values first, so their latency runs under the transform)
                float yy[4][3];
                float4 k4 = make_float4(0.f, 0.f, 0.f, 0.f);
                float dv = 1.f;
                if (EPI != EPI_FWD) {
                    k4 = a.cf_out[n0 + co];
#pragma unroll
                    for (int r = 0; r < 4; ++r)
#pragma unroll
                        for (int c = 0; c < 3; ++c)
                            yy[r][c] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs_y, eoff[r][c], soff, 0));
                    if (EPI == EPI_BWD_POOLSELP && a.drop_out) dv = a.drop_out[(int64_t)b * a.cout + n0 + co];
                }
                // Y = Ar^T M Ac
                float t[4][5];
#pragma unroll
                for (int c = 0; c < 5; ++c) {
                    float o[4];
                    at6(w4_accrd(acc[c][mi][i]), w4_accrd(acc[5 + c][mi][i]), w4_accrd(acc[10 + c][mi][i]),
                        w4_accrd(acc[15 + c][mi][i]), w4_accrd(acc[20 + c][mi][i]), w4_accrd(acc[25 + c][mi][i]), o);
#pragma unroll
                    for (int r = 0; r < 4; ++r) t[r][c] = o[r];
                }
                float y[4][3];
#pragma unroll
                for (int r = 0; r < 4; ++r) at5(t[r][0], t[r][1], t[r][2], t[r][3], t[r][4], y[r]);
                if (EPI == EPI_FWD) {
#pragma unroll
                    for (int r = 0; r < 4; ++r)
#pragma unroll
                        for (int c = 0; c < 3; ++c)
                            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(y[r][c]), rs_o, eoff[r][c], soff, 0);
                    kv[j] = __shfl(y[0][0], lane & 48, 64);
                    float t1 = 0.f, t2 = 0.f;
#pragma unroll
                    for (int r = 0; r < 4; ++r)
#pragma unroll
                        for (int c = 0; c < 3; ++c) {
                            const float dd = (full || (r < nrow && c < ncol)) ? y[r][c] - kv[j] : 0.f;
                            t1 += dd;
                            t2 = fmaf(dd, dd, t2);
                        }
                    s1[j] = t1;
                    s2[j] = t2;
                } else {
                    // dz = dx through the producer's ReLU(BN) (EPI_BWD_RELU: y_prev; EPI_BWD_POOLSELP: y at each 2x2
                    // window's selected element, dropout; the routed gradient stored at the conv's (pooled)
                    // resolution into dpool) + the producer BN's backward sums
                    float s_z = 0.f, s_x = 0.f;
#pragma unroll
                    for (int r = 0; r < 4; ++r)
#pragma unroll
                        for (int c = 0; c < 3; ++c) {
                            const bool ok = full || (r < nrow && c < ncol);
                            const float dz = (ok && fmaf(yy[r][c], k4.x, k4.y) > 0.f) ? y[r][c] * dv : 0.f;
                            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, dz), rs_o, eoff[r][c], soff, 0);
                            s_z += dz;
                            s_x = fmaf(dz, (yy[r][c] - k4.z) * k4.w, s_x);
                        }
                    s1[j] = s_z;
                    s2[j] = s_x;
                }
            }
        if (EPI == EPI_FWD) {
            const float T1 = w4_xsum8(s1, n), T2 = w4_xsum8(s2, n);
            const float K = w4_xsel8(kv, n);
            const float cnt = w4_row16_sum(cntl);
            if (!(n & 1)) {
                float* dd = red + (wave * 32 + cosel) * 3;
                dd[0] = T1; dd[1] = T2; dd[2] = K;
            }
            if (lane == 0) red[384 + wave] = cnt;
            __syncthreads();
            if (tid < 32) {
                float nn = 0.f, mean = 0.f, m2 = 0.f;
#pragma unroll
                for (int w = 0; w < 4; ++w) {
                    const float nw = red[384 + w];
                    if (nw > 0.f) {
                        const float* dd = red + (w * 32 + tid) * 3;
                        const float rw = __builtin_amdgcn_rcpf(nw);
                        const float mw = dd[2] + dd[0] * rw, m2w = fmaxf(dd[1] - dd[0] * dd[0] * rw, 0.f);
                        const float nt = nn + nw, delta = mw - mean, f = nw * __builtin_amdgcn_rcpf(nt);
                        mean += delta * f;
                        m2 += m2w + delta * delta * nn * f;
                        nn = nt;
                    }
                }
                a.part0[(int64_t)(n0 + tid) * a.nblk + cur.tb] = nn * mean;
                a.part1[(int64_t)(n0 + tid) * a.nblk + cur.tb] = m2;
                if (tid == 0 && n0 == 0) a.partn[cur.tb] = nn;
            }
        } else {
            const float tz = w4_xsum8(s1, n), tx = w4_xsum8(s2, n);
            if (!(n & 1)) {
                red[(wave * 32 + cosel) * 2] = tz;
                red[(wave * 32 + cosel) * 2 + 1] = tx;
            }
            __syncthreads();
            if (tid < 32) {
                float z0 = 0.f, z1 = 0.f;
#pragma unroll
                for (int w = 0; w < 4; ++w) {
                    z0 += red[(w * 32 + tid) * 2];
                    z1 += red[(w * 32 + tid) * 2 + 1];
                }
                a.part0[(int64_t)(n0 + tid) * a.nblk + cur.tb] = z0;
                a.part1[(int64_t)(n0 + tid) * a.nblk + cur.tb] = z1;
            }
        }
        u = un;
        cur = nxt;
        par ^= 1;
    }
    if (a.queue && tid == 0) {
        __threadfence();
        if (atomicAdd(a.queue + 32 * 8, 1) == G - 1) {
            for (int q = 0; q < 9; ++q) atomicExch(a.queue + 32 * q, 0);
        }
    }
}

// U = Gr g Gc^T (6x5) per (GEMM output channel m, GEMM input channel k), float64; packed [m / 32][k][m % 32][36]
// (xi = 5 r + c, 30..35 zero).  flip: the data gradient's GEMM of forward weights w[K][M][3][3] (g[m][k] =
// w[k][m] rotated 180 degrees).
__global__ void wino4_pack_kernel(const float* __restrict__ w, float* __restrict__ u, int M, int K, int flip) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= M * K) return;
    const int m = e / K, k = e - m * K;
    double gg[3][3];
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c)
            gg[r][c] = flip ? (double)w[(((int64_t)k * M + m) * 3 + (2 - r)) * 3 + (2 - c)]
                            : (double)w[(((int64_t)m * K + k) * 3 + r) * 3 + c];
    const double Gr[6][3] = {{0.25, 0.0, 0.0},
                             {-1.0 / 6, -1.0 / 6, -1.0 / 6},
                             {-1.0 / 6, 1.0 / 6, -1.0 / 6},
                             {1.0 / 24, 1.0 / 12, 1.0 / 6},
                             {1.0 / 24, -1.0 / 12, 1.0 / 6},
                             {0.0, 0.0, 1.0}};
    const double Gc[5][3] = {{0.5, 0.0, 0.0},
                             {-0.5, -0.5, -0.5},
                             {-1.0 / 6, 1.0 / 6, -1.0 / 6},
                             {1.0 / 6, 1.0 / 3, 2.0 / 3},
                             {0.0, 0.0, 1.0}};
    double t[6][3];
    for (int i = 0; i < 6; ++i)
        for (int c = 0; c < 3; ++c) t[i][c] = Gr[i][0] * gg[0][c] + Gr[i][1] * gg[1][c] + Gr[i][2] * gg[2][c];
    float* dst = u + (((int64_t)(m >> 5) * K + k) * 32 + (m & 31)) * W4_XS;
    for (int i = 0; i < 6; ++i)
        for (int j = 0; j < 5; ++j) dst[5 * i + j] = (float)(t[i][0] * Gc[j][0] + t[i][1] * Gc[j][1] + t[i][2] * Gc[j][2]);
    for (int x = 30; x < W4_XS; ++x) dst[x] = 0.f;
}

}  // namespace

// ====================================================================== host side
bool wino4_geometry(int B, int H, int W, int cin, int cout, Wino4Geo* g) {
    Wino4Geo r{};
    if (cout % 32 || cin % W4_CK || H < 1 || B < 1) return false;
    r.TR = (H + 3) / 4;
    r.TC = (W + 2) / 3;
    if (r.TC < 16) return false;  // the 16 tiles of a wave span at most two tile rows
    if ((int64_t)8 * (cin > cout ? cin : cout) * H * W >= ((int64_t)1 << 31)) return false;  // 32-bit buffer offsets
    r.NTS = r.TR * r.TC;
    if ((int64_t)B * r.NTS >= ((int64_t)1 << 22)) return false;  // batch-wide tile indices (float division)
    r.NTOT = B * r.NTS;
    r.nblk = ceil_div(r.NTOT, 64);
    r.ncg = cout / 32;
    if ((int64_t)r.nblk * r.ncg >= ((int64_t)1 << 22)) return false;  // unit indices
    r.inv_ncg = 1.f / r.ncg;
    r.inv_NTS = 1.f / r.NTS;
    r.inv_TC = 1.f / r.TC;
    if ((int64_t)4 * ((int64_t)(cin + W4_CK) * H * W + 1) >= ((int64_t)1 << 31)) return false;  // buffer bytes
    if (g) *g = r;
    return true;
}

size_t wino4_nblk(int B, int H, int W, int cin, int cout) {
    Wino4Geo g;
    return wino4_geometry(B, H, W, cin, cout, &g) ? (size_t)g.nblk : 0;
}

bool wino4_supports(int pro, int epi) {
    return (pro == PRO_RAW || pro == PRO_BNRELU) &&
           (epi == EPI_FWD || ((epi == EPI_BWD_RELU || epi == EPI_BWD_POOLSELP) && pro == PRO_RAW));
}

int launch_wino4_pack(const float* w, float* u, int M, int K, int flip, hipStream_t s) {
    PCX_CHECK_ARG(M % 32 == 0, "wino4_pack: %d output channels (multiple of 32 required)", M);
    const int n = M * K;
    wino4_pack_kernel<<<ceil_div(n, 256), 256, 0, s>>>(w, u, M, K, flip);
    PCX_LAUNCH_CHECK("wino4_pack_kernel");
    return PCX_OK;
}

size_t wino4_lds_bytes(int cin) { return (2 * (size_t)W4_BUFF + 2 * (size_t)cin + 512 + 4) * 4; }

int launch_conv3x3_wino4(int pro, int epi, ConvArgs a, hipStream_t s) {
    Wino4Geo g;
    PCX_CHECK_ARG(wino4_geometry(a.B, a.H, a.W, a.cin, a.cout, &g),
                  "conv3x3_wino4: unsupported shape (B %d, %dx%d, cin %d, cout %d)", a.B, a.H, a.W, a.cin, a.cout);
    PCX_CHECK_ARG(wino4_supports(pro, epi), "conv3x3_wino4: prologue %d / epilogue %d", pro, epi);
    PCX_CHECK_ARG(a.nblk == g.nblk, "conv3x3_wino4: partial buffer sized for %d tiles, need %d", a.nblk, g.nblk);
    PCX_CHECK_ARG(a.src_guard, "conv3x3_wino4: needs 4 readable bytes before src (ConvArgs::src_guard)");
    PCX_CHECK_ARG(epi != EPI_BWD_POOLSELP || (a.ysel && a.dpool), "conv3x3_wino4: EPI_BWD_POOLSELP needs ysel, dpool");
    PCX_CHECK_ARG(epi != EPI_BWD_RELU || a.yprev, "conv3x3_wino4: EPI_BWD_RELU needs yprev");
    const size_t smem = wino4_lds_bytes(a.cin);
    PCX_CHECK_ARG(smem <= 160 * 1024, "conv3x3_wino4: %zu B of LDS", smem);
    const int64_t units = (int64_t)g.nblk * g.ncg;
    int64_t nwg = std::min<int64_t>(units, (int64_t)num_cus());
    if (nwg >= 8) nwg &= ~(int64_t)7;
    dim3 grid((unsigned)nwg);
#define PCX_W4_CASE(P_, E_)                                                                             \
    if (pro == P_ && epi == E_) {                                                                       \
        (void)hipFuncSetAttribute((const void*)conv_wino4_kernel<P_, E_>,                               \
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);               \
        conv_wino4_kernel<P_, E_><<<grid, 256, smem, s>>>(a, g);                                        \
        PCX_LAUNCH_CHECK("conv_wino4_kernel");                                                          \
        return PCX_OK;                                                                                  \
    }
    PCX_W4_CASE(PRO_BNRELU, EPI_FWD)
    PCX_W4_CASE(PRO_RAW, EPI_FWD)
    PCX_W4_CASE(PRO_RAW, EPI_BWD_RELU)
    PCX_W4_CASE(PRO_RAW, EPI_BWD_POOLSELP)
#undef PCX_W4_CASE
    set_error("conv3x3_wino4: unsupported combination (pro %d epi %d)", pro, epi);
    return PCX_EINVAL;
}

}  // namespace pcx
