// Backward of cnn_small's layer 2 (32 -> 32 channels, 3x3, stride 1, pad 1 at 40 x 200) in ONE pass:
// the Winograd F(2x2, 3x3) weight gradient and data gradient from a single staging of dz, y (-> dy, the
// BN backward) and y_prev (-> x = relu(BN_prev(y_prev))).
//
// Separately (wgrad_wino + conv_wino) the two kernels move 16.8 + 12.6 GB per B = 4096 step (dz, y,
// y_prev read, dy written; dy, y_prev read, dz_prev written) and the weight gradient is bound by that
// stream (round 3: 5.1 + 4.3 ms, PMC 20.5 + 19 GB).  Fused, dz / y / y_prev are read once and dz_prev
// written once (16.8 GB), dy never leaves the CU, and both GEMMs share the staged rows.
//
// Reference ops: the autograd of conv2 -> BN2 (phoneme_cnn.py:39-40) and of ReLU(BN1) (:35-38).
//
//   weight gradient   dW = G^T dU G,  dU_xi[n][c] = sum_tiles Yh_xi[n][tile] V_xi[c][tile]     (wgrad_wino.hip)
//   data gradient     dx_tile = A^T [ sum_n U'_xi[c][n] V'_xi[n][tile] ] A,  V' = B^T dy_patch B,
//                     U' = G g' G^T of the flipped weights (launch_wino_pack flip 1)           (conv_wino.hip)
//   epilogue          dz_prev = dx [BN_prev(y_prev) > 0], BN_prev backward sums (sum dz, sum dz xhat)
//
// Shape (MI355X): block = 512 threads, one per CU (148 KB of LDS), walking (sample, column strip) tasks tile
// row by tile row.  Waves 0-3 run the weight gradient (wave q: Winograd row q, 4 accumulator tiles of
// 32 x 32 on v_mfma_f32_32x32x2_f32, exactly wgrad_wino's K-step); waves 4-7 the data gradient (wave q:
// Winograd row q of the transposed conv, its 4 x 2 x 8 transformed weights resident in 64 VGPRs,
// 16-tile groups on v_mfma_f32_16x16x4_f32).  Each SIMD thus holds one wave of each GEMM, sharing its
// MFMA pipe.  The data gradient's output transform combines the 4 Winograd rows, so its waves exchange
// (M A) rows through a double-buffered LDS buffer at each 16-tile group, behind one block barrier.
//
// Staging: dy and x live in 4-row LDS rings (rows 2 tr - 1 .. 2 tr + 2 of tile row tr) holding the
// strip's columns plus a one-column halo on either side (position p <-> image column 2 t0 - 1 + p): the
// data gradient's 4 x 4 dy patches and the weight gradient's x patches are two aligned ds_read_b64 per
// row; the weight gradient's 2 x 2 dy values are the middle pair of the same reads.  The next tile row's
// two rows of dz, y, y_prev are loaded into registers over the row's groups (spread: no issue burst),
// turned into dy / x and stored after the row's last group.  Out-of-image items load 0 (buffer offsets
// beyond num_records) and stage exact zeros.  Strips are 48 / 52 tiles at W = 200 (the data gradient
// runs 16-tile groups: 7 groups per tile row, 12 % padding).
#include <type_traits>

#include "kernels.h"
#include "pk_f32.h"

#if defined(WB_KO) && (WB_KO & 4)
#define WB_KO_EPI 1
#else
#define WB_KO_EPI 0
#endif

namespace pcx {
namespace {

template <int V>
using vecf = float __attribute__((ext_vector_type(V)));
typedef float f2 __attribute__((ext_vector_type(2)));

constexpr int BUF_FLAGS = 0x00020000;
constexpr int OOB = 0x7fff0000;  // beyond every num_records: loads return 0
constexpr int CH = 32;           // channels in and out
constexpr int SMAX = 52;         // widest strip (tiles): LDS

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const float* base, int64_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), (short)0, (int)bytes, BUF_FLAGS);
}

template <int V>
__device__ __forceinline__ vecf<V> bload(__amdgpu_buffer_rsrc_t r, int voff) {
    if constexpr (V == 4)
        return __builtin_bit_cast(vecf<4>, __builtin_amdgcn_raw_buffer_load_b128(r, voff, 0, 0));
    else
        return __builtin_bit_cast(vecf<2>, __builtin_amdgcn_raw_buffer_load_b64(r, voff, 0, 0));
}

// single v_fma_f32 (no SLP packing next to the stores of the same registers: see wgrad_s.hip)
__device__ __forceinline__ float fma1(float a, float b, float c) {
    float r;
    asm("v_fma_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

__device__ __forceinline__ f2 ld2(const float* p) { return *reinterpret_cast<const f2*>(p); }

__device__ __forceinline__ f32x4 mfma16(float a, float b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// ---- weight gradient K-step (two tiles): x rows w, u of the lane's input channel, dy rows d0, d1 of
// its output channel (the middle pair of the 4-column patch reads)
struct WOps {
    f2 w0, w1, u0, u1, a0, a1, b0, b1;
};

typedef __attribute__((address_space(3))) const float lds_f;
__device__ __forceinline__ f2 ld2(lds_f* p) { return *reinterpret_cast<const __attribute__((address_space(3))) f2*>(p); }

__device__ __forceinline__ WOps wload(lds_f* w, lds_f* u, lds_f* d0, lds_f* d1, int s) {
    const int p = 4 * s;
    WOps o;
    o.w0 = ld2(w + p);
    o.w1 = ld2(w + p + 2);
    o.u0 = ld2(u + p);
    o.u1 = ld2(u + p + 2);
    o.a0 = ld2(d0 + p);
    o.a1 = ld2(d0 + p + 2);
    o.b0 = ld2(d1 + p);
    o.b1 = ld2(d1 + p + 2);
    return o;
}

// V row Q from e = w + sx u; Yh' row Q from pr = r0 + sy r1 (as wgrad_wino.hip kmul, packed: pk_f32.h; px / py
// are the middle pair of the 4-column dy reads, not a register pair, so they stay two scalar fma)
__device__ __forceinline__ void wmul(const WOps& o, const PkK& k, f2 sxx, float sy, f32x16 (&acc)[4]) {
    const f2 e01 = __builtin_elementwise_fma(o.u0, sxx, o.w0), e23 = __builtin_elementwise_fma(o.u1, sxx, o.w1);
    const f2 pp = {fmaf(sy, o.b0.y, o.a0.y), fmaf(sy, o.b1.x, o.a1.x)};
    const f2 b03 = pk_sub(k, e01, e23);
    const f2 b12 = __builtin_elementwise_fma(e01.yy, k.pm, e23.xx);
    const f2 a12 = __builtin_elementwise_fma(pp.yy, k.pm, pp.xx);
    acc[0] = mfma32(pp.x, b03.x, acc[0]);
    acc[1] = mfma32(a12.x, b12.x, acc[1]);
    acc[2] = mfma32(a12.y, b12.y, acc[2]);
    acc[3] = mfma32(pp.y, b03.y, acc[3]);
}

// (M A) exchange offset of row Q's pair for (channel, tile) pair p = 16 c + t: Q-major, 2 floats per pair, the
// 32-float halves of each 64-float block swapped for odd c >> 2.  A data-gradient wave's write (lanes: 4 channels
// c = 4 n_l + r apart by 4, 16 tiles) then covers the 64 banks once per 32 lanes, and the epilogue's reads
// (consecutive p per lane) are contiguous; round 5's [p][Q][2] layout put the 64 lanes of a write on 8 bank
// pairs (8-way conflicts; SQ_LDS_BANK_CONFLICT 2.36 cycles per LDS instruction in the kernel)
__device__ __forceinline__ int xoff(int q, int p) { return q * 1024 + ((2 * p) ^ (((p >> 6) & 1) << 5)); }

// XCT: the ring's channel stride as a compile-time constant (LDS offsets become instruction immediates:
// ~20 address VALU per 16-tile group less), or 0 for a runtime stride
// PD: dz rebuilt from the pooled gradient and the window selection (WinoBwdArgs::dzpool / parg)
template <int V, int NIR, int XCT, bool PD>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2))) void wgbd_wino_kernel(WinoBwdArgs a) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    constexpr int NIT = 2 * NIR;  // staged items per thread and stage (two rows)
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const bool dg = wave >= 4;  // data-gradient wave
    const int Q = wave & 3;
    const int XCS = XCT ? XCT : a.XCS, H = a.H, W = a.W, HW = H * W;
    float* const xr = smem + 4;                // x ring [4][32][XCS]
    float* const dr = xr + 4 * CH * XCS;       // dy ring [4][32][XCS]
    float* const xb = dr + 4 * CH * XCS;       // (M A) exchange [2][4 Q][512 (c, tile) pairs p][2] (xoff)
    const int slice = blockIdx.x;
    const int TR = (H + 1) >> 1;

    // ---- staging items: channel ch, vectors k = j0 + 16 m of each of the stage's two rows
    const int ch = tid >> 4, j0 = tid & 15;
    const float4 kd = a.cf_dy[ch];  // {a, mb, mgi, mean}: dy = a (dz - mb - (y - mean) mgi)
    const float A1 = kd.x, A2 = -kd.x * kd.z, A3 = kd.x * (kd.w * kd.z - kd.y);
    const float4 kx = a.cf_x[ch];
    const float xs = kx.x, xt = kx.y;
    vecf<V> dzv[NIT], yv[NIT], xv[NIT];
    static_assert(!PD || V == 4, "pooled dz: 4-column items (two pooled columns)");
    vecf<2> dpv[NIT];     // PD: the items' two pooled gradients
    unsigned pav[NIT];    // PD: their two selection bytes

    // ---- Winograd row constants (both GEMMs combine the same patch rows: B^T row Q)
    const int IW = Q == 0 ? 0 : Q == 2 ? 2 : 1, IU = Q == 0 ? 2 : Q == 2 ? 1 : Q == 1 ? 2 : 3;
    const float sx = Q == 1 ? 1.f : -1.f;
    const f2 sxx = {sx, sx};
    const PkK pk = pk_consts();
    // weight gradient: lane channel c32, tile parity g2; dy output rows 2 tr (patch row 1) / 2 tr + 1 (row 2)
    const int c32 = lane & 31, g2 = lane >> 5;
    const int ID0 = Q == 3 ? 2 : 1;
    const float sy = Q == 1 ? 1.f : Q == 2 ? -1.f : 0.f;
    // 64 registers that are the weight gradient's accumulators in waves 0-3 and the data gradient's
    // resident A operands in waves 4-7 (one array, so the allocator does not keep both live)
    f32x16 R[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) R[e] = 0.f;
    // data gradient: lane (n_l = lane >> 4, t_l = lane & 15); A operand U'[Q][e][c = 16 cs + t_l][n = 4 ks + n_l]
    // in R[(2 ks + cs) >> 2][4 ((2 ks + cs) & 3) + e]
    const int n_l = lane >> 4, t_l = lane & 15;
    if (dg) {
#pragma unroll
        for (int ks = 0; ks < 8; ++ks)
#pragma unroll
            for (int cs = 0; cs < 2; ++cs) {
                const f32x4 v = *reinterpret_cast<const f32x4*>(a.up + (((4 * ks + n_l) * 4 + Q) * 128 + (16 * cs + t_l) * 4));
                const int j = 2 * ks + cs;
#pragma unroll
                for (int e = 0; e < 4; ++e) R[j >> 2][4 * (j & 3) + e] = v[e];
            }
    }
    // epilogue (data-gradient waves): pairs p = ld + 256 k2 -> channel p >> 4 (k2 = 0: ld >> 4, 1: + 16), tile p & 15
    const int ld = tid - 256;
    // the lane's BN_prev sums over its tasks: float per tile row, then float64 kept in LDS (registers)
    double* const bsum = reinterpret_cast<double*>(xb + 2 * 4096) + 4 * (dg ? ld : 0);
    if (dg)
        for (int i = 0; i < 4; ++i) bsum[i] = 0.0;
    // epilogue coefficients per channel: the epilogue reads the staged x = relu(s yp + t) instead of yp
    // (no global load inside the row loop: a vmcnt wait there would also wait for the next row's staging
    // loads), so mask = [x > 0] (exactly [s yp + t > 0]) and, where the mask is on, x = s yp + t, hence
    // xhat = (yp - mean) invstd = x r1 + r0 with r1 = invstd / s, r0 = -(t / s + mean) invstd
    // That recovery loses ~eps |t / s| invstd of xhat and cannot work at s == 0 (BN_prev gamma 0: x is the
    // constant relu(t)); such channels (|t| invstd > 16 |s|, NaN-safe) read yp itself in the epilogue: a
    // block-uniform slow path (flag `rare`), so the common path keeps its loop free of global loads.
    // (rare channels: ecf = {0, 0}, ecf_yp = {invstd, -mean invstd}, applied to yp)
    float2* const ecf = reinterpret_cast<float2*>(xb + 2 * 4096 + 2048);
    float2* const ecf_yp = ecf + CH;
    int* const rare = reinterpret_cast<int*>(ecf_yp + CH);
    if (tid == 0) *rare = 0;
    __syncthreads();
    if (tid < CH) {
        const float4 k = a.cf_x[tid];
        const bool ok = fabsf(k.x) * 16.f >= fabsf(k.y) * k.w && k.x != 0.f;
        const float r1 = ok ? k.w / k.x : 0.f;
        ecf[tid] = ok ? make_float2(r1, -(k.y * r1) - k.z * k.w) : make_float2(0.f, 0.f);
        ecf_yp[tid] = ok ? make_float2(0.f, 0.f) : make_float2(k.w, -k.z * k.w);
        if (!ok) atomicOr(rare, 1);
    }

    // the task loop is instantiated once per wave role (the weight-gradient and the data-gradient code
    // then get their registers allocated separately: one loop with a runtime branch spilled); both
    // instantiations execute the same barriers
    auto run = [&](auto role) {
    constexpr bool DG = decltype(role)::value;
    const int t0s = slice * a.per_slice, t1s = min(a.ntask, t0s + a.per_slice);
    // paired: the two strips of a sample run at the same time on two blocks of one XCD (slice, slice + 8),
    // so the 128-byte lines around the strip boundary are fetched once into that XCD's L2; each block
    // alternates strips (48 / 52 tiles), so the pair keeps pace
    const int pair = (slice >> 4) * 8 + (slice & 7), prole = (slice >> 3) & 1;
    const int nk = a.paired ? a.per_slice : t1s - t0s;
    for (int k = 0; k < nk; ++k) {
        int b, seg;
        if (a.paired) {
            b = pair * a.per_slice + k;
            seg = (k + prole) & 1;
        } else {
            const int task = t0s + k;
            b = task / a.nseg;
            seg = task - b * a.nseg;
        }
        const int t0 = a.seg_t0[seg], S = a.seg_S[seg];
        const int c0 = 2 * t0;
        const int ng = (S + 15) >> 4, Ks = S >> 1;
        const int64_t pb = (int64_t)b * CH * HW;
        const int Wp = W >> 1, HWp = (H >> 1) * Wp;
        const int64_t pbp = (int64_t)b * CH * HWp;
        const __amdgpu_buffer_rsrc_t rdz = PD ? rsrc(a.dzpool + pbp, (int64_t)CH * HWp * 4) : rsrc(a.dz + pb, (int64_t)CH * HW * 4);
        const __amdgpu_buffer_rsrc_t rpa = rsrc(reinterpret_cast<const float*>(PD ? a.parg + pbp : nullptr),
                                                PD ? (int64_t)CH * HWp : 0);
        const __amdgpu_buffer_rsrc_t ry = rsrc(a.y + pb, (int64_t)CH * HW * 4);
        const __amdgpu_buffer_rsrc_t rx = rsrc(a.yp + pb, (int64_t)CH * HW * 4);
        // item columns: c0 - V + V k .. + V - 1 (all in or all out: V divides W and c0); LDS position V k - V + 1
        const int nx = (2 * S + 1 + V - 1) / V + 1;
        unsigned colok = 0;
#pragma unroll
        for (int m = 0; m < NIT; ++m) {
            const int k = j0 + 16 * (m % NIR);
            colok |= (unsigned)(k < nx && (unsigned)(c0 - V + V * k) < (unsigned)W) << m;
        }
        unsigned exist = 0;
#pragma unroll
        for (int m = 0; m < NIT; ++m) exist |= (unsigned)(j0 + 16 * (m % NIR) < nx) << m;
        constexpr unsigned R1 = ((1u << NIR) - 1) << NIR;
        auto rowmask = [&](int st) {  // items of stage st (rows 2 st + 1, 2 st + 2) inside the image
            const int r0 = 2 * st + 1, r1 = 2 * st + 2;
            return colok & (((unsigned)r0 < (unsigned)H ? ~R1 : 0u) | ((unsigned)r1 < (unsigned)H ? R1 : 0u));
        };
        auto goff = [&](int m, int st) { return ch * HW + (2 * st + 1 + m / NIR) * W + c0 - V + V * (j0 + 16 * (m % NIR)); };
        // PD: the item's pooled offset: row (2 st + 1 + r) / 2 = st + r (r = m / NIR), columns
        // (c0 - V + V k) / 2 .. + 1 for k = j0 + 16 (m % NIR)
        auto poff_ = [&](int m, int st, int pbase) { return pbase + (st + m / NIR) * Wp + (V / 2) * 16 * (m % NIR); };
        // items of stage st loaded at group gi of ngr (all of them for ngr = 0): the next tile row's loads
        // are spread over the current row's groups (a burst of 3 NIT loads per wave at the row start stalls
        // the issuing waves of every SIMD on the texture unit, MFMA pipes idle)
        auto load = [&](int st, int gi, int ngr) {
#if defined(WB_KO) && (WB_KO & 8)  // analysis builds only (tools/wb_ko.sh): no staging loads
            for (int m = 0; m < NIT; ++m) dzv[m] = yv[m] = xv[m] = vecf<V>(0.f);
            return;
#endif
            const unsigned ok = rowmask(st);
            int pbase = ch * HWp + ((c0 - V + V * j0) >> 1);
            if constexpr (PD) asm volatile("" : "+v"(pbase));  // opaque: offsets formed at the loads
#pragma unroll
            for (int m = 0; m < NIT; ++m) {
                if (ngr && (m * ngr) / NIT != gi) continue;
                const int o = (ok >> m) & 1 ? 4 * goff(m, st) : OOB;
                if constexpr (PD) {
                    const int op = (ok >> m) & 1 ? poff_(m, st, pbase) : OOB / 4;
                    dpv[m] = bload<2>(rdz, 4 * op);
                    pav[m] = (unsigned)__builtin_amdgcn_raw_buffer_load_b16(rpa, op, 0, 0);
                } else {
                    dzv[m] = bload<V>(rdz, o);
                }
                yv[m] = bload<V>(ry, o);
                xv[m] = bload<V>(rx, o);
            }
        };
        auto store = [&](int st) {
            const unsigned ok = rowmask(st);
            // the per-thread LDS base, opaque per call: left alone the compiler precomputes every (slot,
            // item) address once per kernel and spills them
            int lb = ch * XCS + V * j0 - (V - 1);
            asm volatile("" : "+v"(lb));
#pragma unroll
            for (int m = 0; m < NIT; ++m) {
                if (!((exist >> m) & 1)) continue;
                const bool in = (ok >> m) & 1;
                const float a3 = in ? A3 : 0.f, tt = in ? xt : 0.f;
                if constexpr (PD) {
                    // dz of the 4 columns: each pooled gradient goes to its window's selected element (row
                    // parity i of this image row, column parity j), zero elsewhere
                    const unsigned i2 = 2u * (unsigned)((2 * st + 1 + m / NIR) & 1);
#pragma unroll
                    for (int e = 0; e < V; ++e) {
                        const unsigned sel = (pav[m] >> (8 * (e >> 1))) & 3u;
                        dzv[m][e] = sel == i2 + (unsigned)(e & 1) ? dpv[m][e >> 1] : 0.f;
                    }
                }
                vecf<V> d, x;
#pragma unroll
                for (int e = 0; e < V; ++e) {
                    d[e] = fma1(A1, dzv[m][e], fma1(A2, yv[m][e], a3));
                    x[e] = fmaxf(fmaf(xv[m][e], xs, tt), 0.f);
                }
                const int rho = 2 * st + 1 + m / NIR;
                const int o = ((rho + 1) & 3) * CH * XCS + lb + V * 16 * (m % NIR);
                float* pd = dr + o;
                float* px = xr + o;
                if constexpr (V == 4) {  // positions 4k - 3 .. 4k: the middle pair 8-byte aligned
                    pd[0] = d[0];
                    *reinterpret_cast<f2*>(pd + 1) = f2{d[1], d[2]};
                    pd[3] = d[3];
                    px[0] = x[0];
                    *reinterpret_cast<f2*>(px + 1) = f2{x[1], x[2]};
                    px[3] = x[3];
                } else {
                    pd[0] = d[0];
                    pd[1] = d[1];
                    px[0] = x[0];
                    px[1] = x[1];
                }
            }
        };

        // task prologue: stage -1 (rows -1, 0) and stage 0 (rows 1, 2)
        load(-1, 0, 0);
        store(-1);
        load(0, 0, 0);
        store(0);
        __syncthreads();

        for (int tr = 0; tr < TR; ++tr) {
            const bool pre = tr + 1 < TR;
            // ring rows of this tile row: patch row i (image row 2 tr - 1 + i) in slot (2 tr + i) & 3
            const int sw = ((2 * tr + IW) & 3) * CH * XCS, su = ((2 * tr + IU) & 3) * CH * XCS;
            float rz[2] = {0.f, 0.f}, rx_[2] = {0.f, 0.f};  // this row's BN sums (data-gradient epilogue)
            float ex[2][4];                                  // the epilogue's x values (prefetched)
            for (int g = 0; g < ng; ++g) {
#ifndef WB_LOADPOS
#define WB_LOADPOS 1
#endif
                // the next tile row's staging loads, spread over the groups: the weight-gradient waves at the
                // group start, the data-gradient waves after the group's MFMAs (WB_LOADPOS 1; same-box A/B
                // 7.38-7.41 -> 7.29-7.33 ms against all waves at the group start, 0; 2 = all items at once,
                // weight-gradient waves at group 0, data-gradient waves after group 1's MFMAs: slower)
                if (pre && (WB_LOADPOS == 0 || (WB_LOADPOS == 1 && !DG))) load(tr + 1, g, ng);
                if (pre && WB_LOADPOS == 2 && !DG && g == 0) load(tr + 1, 0, 0);
                if constexpr (!DG) {
#if !(defined(WB_KO) && (WB_KO & 1))
                    // ---- weight gradient: K-steps 8 g .. 8 g + 7 (tiles 16 g .. 16 g + 15)
                    // (LDS pointers advanced once per two K-steps: every read is a base register plus an
                    // immediate; the look-ahead read past an even group end stays inside the LDS row, unused)
                    const int s0 = 8 * g, s1 = min(8 * g + 8, Ks);
                    lds_f* w = (lds_f*)(xr + sw + c32 * XCS + 2 * g2 + 4 * s0);
                    lds_f* u = (lds_f*)(xr + su + c32 * XCS + 2 * g2 + 4 * s0);
                    lds_f* d0 = (lds_f*)(dr + ((2 * tr + ID0) & 3) * CH * XCS + c32 * XCS + 2 * g2 + 4 * s0);
                    lds_f* d1 = (lds_f*)(dr + ((2 * tr + 2) & 3) * CH * XCS + c32 * XCS + 2 * g2 + 4 * s0);
                    asm volatile("" : "+v"(w), "+v"(u), "+v"(d0), "+v"(d1));
                    WOps A = wload(w, u, d0, d1, 0);
                    int s = s0;
                    for (; s + 2 <= s1; s += 2) {
                        const WOps Bn = wload(w, u, d0, d1, 1);
                        __builtin_amdgcn_sched_barrier(0);
                        wmul(A, pk, sxx, sy, R);
                        __builtin_amdgcn_sched_barrier(0);
                        A = wload(w, u, d0, d1, 2);
                        __builtin_amdgcn_sched_barrier(0);
                        wmul(Bn, pk, sxx, sy, R);
                        __builtin_amdgcn_sched_barrier(0);
                        w += 8;
                        u += 8;
                        d0 += 8;
                        d1 += 8;
                    }
                    if (s < s1) wmul(A, pk, sxx, sy, R);
#endif
                } else {
#if !(defined(WB_KO) && (WB_KO & 2))
                    // ---- data gradient: tiles 16 g + t_l (clamped into the strip), K = 32 dy channels
                    const int tl = min(16 * g + t_l, S - 1);
                    const float* pw = dr + sw + n_l * XCS + 2 * tl;
                    const float* pu = dr + su + n_l * XCS + 2 * tl;
                    f32x4 acc[4][2];
#pragma unroll
                    for (int e = 0; e < 4; ++e) acc[e][0] = acc[e][1] = f32x4{0.f, 0.f, 0.f, 0.f};
                    // software-pipelined: the reads of K-step ks + 1 are in flight under the MFMAs of ks
                    f2 op[2][4];
                    auto dload = [&](f2 (&o)[4], int ks) {
                        o[0] = ld2(pw + 4 * ks * XCS);
                        o[1] = ld2(pw + 4 * ks * XCS + 2);
                        o[2] = ld2(pu + 4 * ks * XCS);
                        o[3] = ld2(pu + 4 * ks * XCS + 2);
                    };
                    dload(op[0], 0);
#pragma unroll
                    for (int ks = 0; ks < 8; ++ks) {
                        if (ks + 1 < 8) dload(op[(ks + 1) & 1], ks + 1);
                        __builtin_amdgcn_sched_barrier(0);
                        const f2* o = op[ks & 1];
                        // (packed: {q0, q1}, {q2, q3}, {q0 - q2, q1 - q3}, {q1 + q2, q2 - q1}; pk_f32.h)
                        const f2 q01 = __builtin_elementwise_fma(o[2], sxx, o[0]);
                        const f2 q23 = __builtin_elementwise_fma(o[3], sxx, o[1]);
                        const f2 b03 = pk_sub(pk, q01, q23);
                        const f2 b12 = __builtin_elementwise_fma(q01.yy, pk.pm, q23.xx);
                        const float v[4] = {b03.x, b12.x, b12.y, b03.y};
#pragma unroll
                        for (int e = 0; e < 4; ++e)
#pragma unroll
                            for (int cs = 0; cs < 2; ++cs)
                                acc[e][cs] = mfma16(R[(2 * ks + cs) >> 2][4 * ((2 * ks + cs) & 3) + e], v[e], acc[e][cs]);
                        __builtin_amdgcn_sched_barrier(0);
                    }
                    // (M A) row Q: j = 0: e0 + e1 + e2, j = 1: e1 - e2 - e3; D row 4 n_l + r, column t_l
                    float* xo = xb + (g & 1) * 4096;
#pragma unroll
                    for (int cs = 0; cs < 2; ++cs)
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            const int c = 16 * cs + 4 * n_l + r;
                            const float m0 = acc[0][cs][r] + acc[1][cs][r] + acc[2][cs][r];
                            const float m1 = acc[1][cs][r] - acc[2][cs][r] - acc[3][cs][r];
                            *reinterpret_cast<f2*>(xo + xoff(Q, c * 16 + t_l)) = f2{m0, m1};
                        }
#endif
                    if (pre && WB_LOADPOS == 1) load(tr + 1, g, ng);
                    if (pre && WB_LOADPOS == 2 && g == min(1, ng - 1)) load(tr + 1, 0, 0);
                    // the epilogue's x values (rows 2 tr, 2 tr + 1 = ring slots of patch rows 1, 2) read
                    // before the barrier: after the last group's barrier the next stage overwrites row 2 tr
                    const int so1 = ((2 * tr + 1) & 3) * CH * XCS, so2 = ((2 * tr + 2) & 3) * CH * XCS;
#pragma unroll
                    for (int k2 = 0; k2 < 2; ++k2) {
                        const int p = ld + 256 * k2, c = p >> 4, tile = min(16 * g + (p & 15), S - 1);
                        const float* xp = xr + c * XCS + 2 * tile + 1;
                        ex[k2][0] = xp[so1];
                        ex[k2][1] = xp[so1 + 1];
                        ex[k2][2] = xp[so2];
                        ex[k2][3] = xp[so2 + 1];
                    }
                }
                __syncthreads();  // group g's (M A) rows visible; group g - 1's exchange buffer consumed
                if constexpr (DG && !(WB_KO_EPI)) {
                    // ---- epilogue of group g: dx = A^T (M A) over the 4 rows, ReLU(BN_prev) mask, BN_prev sums
                    const float* xi = xb + (g & 1) * 4096;
                    const int h0 = 2 * tr;
                    const bool r1ok = h0 + 1 < H;
#pragma unroll
                    for (int k2 = 0; k2 < 2; ++k2) {
                        const int p = ld + 256 * k2, c = p >> 4, tile = 16 * g + (p & 15);
                        if (tile >= S) continue;
                        const f2 v0 = *reinterpret_cast<const f2*>(xi + xoff(0, p));
                        const f2 v1 = *reinterpret_cast<const f2*>(xi + xoff(1, p));
                        const f2 v2 = *reinterpret_cast<const f2*>(xi + xoff(2, p));
                        const f2 v3 = *reinterpret_cast<const f2*>(xi + xoff(3, p));
                        const f32x4 m0 = {v0.x, v0.y, v1.x, v1.y};
                        const f32x4 m1 = {v2.x, v2.y, v3.x, v3.y};
                        // m0 = {q0 j0, q0 j1, q1 j0, q1 j1}, m1 = {q2 j0, q2 j1, q3 j0, q3 j1}
                        const float y00 = m0[0] + m0[2] + m1[0], y01 = m0[1] + m0[3] + m1[1];
                        const float y10 = m0[2] - m1[0] - m1[2], y11 = m0[3] - m1[1] - m1[3];
                        const int64_t o = pb + (int64_t)c * HW + h0 * W + 2 * (t0 + tile);
                        const float2 k = ecf[c];
                        const float gv[4] = {y00, y01, y10, y11};
                        float dz[4], xh[4];
#pragma unroll
                        for (int e = 0; e < 4; ++e) xh[e] = fmaf(ex[k2][e], k.x, k.y);
                        if (__builtin_amdgcn_readfirstlane(*rare)) {  // block-uniform: some channel's BN_prev scale is (near) zero
                            const float2 kr = ecf_yp[c];
                            if (kr.x != 0.f) {
                                const float* yq = a.yp + o;
#pragma unroll
                                for (int e = 0; e < 4; ++e)
                                    xh[e] = (e < 2 || r1ok) ? fmaf(yq[(e >> 1) * W + (e & 1)], kr.x, kr.y) : 0.f;
                            }
                        }
#pragma unroll
                        for (int e = 0; e < 4; ++e) {
                            const float xe = ex[k2][e];  // 0 outside the image (row H of an odd H)
                            dz[e] = xe > 0.f ? gv[e] : 0.f;
                            rz[k2] += dz[e];
                            rx_[k2] = fmaf(dz[e], xh[e], rx_[k2]);
                        }
                        if constexpr (PCX_AB_NO_NT_STORES) {
                            *reinterpret_cast<float2*>(a.dzp + o) = make_float2(dz[0], dz[1]);
                            if (r1ok) *reinterpret_cast<float2*>(a.dzp + o + W) = make_float2(dz[2], dz[3]);
                        } else {  // (streaming stores: dz_prev is read once, by the layer-1 weight gradient)
                            __builtin_nontemporal_store(f2{dz[0], dz[1]}, reinterpret_cast<f2*>(a.dzp + o));
                            if (r1ok) __builtin_nontemporal_store(f2{dz[2], dz[3]}, reinterpret_cast<f2*>(a.dzp + o + W));
                        }
                    }
                }
            }
            if constexpr (DG) {
#pragma unroll
                for (int k2 = 0; k2 < 2; ++k2) {
                    bsum[k2] += (double)rz[k2];
                    bsum[2 + k2] += (double)rx_[k2];
                }
            }
            // every ring read of this tile row precedes the last group's barrier: stage the next rows
            if (pre) store(tr + 1);
            __syncthreads();
        }
    }
    };
    if (dg) run(std::true_type{});
    else run(std::false_type{});
    // ---- outputs: weight-gradient partials (as wgrad_wino: row (r & 3) + 8 (r >> 2) + 4 g2, column c32)
    if (!dg) {
        float* out = a.part + (int64_t)slice * CH * CH * 16;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int co = (r & 3) + 8 * (r >> 2) + 4 * g2;
            *reinterpret_cast<float4*>(out + ((int64_t)co * CH + c32) * 16 + 4 * Q) =
                make_float4(R[0][r], R[1][r], R[2][r], R[3][r]);
        }
    } else {
        // BN_prev backward partials [32][nslice]: the 16 lanes of a channel summed in a fixed order
#pragma unroll
        for (int k2 = 0; k2 < 2; ++k2) {
            double bz = bsum[k2], bx = bsum[2 + k2];
#pragma unroll
            for (int o = 1; o < 16; o <<= 1) {
                bz += __shfl_xor(bz, o, 64);
                bx += __shfl_xor(bx, o, 64);
            }
            if ((ld & 15) == 0) {
                const int c = 16 * k2 + (ld >> 4);
                a.bn0[(int64_t)c * a.nslice + slice] = (float)bz;
                a.bn1[(int64_t)c * a.nslice + slice] = (float)bx;
            }
        }
    }
}

int smallest_2odd(int n) {  // smallest m >= n with m = 2 * odd
    while ((n & 3) != 2) ++n;
    return n;
}

}  // namespace

bool wgbd_wino_geometry(int B, int H, int W, int C, WinoBwdArgs* a) {
    if (C != CH || H < 2 || W < 8 || (W & 3) != 0) return false;  // (V = 4: 16-byte items)
    const int TC = W / 2;
    if (TC & 1) return false;  // strips of whole K-steps (two tiles)
    const int nseg = ceil_div(TC, SMAX);
    if (nseg > 4) return false;
    int S[4] = {0, 0, 0, 0};
    // strips of 16-tile multiples where possible (the data gradient runs 16-tile groups), the last the rest
    int base = (TC / nseg) & ~15;
    if (nseg == 1) base = TC;
    int last = TC - base * (nseg - 1);
    if (base <= 0 || last <= 0 || last > SMAX || (last & 1)) {
        base = ((ceil_div(TC, nseg) + 1) & ~1);
        last = TC - base * (nseg - 1);
        if (last <= 0 || last > SMAX || base > SMAX || (last & 1)) return false;
    }
    for (int i = 0; i < nseg; ++i) S[i] = i + 1 < nseg ? base : last;
    const int V = 4;
    int smax = 0;
    for (int i = 0; i < nseg; ++i) smax = std::max(smax, S[i]);
    const int kmax = (2 * smax + 1 + V - 1) / V, nx = kmax + 1;
    if (nx > 16 * 2) return false;  // 16 threads x NIR = 2 items per row and channel
    const int XCS = smallest_2odd(std::max(V * kmax + 1, 2 * smax + 5));
    // rings, exchange buffer, the lanes' float64 sums, the epilogue coefficients
    const size_t lds = ((size_t)4 + 8 * CH * XCS + 2 * 4096) * 4 + 256 * 4 * 8 + 2 * CH * 8 + 16;
    if (lds > 160 * 1024) return false;
    if ((int64_t)CH * H * W * 4 >= OOB) return false;
    if (a) {
        a->nseg = nseg;
        int t0 = 0;
        for (int i = 0; i < 4; ++i) {
            a->seg_t0[i] = t0;
            a->seg_S[i] = S[i];
            t0 += S[i];
        }
        a->V = V;
        a->NIR = 2;
        a->XCS = XCS;
        a->lds = lds;
        a->ntask = B * nseg;
        const int want = std::min(num_cus(), a->ntask);  // one block per CU
        a->per_slice = ceil_div(a->ntask, want);
        a->nslice = ceil_div(a->ntask, a->per_slice);
        // XCD-paired strips (PCX_AB_WGBD_UNPAIRED: each block walks its own run of tasks)
        constexpr bool unpaired = PCX_AB_WGBD_UNPAIRED;
        a->paired = !unpaired && nseg == 2 && a->nslice % 16 == 0 && a->nslice * a->per_slice == a->ntask;
    }
    return true;
}

int launch_wgbd_wino(WinoBwdArgs a, hipStream_t s) {
    WinoBwdArgs g{};
    PCX_CHECK_ARG(wgbd_wino_geometry(a.B, a.H, a.W, CH, &g), "wgbd_wino: unsupported shape %dx%d", a.H, a.W);
    PCX_CHECK_ARG(g.XCS == a.XCS && g.nslice == a.nslice && g.per_slice == a.per_slice && g.ntask == a.ntask &&
                      g.nseg == a.nseg && g.paired == a.paired,
                  "wgbd_wino: geometry mismatch");
    PCX_CHECK_ARG((a.dz != nullptr) != (a.dzpool != nullptr), "wgbd_wino: exactly one of dz / dzpool");
    PCX_CHECK_ARG(a.y && a.cf_dy && a.yp && a.cf_x && a.up && a.part && a.dzp && a.bn0 && a.bn1,
                  "wgbd_wino: NULL argument");
    const bool pd = a.dzpool != nullptr;
    if (pd) {  // pooled dz: whole windows, 2-byte aligned selection pairs (even strip starts)
        PCX_CHECK_ARG(a.parg && !(a.H & 1) && a.W % 4 == 0, "wgbd_wino: pooled dz needs parg, even H, W %% 4 == 0");
        for (int i = 0; i < a.nseg; ++i) PCX_CHECK_ARG(!(a.seg_t0[i] & 1), "wgbd_wino: odd strip start %d", a.seg_t0[i]);
    }
#define PCX_WB(XC_, PD_)                                                                               \
    if ((a.XCS == XC_ || XC_ == 0) && pd == PD_) {                                                     \
        (void)hipFuncSetAttribute((const void*)wgbd_wino_kernel<4, 2, XC_, PD_>,                       \
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)a.lds);              \
        wgbd_wino_kernel<4, 2, XC_, PD_><<<dim3((unsigned)a.nslice), 512, a.lds, s>>>(a);              \
        PCX_LAUNCH_CHECK("wgbd_wino_kernel");                                                          \
        return PCX_OK;                                                                                 \
    }
    PCX_WB(110, false) PCX_WB(110, true)  // T = 200 (strips of 48 / 52 tiles)
    PCX_WB(106, false)                    // T = 100
    PCX_WB(0, false) PCX_WB(0, true)
#undef PCX_WB
    return PCX_OK;
}

}  // namespace pcx
