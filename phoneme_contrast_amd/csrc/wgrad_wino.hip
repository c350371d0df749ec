// Weight gradient of the stride-1 3x3 convs as Winograd F(2x2, 3x3) on v_mfma_f32_32x32x2_f32.
//
//   dW[n][c] = sum over 2x2 output tiles of the adjoint of Y = A^T [(G g G^T) (.) V] A:
//   dW = G^T dU G,   dU_xi[n][c] = sum_tiles Yh_xi[n][tile] V_xi[c][tile]
//   Yh = A dY A^T (4x4 from the tile's 2x2 output gradient dy),  V = B^T d B (4x4 input patch)
//
// (reference: autograd of the 3x3 convs of phoneme_cnn.py:35-65).  Per Winograd element xi the
// tile sum is a GEMM over K = tiles with M = output channels (dy) and N = input channels (x): 16
// multiplies per tile and channel pair instead of the direct form's 36, all in float32 (the
// transforms are additions; dW = G^T dU G is evaluated in float64 from the summed partials).
// Checked in float64 (tests/test_winograd_host.py); the signs of row / column 3 of A are folded
// into the final transform (Yh' = Yh with row 3 and column 3 negated).
//
// Shape (MI355X):
//  * block = 32 output x 32 input channels, 4 waves; wave q owns the 4 Winograd elements of row q
//    of the 4x4 domain (xi = 4 q + e): 4 accumulator tiles of 32x32 (64 VGPRs), so the block's
//    waves never duplicate an MFMA, and each wave needs only the two input rows (and the one or two
//    dy rows) its row q combines: per K-step (2 tiles) 4 MFMAs against 4 + 2 ds_read_b64 and ~12 VALU.
//  * K = tiles: lane l of a K-step takes tile 2 s + (l >> 5) of the current tile row strip, channel
//    l & 31 on both operands (A = Yh (cout x tiles), B = V (tiles x cin)).
//  * a block walks (sample, column strip) tasks tile row by tile row: dy rows 2 tr, 2 tr + 1 and x
//    rows 2 tr - 1 .. 2 tr + 2 live in LDS (x in a 4-row ring: two rows carried to the next tile
//    row), the next tile row's 2 + 2 rows are loaded into registers under the current row's MFMAs
//    and stored after a barrier, the BN backward dy = A1 dz + A2 y + A3 and the producer's BN + ReLU
//    applied between load and store; the cin-group-0 blocks also write dy to HBM for the data
//    gradient.  Out-of-image items carry an out-of-range buffer offset (the hardware returns 0) and
//    a zero additive term, so they stage exact zeros; padded tiles of a K-step read zeros.
//  * x rows sit in LDS shifted by one column (position p <-> image column 2 t0 - 1 + p), so a patch
//    is two aligned ds_read_b64 per row; channel strides are 2 * odd (the 32 lanes of a read group
//    cover the 64 banks once).  Strips of <= 50 tiles keep the block at <= 80 KB: two blocks per CU.
//  * per-slice partials [slice][cout][cin][16], summed in a fixed order by wgrad_wino_reduce
//    (float64): deterministic.
#include <type_traits>

#include "kernels.h"
#include "pk_f32.h"

namespace pcx {
namespace {

template <int V>
using vecf = float __attribute__((ext_vector_type(V)));
typedef float f2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

constexpr int BUF_FLAGS = 0x00020000;  // raw buffer, 32-bit data
constexpr int OOB = 0x7fff0000;        // beyond every num_records: loads 0, stores dropped
constexpr int NIR = 4;                 // staged x vectors per thread and row: 8 threads x 4 >= 32 per channel
constexpr int NIT = 2 * NIR;           // per stage (two rows)

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const float* base, int64_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), (short)0, (int)bytes, BUF_FLAGS);
}

template <int V>
__device__ __forceinline__ vecf<V> bload(__amdgpu_buffer_rsrc_t r, int voff) {
    if constexpr (V == 4)
        return __builtin_bit_cast(vecf<4>, __builtin_amdgcn_raw_buffer_load_b128(r, voff, 0, 0));
    else if constexpr (V == 2)
        return __builtin_bit_cast(vecf<2>, __builtin_amdgcn_raw_buffer_load_b64(r, voff, 0, 0));
    else
        return vecf<1>{__builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, voff, 0, 0))};
}

template <int V>
__device__ __forceinline__ void bstore(__amdgpu_buffer_rsrc_t r, int voff, vecf<V> v) {
    if constexpr (V == 4)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), r, voff, 0, PCX_AB_NO_NT_STORES ? 0 : 2);
    else if constexpr (V == 2)
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, v), r, voff, 0, PCX_AB_NO_NT_STORES ? 0 : 2);
    else {
        const float f = v.x;  // (a named copy: no bit_cast of a vector-lane lvalue)
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, f), r, voff, 0, PCX_AB_NO_NT_STORES ? 0 : 2);
    }
}

// single v_fma_f32 (no SLP packing next to the stores of the same registers: see wgrad_s.hip)
__device__ __forceinline__ float fma1(float a, float b, float c) {
    float r;
    asm("v_fma_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}


// Operands of one K-step (2 tiles, lane tile 2 s + g): the wave's two x rows (w, u: 4 values
// each) and the two dy rows (r0, r1: 2 values each) of the lane's channel.
struct KOps {
    f2 w0, w1, u0, u1, r0, r1;
};

typedef __attribute__((address_space(3))) const float lds_f;
__device__ __forceinline__ f2 ld2(lds_f* p) { return *reinterpret_cast<const __attribute__((address_space(3))) f2*>(p); }

__device__ __forceinline__ KOps kload(lds_f* w, lds_f* u, lds_f* q0, lds_f* q1, int s) {
    const int p = 4 * s;  // 2 * (2 s + g), the lane's 2 g folded into the row bases
    KOps o;
    o.w0 = ld2(w + p);
    o.w1 = ld2(w + p + 2);
    o.u0 = ld2(u + p);
    o.u1 = ld2(u + p + 2);
    o.r0 = ld2(q0 + p);
    o.r1 = ld2(q1 + p);
    return o;
}

// V row Q = (B^T d B) row Q from e = w + sx u; Yh' row Q = (A dY A^T) row Q (row / column 3 sign-
// folded) from pr = r0 + sy r1; four 32x32x2 MFMAs.  Packed (pk_f32.h, round 6): 6 v_pk_fma_f32 instead of
// 12 scalar operations, each lane bit-identical to the scalar form:
//   {e0, e1} = fma(u0, sx, w0), {e2, e3} = fma(u1, sx, w1), {px, py} = fma(r1, sy, r0),
//   {e0 - e2, e1 - e3},  {e1 + e2, e2 - e1} = fma({e1, e1}, {1, -1}, {e2, e2}),  {px + py, px - py} likewise
__device__ __forceinline__ void kmul(const KOps& o, const PkK& k, f2 sxx, f2 syy, f32x16 (&acc)[4]) {
    const f2 e01 = __builtin_elementwise_fma(o.u0, sxx, o.w0), e23 = __builtin_elementwise_fma(o.u1, sxx, o.w1);
    const f2 pp = __builtin_elementwise_fma(o.r1, syy, o.r0);
    const f2 b03 = pk_sub(k, e01, e23);
    const f2 b12 = __builtin_elementwise_fma(e01.yy, k.pm, e23.xx);
    const f2 a12 = __builtin_elementwise_fma(pp.yy, k.pm, pp.xx);
    acc[0] = mfma32(pp.x, b03.x, acc[0]);
    acc[1] = mfma32(a12.x, b12.x, acc[1]);
    acc[2] = mfma32(a12.y, b12.y, acc[2]);
    acc[3] = mfma32(pp.y, b03.y, acc[3]);
}

// K-steps 0 .. n - 1 from the row pointers, software-pipelined: the reads of step s + 1 are in flight while
// step s multiplies (two operand sets, alternating: no register moves).  The pointers advance once per two
// steps, so each read is a base register plus an immediate offset (no address arithmetic per step); the
// last pair's look-ahead read of step n (n even) is a read past the strip inside the LDS row (unused).
__device__ __forceinline__ void kloop(const float* w_, const float* u_, const float* q0_, const float* q1_, const PkK& k,
                                      f2 sxx, f2 syy, f32x16 (&acc)[4], int n) {
    if (n <= 0) return;
    // LDS pointers, opaque: the compiler re-added a lane offset to each pointer per step instead of folding it
    // in once
    lds_f* w = (lds_f*)w_;
    lds_f* u = (lds_f*)u_;
    lds_f* q0 = (lds_f*)q0_;
    lds_f* q1 = (lds_f*)q1_;
    asm volatile("" : "+v"(w), "+v"(u), "+v"(q0), "+v"(q1));
    KOps A = kload(w, u, q0, q1, 0);
    int s = 0;
    for (; s + 2 <= n; s += 2) {
        const KOps Bn = kload(w, u, q0, q1, 1);
        __builtin_amdgcn_sched_barrier(0);  // reads issued ahead of the MFMAs they overlap
        kmul(A, k, sxx, syy, acc);
        __builtin_amdgcn_sched_barrier(0);
        A = kload(w, u, q0, q1, 2);
        __builtin_amdgcn_sched_barrier(0);
        kmul(Bn, k, sxx, syy, acc);
        __builtin_amdgcn_sched_barrier(0);
        w += 8;
        u += 8;
        q0 += 8;
        q1 += 8;
    }
    if (s < n) kmul(A, k, sxx, syy, acc);
}

// one wave's work: Winograd row Q = wave & 3 (elements 4 Q .. 4 Q + 3) of the 32 x 32 channel block of input
// channel half h = wave >> 2.  NH = 2 (round 6): a block of 8 waves covers 32 output x 64 input channels, so every
// staged dy value (two loads, the BN backward, an LDS and an HBM store) feeds twice the MFMAs; x staging per MFMA
// is unchanged.  One block per CU instead of two (the same 8 waves).
template <int PRO, int V, bool PD, int NH>
__device__ __forceinline__ void ww_body(const WinoWgradArgs& a, float* smem, int co0, int ci0, int slice) {
    const int tid = threadIdx.x, lane = tid & 63, c32 = lane & 31, g = lane >> 5;
    const int Q = __builtin_amdgcn_readfirstlane((tid >> 6) & 3);
    const int hx = __builtin_amdgcn_readfirstlane(tid >> 8);  // the wave's input channel half (NH = 2)
    constexpr int NPT = V == 4 ? 2 : 4;  // parts of the next tile row's loads (V = 4: 4 parts spill)
    constexpr int CX = 32 * NH;          // staged x channels
    constexpr int TPD = 8 * NH;          // threads per dy channel
    constexpr int NIRD = NIR / NH, NITD = 2 * NIRD;  // dy vectors per thread and row / stage
    const int XCS = a.XCS, DCS = a.DCS;
    float* const xl = smem + 4;                   // [4 ring slots][CX][XCS]
    float* const dyl = xl + 4 * CX * XCS;         // [2 rows][32][DCS]
    const int H = a.H, W = a.W, HW = H * W;
    const int nd = a.nd, nx = a.nx;

    // staging items: x: thread -> channel ch = tid >> 3 (cin ci0 + ch) and, in each of the stage's two rows r,
    // the vectors k = (tid & 7) + 8 m (m < NIR): item i = NIR r + m; dy: channel chd = tid / TPD (cout co0 + chd),
    // vectors k = jd + TPD m (m < NIRD), jd = tid % TPD.  Offsets are one per-thread base plus compile-time /
    // uniform terms.
    const int ch = tid >> 3, j0 = tid & 7;
    const int chd = tid / TPD, jd = tid % TPD;
    const int dgb = chd * HW + V * jd, dlb = chd * DCS + V * jd;
    const int xgb = ch * HW + V * j0 - V, xlb = ch * XCS + V * j0 - (V - 1);
    unsigned dex = 0, xex = 0;  // existing items (bit masks)
#pragma unroll
    for (int i = 0; i < NITD; ++i) dex |= (unsigned)(jd + TPD * (i % NIRD) < nd) << i;
#pragma unroll
    for (int i = 0; i < NIT; ++i) xex |= (unsigned)(j0 + 8 * (i % NIR) < nx) << i;
    // BN backward coefficients of this thread's dy channel, BN + ReLU of its x channel
    const float4 kd = a.cf_dy[co0 + chd];  // {a, mb, mgi, mean}: dy = a (dz - mb - (y - mean) mgi)
    const float A1 = kd.x, A2 = -kd.x * kd.z, A3 = kd.x * (kd.w * kd.z - kd.y);
    float xs = 1.f, xt = 0.f;
    if (PRO == PRO_BNRELU) {
        const float4 k = a.cf_x[ci0 + ch];
        xs = k.x;
        xt = k.y;
    }

    f32x16 acc[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) acc[e] = 0.f;

    const bool write_dy = a.dy_out != nullptr && ci0 == 0;
    const int TR = (H + 1) >> 1;
    const int t0s = slice * a.per_slice, t1s = min(a.ntask, t0s + a.per_slice);
    vecf<V> dzv[NITD], yv[NITD], xv[NIT];
    static_assert(!PD || V == 4, "pooled dz: 4-column items");
    unsigned pav[NITD];  // PD: the items' two selection bytes (their two pooled gradients wait in dzv[m][0..1])
    const int Wp = W >> 1, HWp = (H >> 1) * Wp;

    // per-task state: the sample's buffer resources and the items' column validity (whole vectors: V
    // divides W and 2 t0)
    struct Task {
        int c0;
        __amdgpu_buffer_rsrc_t rdz, rpa, ry, rdo, rx;
        unsigned dcol, xcol;
    };
    auto task_of = [&](int task) {
        Task t;
        const int b = task / a.nseg;
        const int t0 = (task - b * a.nseg) * a.S;
        t.c0 = 2 * t0;
        t.rdz = PD ? rsrc(a.dzpool + ((int64_t)b * a.cout + co0) * HWp, (int64_t)32 * HWp * 4)
                   : rsrc(a.dz + ((int64_t)b * a.cout + co0) * HW, (int64_t)32 * HW * 4);
        t.rpa = rsrc(reinterpret_cast<const float*>(PD ? a.parg + ((int64_t)b * a.cout + co0) * HWp : nullptr),
                     PD ? (int64_t)32 * HWp : 0);
        t.ry = rsrc(a.y + ((int64_t)b * a.cout + co0) * HW, (int64_t)32 * HW * 4);
        t.rdo = rsrc(write_dy ? a.dy_out + ((int64_t)b * a.cout + co0) * HW : a.dz, write_dy ? (int64_t)32 * HW * 4 : 0);
        t.rx = rsrc(a.src + ((int64_t)b * a.cin + ci0) * HW, (int64_t)CX * HW * 4);
        unsigned dcol = 0, xcol = 0;
#pragma unroll
        for (int i = 0; i < NITD; ++i) dcol |= (unsigned)(t.c0 + V * (jd + TPD * (i % NIRD)) < W) << i;
#pragma unroll
        for (int i = 0; i < NIT; ++i) {
            const int kc = V * (j0 + 8 * (i % NIR));
            xcol |= (unsigned)((unsigned)(t.c0 + kc - V) < (unsigned)W) << i;
        }
        t.dcol = dcol & dex;
        t.xcol = xcol & xex;
        return t;
    };

    // stage st (= -1 .. TR - 1): dy rows 2 st, 2 st + 1 and x rows 2 st + 1, 2 st + 2
    constexpr unsigned R1 = ((1u << NIR) - 1) << NIR;     // x items of the stage's second row
    constexpr unsigned R1D = ((1u << NIRD) - 1) << NIRD;  // dy items of the stage's second row
    auto masks = [&](const Task& t, int st, unsigned& dm, unsigned& xm) {
        const bool d0 = 2 * st >= 0, d1 = 2 * st + 1 >= 0 && 2 * st + 1 < H;
        const bool x0 = 2 * st + 1 >= 0 && 2 * st + 1 < H, x1 = 2 * st + 2 < H;
        dm = t.dcol & ((d0 ? ~R1D : 0u) | (d1 ? R1D : 0u));
        xm = t.xcol & ((x0 ? ~R1 : 0u) | (x1 ? R1 : 0u));
    };
    auto dgo = [&](int i) { return dgb + (i / NIRD) * W + TPD * V * (i % NIRD); };
    auto xgo = [&](int i) { return xgb + (i / NIR) * W + 8 * V * (i % NIR); };
    // part: only the items m with m NPT / NIT == part (-1: all items)
    auto load_dy = [&](const Task& t, int st, int part) {
        unsigned dm, xm;
        masks(t, st, dm, xm);
        int db = 2 * st * W + t.c0 + dgb;
        asm volatile("" : "+v"(db));  // opaque: per-item offsets formed at the load, not kept live
        int pb = chd * HWp + st * Wp + ((t.c0 + V * jd) >> 1);  // PD: pooled row st (dy rows 2 st, 2 st + 1)
        if constexpr (PD) asm volatile("" : "+v"(pb));
#pragma unroll
        for (int m = 0; m < NITD; ++m) {
            if (part >= 0 && m * NPT / NITD != part) continue;
            const int o = (dm >> m) & 1 ? 4 * (dgo(m) - dgb + db) : OOB;
            if constexpr (PD) {
                const int op = (dm >> m) & 1 ? pb + (TPD * V / 2) * (m % NIRD) : OOB / 4;
                const vecf<2> dp = bload<2>(t.rdz, 4 * op);
                dzv[m][0] = dp[0];
                dzv[m][1] = dp[1];
                pav[m] = (unsigned)__builtin_amdgcn_raw_buffer_load_b16(t.rpa, op, 0, 0);
            } else {
                dzv[m] = bload<V>(t.rdz, o);
            }
            yv[m] = bload<V>(t.ry, o);
        }
    };
    // dy = A1 dz + A2 y + A3 (exact 0 outside the image) into dzv
    auto form_dy = [&](const Task& t, int st) {
        unsigned dm, xm;
        masks(t, st, dm, xm);
#pragma unroll
        for (int m = 0; m < NITD; ++m) {
            const float a3 = (dm >> m) & 1 ? A3 : 0.f;
            if constexpr (PD) {  // dz: each pooled gradient at its window's selected element (row parity m / NIRD)
                const float g0 = dzv[m][0], g1 = dzv[m][1];
                const unsigned pa = pav[m], i2 = 2u * (unsigned)(m / NIRD);
#pragma unroll
                for (int e = 0; e < V; ++e)
                    dzv[m][e] = ((pa >> (8 * (e >> 1))) & 3u) == i2 + (unsigned)(e & 1) ? (e >> 1 ? g1 : g0) : 0.f;
            }
#pragma unroll
            for (int e = 0; e < V; ++e) dzv[m][e] = fma1(A1, dzv[m][e], fma1(A2, yv[m][e], a3));
        }
    };
    auto load_x = [&](const Task& t, int st, int part, vecf<V> (&xr)[NIT]) {
        unsigned dm, xm;
        masks(t, st, dm, xm);
        int xb = (2 * st + 1) * W + t.c0 + xgb;
        asm volatile("" : "+v"(xb));
#pragma unroll
        for (int m = 0; m < NIT; ++m)
            if (part < 0 || m * NPT / NIT == part) xr[m] = bload<V>(t.rx, (xm >> m) & 1 ? 4 * (xgo(m) - xgb + xb) : OOB);
    };
    auto store_x = [&](const Task& t, int st, const vecf<V> (&xr)[NIT]) {
        unsigned dm, xm;
        masks(t, st, dm, xm);
        // x rows 2 st + 1, 2 st + 2 -> ring slots (2 st + 2) & 3, (2 st + 3) & 3
        const int sl0 = ((2 * st + 2) & 3) * CX * XCS, sl1 = ((2 * st + 3) & 3) * CX * XCS;
#pragma unroll
        for (int m = 0; m < NIT; ++m) {
            if (!((xex >> m) & 1)) continue;
            vecf<V> v = xr[m];
            if (PRO == PRO_BNRELU) {
                const float tt = (xm >> m) & 1 ? xt : 0.f;
#pragma unroll
                for (int e = 0; e < V; ++e) v[e] = fmaxf(fmaf(v[e], xs, tt), 0.f);
            }
            float* d = xl + (m / NIR ? sl1 : sl0) + xlb + 8 * V * (m % NIR);
            if constexpr (V == 4) {
                d[0] = v[0];
                *reinterpret_cast<f2*>(d + 1) = f2{v[1], v[2]};
                d[3] = v[3];
            } else if constexpr (V == 2) {
                d[0] = v[0];
                d[1] = v[1];
            } else {
                d[0] = v[0];
            }
        }
    };
    auto store = [&](const Task& t, int st) {
        unsigned dm, xm;
        masks(t, st, dm, xm);
        const int db = 2 * st * W + t.c0;
#pragma unroll
        for (int m = 0; m < NITD; ++m) {
            if (!((dex >> m) & 1)) continue;
            const bool ok = (dm >> m) & 1;
            const vecf<V> v = dzv[m];
            float* d = dyl + dlb + (m / NIRD) * 32 * DCS + TPD * V * (m % NIRD);
            if constexpr (V == 1) {
                d[0] = v[0];
            } else {
                *reinterpret_cast<f2*>(d) = f2{v[0], v[1]};
                if constexpr (V == 4) *reinterpret_cast<f2*>(d + 2) = f2{v[2], v[3]};
            }
            if (write_dy) bstore<V>(t.rdo, ok ? 4 * (dgo(m) + db) : OOB, v);
        }
        store_x(t, st, xv);
    };
    // x rows -1, 0 of a task (stage -1): row -1 is outside (zeros; the ring slot holds the previous task's rows)
    auto load_xa = [&](const Task& t, vecf<V> (&xa)[NIT]) {
        unsigned dm, xm;
        masks(t, -1, dm, xm);
        const int xb = -W + t.c0;
#pragma unroll
        for (int m = 0; m < NIT; ++m) xa[m] = bload<V>(t.rx, (xm >> m) & 1 ? 4 * (xgo(m) + xb) : OOB);
    };

    // wave constants of row Q: e = w + sx u from x rows (w, u) of the tile row's four; the dy row
    // combination pr = r0 + sy r1 (Q 0: r0, 1: r0 + r1, 2: r0 - r1, 3: r1 via r0 := row 1, sy = 0)
    const int IW = Q == 0 ? 0 : Q == 2 ? 2 : 1, IU = Q == 0 ? 2 : Q == 2 ? 1 : Q == 1 ? 2 : 3;
    const float sx = Q == 1 ? 1.f : -1.f;
    const float sy = Q == 1 ? 1.f : Q == 2 ? -1.f : 0.f;
    const PkK pk = pk_consts();
    const float* const dr0 = dyl + (Q == 3 ? 32 * DCS : 0) + c32 * DCS + 2 * g;
    const float* const dr1 = dyl + 32 * DCS + c32 * DCS + 2 * g;
    auto ksteps = [&](const float* xw, const float* xu, int s0, int s1) {
        const int n = s1 - s0;
        const float* w = xw + 4 * s0;
        const float* u = xu + 4 * s0;
        const float* q0 = dr0 + 4 * s0;
        const float* q1 = dr1 + 4 * s0;
        kloop(w, u, q0, q1, pk, f2{sx, sx}, f2{sy, sy}, acc, n);
    };
    const int Ks = a.Ksteps;
    // Round 6 (PF: the V = 2 / 1 narrow images, 5-row tasks at cnn_small layers 5 / 6): the NEXT task's
    // stages -1 / 0 are loaded during this task's last tile row, in parts under its K-steps like any next
    // row, so its prologue round trip no longer stalls the block between tasks.  (V = 4: the extra staging
    // registers spilled; its tasks are 10+ rows long.)
    constexpr bool PF = V != 4;
    vecf<V> xa[NIT];
    // one tile row: KIND 0 = a row with a successor (loads row tr + 1 of t), 1 = the task's last row loading
    // the next task's prologue (t = that task), 2 = the last row with nothing to load
    auto row = [&](const Task& t, int tr, auto kind) {
        constexpr int KIND = decltype(kind)::value;
        // x rows 2 tr - 1 + i of this tile row live in ring slot (2 tr + i) & 3
        const float* xw = xl + ((2 * tr + IW) & 3) * CX * XCS + (32 * hx + c32) * XCS + 2 * g;
        const float* xu = xl + ((2 * tr + IU) & 3) * CX * XCS + (32 * hx + c32) * XCS + 2 * g;
        // the next tile row's dz / y / x rows loaded over this row's K-steps in NPT parts (a burst of 3
        // NIT loads at the row start stalls the issuing waves on the texture unit, MFMA pipes idle); dy
        // formed after the last part
#pragma unroll
        for (int pt = 0; pt < NPT; ++pt) {
            __builtin_amdgcn_sched_barrier(0);  // (no hoisting of later parts' loads: registers)
            if constexpr (KIND == 0) {
                load_dy(t, tr + 1, pt);
                load_x(t, tr + 1, pt, xv);
            } else if constexpr (KIND == 1) {
                load_dy(t, 0, pt);
                load_x(t, 0, pt, xv);
                if (pt == 0) load_xa(t, xa);
            }
            __builtin_amdgcn_sched_barrier(0);
            ksteps(xw, xu, Ks * pt / NPT, Ks * (pt + 1) / NPT);
        }
        if constexpr (KIND != 2) form_dy(t, KIND == 0 ? tr + 1 : 0);
        __syncthreads();  // the dy rows and the two oldest x rows are free (last row: every ring slot)
        if constexpr (KIND == 0) {
            store(t, tr + 1);
            __syncthreads();
        } else if constexpr (KIND == 1) {
            store_x(t, -1, xa);
            store(t, 0);
        }
    };
    auto prologue = [&](const Task& t) {  // stages -1 and 0 (x rows -1 .. 2, dy rows 0, 1): one round trip
        load_dy(t, 0, -1);
        load_x(t, 0, -1, xv);
        load_xa(t, xa);
        store_x(t, -1, xa);
        form_dy(t, 0);
        store(t, 0);
    };
    bool staged = false;  // (PF) the current task's prologue was stored by the previous task's last row
    for (int task = t0s; task < t1s; ++task) {
        const Task cur = task_of(task);
        if (!staged) prologue(cur);
        __syncthreads();
        for (int tr = 0; tr + 1 < TR; ++tr) row(cur, tr, std::integral_constant<int, 0>{});
        staged = PF && task + 1 < t1s;
        if (staged) row(task_of(task + 1), TR - 1, std::integral_constant<int, 1>{});
        else row(cur, TR - 1, std::integral_constant<int, 2>{});
    }
    // partials: C register r of lane l = (cout row (r & 3) + 8 (r >> 2) + 4 g, cin c32); xi = 4 Q + e
    float* out = a.part + (int64_t)slice * a.cout * a.cin * 16;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int co = co0 + (r & 3) + 8 * (r >> 2) + 4 * g;
        *reinterpret_cast<float4*>(out + ((int64_t)co * a.cin + ci0 + 32 * hx + c32) * 16 + 4 * Q) =
            make_float4(acc[0][r], acc[1][r], acc[2][r], acc[3][r]);
    }
}

template <int PRO, int V, bool PD, int NH>
__global__ __launch_bounds__(256 * NH) __attribute__((amdgpu_waves_per_eu(2))) void wgrad_wino_kernel(WinoWgradArgs a) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int tid = threadIdx.x;
    const int ncgi = a.cin / (32 * NH), ngroups = (a.cout / 32) * ncgi;
    const int f = blockIdx.x, kk = f >> 3;
    const int group = kk % ngroups;
    const int slice = (kk / ngroups) * 8 + (f & 7);  // XCD-aware: a slice's groups share an XCD
    if (slice >= a.nslice) return;
    const int co0 = (group / ncgi) * 32, ci0 = (group % ncgi) * 32 * NH;
    // zero the staging image (padding positions and padded tiles read zeros)
    const int nz = 4 + 4 * 32 * NH * a.XCS + 2 * 32 * a.DCS;
    for (int i = tid; i < nz; i += 256 * NH) smem[i] = 0.f;
    __syncthreads();
    ww_body<PRO, V, PD, NH>(a, smem, co0, ci0, slice);
}

// dW[n][c] = G^T dU G per (n, c) from the slices' sum (float64, fixed order); the partials carry
// row / column 3 of the Winograd domain negated (Yh' of the kernel).  Block = 16 (n, c) pairs x 16
// slice groups: thread (group g, pair j) sums slices g, g + 16, ... of its pair (the 16 pairs of a
// slice are 1 KB contiguous), the groups are added in order through LDS, then 16 threads transform.
constexpr int RP = 16, RG = 16;
__global__ __launch_bounds__(256) void wgrad_wino_reduce_kernel(const float* __restrict__ part, int nslice, int npair,
                                                                float* __restrict__ dw) {
    __shared__ double red[RG][RP][17];
    const int j = threadIdx.x & (RP - 1), g = threadIdx.x / RP;
    const int i = blockIdx.x * RP + j;
    double u[16];
#pragma unroll
    for (int x = 0; x < 16; ++x) u[x] = 0.0;
    if (i < npair) {
        for (int s = g; s < nslice; s += RG) {
            const float4* p = reinterpret_cast<const float4*>(part + ((int64_t)s * npair + i) * 16);
            float4 v[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) v[q] = p[q];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                u[4 * q + 0] += v[q].x;
                u[4 * q + 1] += v[q].y;
                u[4 * q + 2] += v[q].z;
                u[4 * q + 3] += v[q].w;
            }
        }
    }
#pragma unroll
    for (int x = 0; x < 16; ++x) red[g][j][x] = u[x];
    __syncthreads();
    if (g != 0 || i >= npair) return;
#pragma unroll
    for (int x = 0; x < 16; ++x) {
        double t = red[0][j][x];
        for (int q = 1; q < RG; ++q) t += red[q][j][x];
        u[x] = t;
    }
    // undo the folded signs: dU[q][e] = s_q s_e dU'[q][e], s_3 = -1
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        u[4 * q + 3] = -u[4 * q + 3];
        u[12 + q] = -u[12 + q];
    }
    // t = G^T dU (3 x 4), G = [[1,0,0],[1/2,1/2,1/2],[1/2,-1/2,1/2],[0,0,1]]
    double t[3][4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        const double u0 = u[e], u1 = u[4 + e], u2 = u[8 + e], u3 = u[12 + e];
        t[0][e] = u0 + 0.5 * (u1 + u2);
        t[1][e] = 0.5 * (u1 - u2);
        t[2][e] = 0.5 * (u1 + u2) + u3;
    }
    float* o = dw + (int64_t)i * 9;
#pragma unroll
    for (int r = 0; r < 3; ++r) {
        const double t0 = t[r][0], t1 = t[r][1], t2 = t[r][2], t3 = t[r][3];
        o[3 * r + 0] = (float)(t0 + 0.5 * (t1 + t2));
        o[3 * r + 1] = (float)(0.5 * (t1 - t2));
        o[3 * r + 2] = (float)(0.5 * (t1 + t2) + t3);
    }
}

int smallest_2odd(int n) {  // smallest m >= n with m = 2 * odd
    while ((n & 3) != 2) ++n;
    return n;
}

}  // namespace

bool wgrad_wino_geometry(int B, int H, int W, int cin, int cout, WinoWgradArgs* a) {
    if (cin % 32 || cout % 32 || H < 1 || W < 4) return false;
    // staging vector: 16 / 8 bytes where the width allows, single floats at odd widths (round 5: the narrow
    // 5 x 25 / 3 x 13 blocks of cnn_deep; the last tile column is half outside and stages zeros)
    const int V = W % 4 == 0 ? 4 : W % 2 == 0 ? 2 : 1;
    const int TC = (W + 1) / 2;
    // odd widths only where the 2 x 2 tiles cover the image well: 5 x 25 (0.80 of the tiles' outputs real)
    // 5.77 vs 6.05 ms on the row-window kernel; 3 x 13 (0.70) 10.8 vs 8.7 ms (profiles/r5_wgrad_wino_odd.txt)
    if (V == 1 && !PCX_AB_WW_ODD_ALL && (double)H * W < 0.75 * 4.0 * ((H + 1) / 2) * TC) return false;
    int nseg = ceil_div(TC, 50);
    int S = ceil_div(TC, nseg);
    if (nseg > 1) S = (S + 1) & ~1;  // strip starts 2 t0 on a 16-byte boundary (V = 4)
    nseg = ceil_div(TC, S);
    const int Ksteps = (S + 1) / 2;
    const int nd = 2 * S / V, kmax = (2 * S + 1 + V - 1) / V, nx = kmax + 1;
    if ((2 * S) % V) return false;
    if (2 * nd > 8 * NIT || 2 * nx > 8 * NIT) return false;  // 8 threads x NIT items per channel
    const int XCS = smallest_2odd(std::max(std::max(V * kmax + 1, 4 * Ksteps + 2), 2 * S + 5));
    const int DCS = smallest_2odd(4 * Ksteps);
    // NH = 2 (64 input channels per block of 8 waves, one block per CU) where the input channels and LDS allow
    const int NH = (cin % 64 == 0 && !PCX_AB_WW_NH1 &&
                    ((size_t)4 + 256 * XCS + 64 * DCS) * 4 <= 160 * 1024) ? 2 : 1;
    const size_t lds = ((size_t)4 + 128 * NH * XCS + 64 * DCS) * 4;
    if (lds > 80 * 1024 * NH) return false;
    if ((int64_t)64 * H * W * 4 >= OOB) return false;  // valid offsets (NH = 2: 64 x planes) stay below the marker
    if (a) {
        a->S = S;
        a->nseg = nseg;
        a->V = V;
        a->XCS = XCS;
        a->DCS = DCS;
        a->nd = nd;
        a->nx = nx;
        a->Ksteps = Ksteps;
        a->lds = lds;
        a->NH = NH;
        a->ntask = B * nseg;
        const int ngroups = (cout / 32) * (cin / (32 * NH));
        int want = std::max(8, (2 / NH) * num_cus() / ngroups);  // ~2 (NH = 2: 1) resident blocks per CU
        want = std::min(want, a->ntask);
        a->per_slice = ceil_div(a->ntask, want);
        a->nslice = ceil_div(a->ntask, a->per_slice);
    }
    return true;
}

int launch_wgrad_wino(int pro, WinoWgradArgs a, hipStream_t s) {
    WinoWgradArgs g{};
    PCX_CHECK_ARG(wgrad_wino_geometry(a.B, a.H, a.W, a.cin, a.cout, &g), "wgrad_wino: unsupported shape %dx%d (%d, %d)",
                  a.H, a.W, a.cin, a.cout);
    PCX_CHECK_ARG(g.S == a.S && g.V == a.V && g.XCS == a.XCS && g.DCS == a.DCS && g.nslice == a.nslice &&
                      g.per_slice == a.per_slice && g.ntask == a.ntask && g.NH == a.NH,
                  "wgrad_wino: geometry mismatch");
    PCX_CHECK_ARG(pro == PRO_RAW || pro == PRO_BNRELU, "wgrad_wino: prologue %d", pro);
    const int ngroups = (a.cout / 32) * (a.cin / (32 * a.NH));
    dim3 grid((unsigned)(((a.nslice + 7) / 8) * 8 * ngroups));
    PCX_CHECK_ARG((a.dz != nullptr) != (a.dzpool != nullptr), "wgrad_wino: exactly one of dz / dzpool");
    const bool pd = a.dzpool != nullptr;
    // pooled dz: 4-column items over whole windows, 2-byte aligned selection pairs (even strip starts)
    PCX_CHECK_ARG(!pd || (a.parg && pro == PRO_BNRELU && a.V == 4 && !(a.H & 1) && (a.nseg == 1 || !(a.S & 1))),
                  "wgrad_wino: pooled dz needs parg, PRO_BNRELU, V = 4, even H and even strip starts");
#define PCX_WW1(P_, V_, PD_, NH_)                                                                        \
    if (pro == P_ && a.V == V_ && pd == PD_ && a.NH == NH_) {                                            \
        (void)hipFuncSetAttribute((const void*)wgrad_wino_kernel<P_, V_, PD_, NH_>,                      \
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)a.lds);               \
        wgrad_wino_kernel<P_, V_, PD_, NH_><<<grid, 256 * NH_, a.lds, s>>>(a);                           \
        PCX_LAUNCH_CHECK("wgrad_wino_kernel");                                                           \
        return PCX_OK;                                                                                   \
    }
#define PCX_WW(P_, V_, PD_) PCX_WW1(P_, V_, PD_, 1) PCX_WW1(P_, V_, PD_, 2)
    PCX_WW(PRO_RAW, 4, false)
    PCX_WW(PRO_RAW, 2, false)
    PCX_WW(PRO_BNRELU, 4, false)
    PCX_WW(PRO_BNRELU, 2, false)
    PCX_WW(PRO_BNRELU, 4, true)  // cnn_small layer 4 (behind layer 5's pool)
    PCX_WW(PRO_RAW, 1, false)
    PCX_WW(PRO_BNRELU, 1, false)
#undef PCX_WW
#undef PCX_WW1
    set_error("wgrad_wino: unsupported combination (pro %d, vec %d)", pro, a.V);
    return PCX_EINVAL;
}

int launch_wgrad_wino_reduce(const float* part, int nslice, int cout, int cin, float* dw, hipStream_t s) {
    const int npair = cout * cin;
    wgrad_wino_reduce_kernel<<<ceil_div(npair, RP), RP * RG, 0, s>>>(part, nslice, npair, dw);
    PCX_LAUNCH_CHECK("wgrad_wino_reduce_kernel");
    return PCX_OK;
}

}  // namespace pcx
