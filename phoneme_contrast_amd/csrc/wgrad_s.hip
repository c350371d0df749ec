// Weight gradient of the stride-1 3x3 convs on v_mfma_f32_16x16x4_f32, four pixel streams per row.
//
//   dW[n][c][tap] = sum_{b,h,w} dy[b,n,h,w] * x[b,c,h+dh,w+dw]      (reference: autograd of the
//   3x3 convs of phoneme_cnn.py:35-65 and of the stride-1 convs of ResidualBlock :159-184)
//   dy = A1 dz + A2 y + A3   (BN backward with the per-channel coefficients of the finaliser;
//                             identity coefficients when dy is given)
//   x  = relu(y_prev * s + t) (PRO_BNRELU) or a materialised input (PRO_RAW)
//
// Shape, from MI355X measurements (dbg/mfma_valu.hip): an f32 MFMA holds the SIMD's vector issue
// for its whole duration, so every VALU / LDS instruction of any wave on the SIMD adds to the MFMA
// time; and one wave per SIMD leaves barrier and load waits exposed.  Hence:
//
//  * GEMM view M = cout (dy), N = cin (x), K = pixels, on 16 x 16 x 4 tiles: lane l holds channel
//    l & 15 and pixel STREAM g = l >> 4.  A block row strip of width 4R is cut into four streams
//    of R pixels (R even); each MFMA takes one pixel of each stream.
//  * A lane walks its stream two pixels at a time: one ds_read_b64 of dy and one of x per row
//    offset dh feed 18 MFMAs (9 taps x 2 pixels) per 16-row cout tile; the dw = -1 / +1 taps are
//    register renames (previous pair's .y, next pair's .x).  x rows live in LDS as contiguous
//    image rows with a 4-column halo, so stream g starts at column g R and its halo columns are
//    its neighbours' pixels.
//  * Small tiles (36 or 72 accumulator registers per wave) and row strips that keep the LDS
//    image at or below 80 KB give two blocks (8 waves) per CU: one block's barriers, staging and
//    load latency run under the other's MFMAs.
//  * Staging is lean: every thread owns fixed (channel, vector) items of the dy and x rows;
//    global reads are buffer loads whose per-row offset is the scalar soffset (no per-row VALU
//    address math), and items outside the strip / image carry an out-of-range offset, so the
//    hardware returns 0 and a per-item constant (A3 -> 0, t -> 0) keeps dy / x at exactly 0
//    there.  BN backward (2 fma) and the BN+ReLU prologue (fma+max) are applied between load and
//    LDS store; the first cin group stores dy to HBM for the data-gradient conv that follows.
//  * A block walks (sample, strip) tasks top to bottom: dy row in one LDS slot, x rows in a
//    3-slot ring, the next rows loaded into registers under the current row's MFMAs, two
//    barriers per row.  The rows above / below the image are one shared zero row (one loop body
//    for every row: the 2 / (3 H) of MFMAs they cost beat the branches and code copies of skipping).
// Per-slice partials are summed in a fixed order by launch_sum_slices: deterministic.
#include "kernels.h"

namespace pcx {
namespace {

template <int V>
using vecf = float __attribute__((ext_vector_type(V)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

constexpr int BUF_FLAGS = 0x00020000;  // buffer resource word 3 (gfx9 raw buffer, 32-bit data)
constexpr int OOB = 0x7fff0000;        // item offset beyond every num_records: loads 0, stores dropped

// staged vectors per thread and row (the register budget beside the accumulators); every thread
// always stages exactly this many, the LDS rows are sized to match (dy rows hold s_nd (256 / NB)
// vectors, x rows s_nx 8; strips are cut to fit)
__host__ __device__ constexpr int s_nd(int v) { return v == 4 ? 4 : 8; }
__host__ __device__ constexpr int s_nx(int v) { return v == 1 ? 8 : 4; }

__device__ __forceinline__ f32x4 mfma16(float a, float b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

template <int V>
__device__ __forceinline__ vecf<V> bload(__amdgpu_buffer_rsrc_t r, int voff, int soff) {
    if constexpr (V == 4)
        return __builtin_bit_cast(vecf<4>, __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0));
    else if constexpr (V == 2)
        return __builtin_bit_cast(vecf<2>, __builtin_amdgcn_raw_buffer_load_b64(r, voff, soff, 0));
    else
        return __builtin_bit_cast(vecf<1>, __builtin_amdgcn_raw_buffer_load_b32(r, voff, soff, 0));
}

template <int V>
__device__ __forceinline__ void bstore(__amdgpu_buffer_rsrc_t r, int voff, int soff, vecf<V> v) {
    if constexpr (V == 4)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), r, voff, soff, 0);
    else if constexpr (V == 2)
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, v), r, voff, soff, 0);
    else
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), r, voff, soff, 0);
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const float* base, int64_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), (short)0, (int)bytes, BUF_FLAGS);
}

__device__ __forceinline__ f32x2 ld2(const float* p) { return *reinterpret_cast<const f32x2*>(p); }

// single v_fma_f32: keeps the compiler from SLP-packing the dy arithmetic into v_pk_fma_f32, whose
// write of a register still being read by the preceding buffer_store_dwordx4 of dy was not given
// its wait state (gfx950, hipcc 7.2: every second float of the stored dy corrupted)
__device__ __forceinline__ float fma1(float a, float b, float c) {
    float r;
    asm("v_fma_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

// One pixel pair of a lane's stream: 2 pixels x 9 taps x TMW cout tiles.  pv[dh] = x of the pixel
// before the pair, c[dh] = the pair, n[dh].x = the pixel after it.
template <int TMW>
__device__ __forceinline__ void pair_mfma(f32x4 (&acc)[TMW][9], const f32x2 (&a)[TMW], const float (&pv)[3],
                                          const f32x2 (&c)[3], const f32x2 (&n)[3]) {
#pragma unroll
    for (int e = 0; e < 2; ++e) {
#pragma unroll
        for (int dh = 0; dh < 3; ++dh) {
            const float vm = e == 0 ? pv[dh] : c[dh].x;
            const float v0 = e == 0 ? c[dh].x : c[dh].y;
            const float vp = e == 0 ? c[dh].y : n[dh].x;
#pragma unroll
            for (int tm = 0; tm < TMW; ++tm) {
                const float av = e == 0 ? a[tm].x : a[tm].y;
                acc[tm][3 * dh + 0] = mfma16(av, vm, acc[tm][3 * dh + 0]);
                acc[tm][3 * dh + 1] = mfma16(av, v0, acc[tm][3 * dh + 1]);
                acc[tm][3 * dh + 2] = mfma16(av, vp, acc[tm][3 * dh + 2]);
            }
        }
    }
}

// MFMAs of one image row: np pixel pairs of the lane's stream.  A[tm]: dy stream start, X[dh]: x
// stream start in the slot of row r - 1 + dh.  Pair j + 2 is read while pair j is multiplied (the
// dw = +1 tap of pair j already needs pair j + 1), through three register buffers rotated by a
// 3-fold unrolled loop: no register moves beyond the carried pixel pv.  Reads run at most two
// pairs past the stream (next stream, halo or padding of the LDS row; never multiplied).
template <int TMW>
__device__ __forceinline__ void row_s(f32x4 (&acc)[TMW][9], const float* const (&A)[TMW], const float* X0,
                                      const float* X1, const float* X2, int np) {
    const float* X[3] = {X0, X1, X2};
    f32x2 a0[TMW], a1[TMW], a2[TMW], b0[3], b1[3], b2[3];
    float pv[3];
#pragma unroll
    for (int dh = 0; dh < 3; ++dh) {
        pv[dh] = X[dh][-1];
        b0[dh] = ld2(X[dh]);
        b1[dh] = ld2(X[dh] + 2);
    }
#pragma unroll
    for (int tm = 0; tm < TMW; ++tm) {
        a0[tm] = ld2(A[tm]);
        a1[tm] = ld2(A[tm] + 2);
    }
    auto load = [&](f32x2 (&b)[3], f32x2 (&av)[TMW], int pair) {
#pragma unroll
        for (int dh = 0; dh < 3; ++dh) b[dh] = ld2(X[dh] + 2 * pair);
#pragma unroll
        for (int tm = 0; tm < TMW; ++tm) av[tm] = ld2(A[tm] + 2 * pair);
    };
    auto carry = [&](const f32x2 (&b)[3]) {
#pragma unroll
        for (int dh = 0; dh < 3; ++dh) pv[dh] = b[dh].y;
    };
    int j = 0;
    for (; j + 3 <= np; j += 3) {
        load(b2, a2, j + 2);
        __builtin_amdgcn_sched_barrier(0);
        pair_mfma<TMW>(acc, a0, pv, b0, b1);
        __builtin_amdgcn_sched_barrier(0);
        carry(b0);
        load(b0, a0, j + 3);
        __builtin_amdgcn_sched_barrier(0);
        pair_mfma<TMW>(acc, a1, pv, b1, b2);
        __builtin_amdgcn_sched_barrier(0);
        carry(b1);
        load(b1, a1, j + 4);
        __builtin_amdgcn_sched_barrier(0);
        pair_mfma<TMW>(acc, a2, pv, b2, b0);
        __builtin_amdgcn_sched_barrier(0);
        carry(b2);
    }
    if (j < np) {
        if (j + 1 < np) load(b2, a2, j + 2);
        __builtin_amdgcn_sched_barrier(0);
        pair_mfma<TMW>(acc, a0, pv, b0, b1);
        if (j + 1 < np) {
            __builtin_amdgcn_sched_barrier(0);
            carry(b0);
            pair_mfma<TMW>(acc, a1, pv, b1, b2);
        }
    }
}

template <int PRO, int V, int TMW>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void wgrad_s_kernel(WgradArgs a) {
    constexpr int NB = 32 * TMW, CB = 32;
    constexpr int ND = s_nd(V), NX = s_nx(V);
    constexpr int TPD = 256 / NB, TPX = 256 / CB;  // threads per staged channel row
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int DCS = a.DCS, XCS = a.XCS;
    float* dyl = smem;            // [NB][DCS]
    float* xl = smem + NB * DCS;  // [3][CB][XCS]: image row rho in slot (rho + 1) % 3
    float* zl = xl + 3 * CB * XCS;  // [XCS] zeros: the rows above / below the image, every channel
    for (int i = threadIdx.x; i < XCS; i += 256) zl[i] = 0.f;

    const int tid = threadIdx.x, lane = tid & 63, cl = lane & 15, g = lane >> 4;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave >> 1, wn = wave & 1;
    const int ncb = a.cin / CB;
    const int ngroups = (a.cout / NB) * ncb;
    // XCD-aware (slice, group) mapping: blocks f and f + 8 share an XCD and get the groups of one
    // slice (the same dz / y / x rows)
    const int f = blockIdx.x;
    const int kk = f >> 3;
    const int group = kk % ngroups;
    const int slice = (kk / ngroups) * 8 + (f & 7);
    if (slice >= a.ntslice) return;
    const int n0 = (group / ncb) * NB, c0 = (group % ncb) * CB;
    const int H = a.H, W = a.W, HW = H * W;

    // staging items: thread -> one dy channel (vectors dj0 + TPD k) and one x channel
    const int dch = tid / TPD, dj0 = tid % TPD;
    const int xch = tid / TPX, xj0 = tid % TPX;
    const float4 kd = a.cf_dy[n0 + dch];  // {a, mb, mgi, mean}
    const float A1 = kd.x, A2 = -kd.x * kd.z, A3 = kd.x * (kd.w * kd.z - kd.y);
    float xs = 1.f, xt = 0.f;
    if (PRO == PRO_BNRELU) {
        const float4 k = a.cf_x[c0 + xch];
        xs = k.x;
        xt = k.y;
    }
    float* const dst_d = dyl + dch * DCS + dj0 * V;
    float* const dst_x = xl + xch * XCS + xj0 * V;

    f32x4 acc[TMW][9];
#pragma unroll
    for (int tm = 0; tm < TMW; ++tm)
#pragma unroll
        for (int t = 0; t < 9; ++t) acc[tm][t] = f32x4{0.f, 0.f, 0.f, 0.f};

    const bool write_dy = a.dy_out != nullptr && c0 == 0;
    const int t0 = slice * a.per_slice, t1 = min(a.nchunks, t0 + a.per_slice);
    vecf<V> dzv[ND], yv[ND], xv[NX];
    int dvo[ND], xvo[NX];
    float a3v[ND], xtv[NX];

    for (int task = t0; task < t1; ++task) {
        const int b = task / a.nseg;
        const int w0 = (task - b * a.nseg) * a.CW;
        const int cw = min(a.CW, W - w0);
        const int R = ((cw + 7) >> 3) << 1;  // stream length: 4 R >= cw, R even
        const size_t dbase = ((size_t)b * a.cout + n0) * HW + w0;
        const __amdgpu_buffer_rsrc_t rdz = rsrc(a.dz + dbase, (int64_t)NB * HW * 4);
        const __amdgpu_buffer_rsrc_t ry = rsrc(a.y + dbase, (int64_t)NB * HW * 4);
        const __amdgpu_buffer_rsrc_t rdo = rsrc(write_dy ? a.dy_out + dbase : a.dz, write_dy ? (int64_t)NB * HW * 4 : 0);
        const __amdgpu_buffer_rsrc_t rx =
            rsrc(a.src + ((size_t)b * a.cin + c0) * HW + w0 - 4, ((int64_t)CB * HW + 8) * 4);
#pragma unroll
        for (int k = 0; k < ND; ++k) {
            const int col = (dj0 + TPD * k) * V;
            const bool ok = col < cw;
            dvo[k] = ok ? (dch * HW + col) * 4 : OOB;
            a3v[k] = ok ? A3 : 0.f;
        }
#pragma unroll
        for (int k = 0; k < NX; ++k) {
            const int p = (xj0 + TPX * k) * V;  // LDS position p <-> column w0 - 4 + p
            const bool ok = w0 - 4 + p >= 0 && w0 - 4 + p < W;
            xvo[k] = ok ? (xch * HW + p) * 4 : OOB;
            xtv[k] = ok ? xt : 0.f;
        }

        auto load_dy = [&](int r) {
#pragma unroll
            for (int k = 0; k < ND; ++k) {
                dzv[k] = bload<V>(rdz, dvo[k], r * W * 4);
                yv[k] = bload<V>(ry, dvo[k], r * W * 4);
            }
        };
        auto store_dy = [&](int r) {
#pragma unroll
            for (int k = 0; k < ND; ++k) {
                vecf<V> v;
#pragma unroll
                for (int e = 0; e < V; ++e) v[e] = fma1(A1, dzv[k][e], fma1(A2, yv[k][e], a3v[k]));
                *reinterpret_cast<vecf<V>*>(dst_d + TPD * V * k) = v;
                if (write_dy) bstore<V>(rdo, dvo[k], r * W * 4, v);
            }
        };
        auto load_x = [&](int r) {
#pragma unroll
            for (int k = 0; k < NX; ++k) xv[k] = bload<V>(rx, xvo[k], r * W * 4);
        };
        auto store_x = [&](int slot) {
            float* d = dst_x + slot * CB * XCS;
#pragma unroll
            for (int k = 0; k < NX; ++k) {
                vecf<V> v = xv[k];
                if (PRO == PRO_BNRELU) {
#pragma unroll
                    for (int e = 0; e < V; ++e) v[e] = fmaxf(fmaf(v[e], xs, xtv[k]), 0.f);
                }
                *reinterpret_cast<vecf<V>*>(d + TPX * V * k) = v;
            }
        };

        const float* A[TMW];
#pragma unroll
        for (int tm = 0; tm < TMW; ++tm) A[tm] = dyl + (wm * 16 * TMW + tm * 16 + cl) * DCS + g * R;
        const float* xlane = xl + (wn * 16 + cl) * XCS + 4 + g * R;
        const float* zlane = zl + 4 + g * R;
        const int np = R >> 1;

        // task prologue: dy row 0; x rows 0, 1 -> slots 1, 2
        load_dy(0);
        load_x(0);
        store_dy(0);
        store_x(1);
        if (H > 1) {
            load_x(1);
            store_x(2);
        }
        __syncthreads();
        for (int r = 0; r < H; ++r) {
            const bool pre = r + 1 < H, prex = r + 2 < H;
            if (pre) load_dy(r + 1);
            if (prex) load_x(r + 2);
            const int s0 = r % 3;
            const int s1 = s0 == 2 ? 0 : s0 + 1;
            const int s2 = s1 == 2 ? 0 : s1 + 1;
            // rows -1 / H: the shared zero row (their MFMAs run on zeros; one loop body for all rows)
            const float* X0 = r > 0 ? xlane + s0 * CB * XCS : zlane;
            const float* X1 = xlane + s1 * CB * XCS;
            const float* X2 = pre ? xlane + s2 * CB * XCS : zlane;
            row_s<TMW>(acc, A, X0, X1, X2, np);
            __syncthreads();  // the dy slot and the x slot of row r - 1 are free
            if (pre) store_dy(r + 1);
            if (prex) store_x(s0);
            __syncthreads();
        }
    }
    float* out = a.part + (int64_t)slice * a.cout * a.cin * 9;
    const int c = c0 + wn * 16 + cl;
#pragma unroll
    for (int tm = 0; tm < TMW; ++tm)
#pragma unroll
        for (int t = 0; t < 9; ++t)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int n = n0 + wm * 16 * TMW + tm * 16 + 4 * g + i;
                out[((int64_t)n * a.cin + c) * 9 + t] = acc[tm][t][i];
            }
}

int odd4(int n) {  // smallest m >= n with m = 4 * odd
    n = (n + 3) & ~3;
    while ((n & 7) == 0) n += 4;
    return n;
}

struct SLayout {
    int R, DCS, XCS;
    size_t lds;
};

// LDS image for strips of width <= CW (or the whole row), load width v, NB dy channels.  Every
// thread stages s_nd(v) dy and s_nx(v) x vectors per row, so a dy row holds s_nd(v) (256 / NB)
// vectors and an x row s_nx(v) 8; the stream reads need 4 R + 4 (dy) and 4 R + 8 (x) floats.
bool s_layout(int W, int CW, int v, int NB, SLayout* L) {
    const int cw = std::min(CW, W);
    L->R = ((cw + 7) / 8) * 2;
    const int ed = s_nd(v) * (256 / NB) * v, ex = s_nx(v) * 8 * v;
    L->DCS = odd4(ed);
    L->XCS = odd4(ex);
    L->lds = ((size_t)NB * L->DCS + (size_t)(3 * 32 + 1) * L->XCS) * 4;
    return 4 * L->R + 4 <= ed && 4 * L->R + 8 <= ex && L->lds <= 160 * 1024;
}

}  // namespace

bool wgrad_s_geometry(int B, int H, int W, int cin, int cout, WgradArgs* a, int force_cw) {
    if (cin % 32 || cout % 32 || W < 1 || H < 1) return false;
    const int TMW = cout % 64 == 0 ? 2 : 1, NB = 32 * TMW;
    const int v = W % 4 == 0 ? 4 : W % 2 == 0 ? 2 : 1;
    double best = 1e300;
    int bcw = 0;
    for (int cw = 8; cw < W + 8; cw += 8) {
        if (force_cw && cw != force_cw) continue;
        SLayout L;
        if (!s_layout(W, cw, v, NB, &L)) continue;
        const int nseg = (W + cw - 1) / cw;
        const int bpc = std::min<int>(2, (int)(160 * 1024 / L.lds));  // blocks per CU (LDS; registers: 2)
        // modelled SIMD cycles per sample and row: MFMAs (32 per 16x16x4, 9 taps x R / 2 pairs x 2)
        // + staging (a few VALU per staged float) + a fixed per-row cost; one block per CU exposes
        // barriers and load latency
        double cyc = 0;
        for (int s = 0; s < nseg; ++s) {
            const int c = std::min(cw, W - s * cw), R = ((c + 7) / 8) * 2;
            const double mf = 288.0 * TMW * R;
            const double st = 4.0 * (s_nd(v) * (2.0 * v + 4) + s_nx(v) * (2.0 * v + 3)) + 600.0;
            cyc += mf + st;
        }
        if (bpc < 2) cyc *= 1.35;
        if (cyc < best) {
            best = cyc;
            bcw = cw;
        }
    }
    if (!bcw) return false;
    SLayout L;
    s_layout(W, bcw, v, NB, &L);
    a->MT = 16;  // marks the stream kernel
    a->NPM = TMW;
    a->NPC = 1;
    a->KW = 1;
    a->CW = bcw;
    a->R0 = L.R;
    a->DCS = L.DCS;
    a->XCS = L.XCS;
    a->nvd = s_nd(v) * (256 / NB);
    a->nvx = s_nx(v) * 8;
    a->VX = v;
    a->nseg = ceil_div(W, bcw);
    a->nchunks = B * a->nseg;
    const int ngroups = (cout / NB) * (cin / 32);
    int want = std::max(8, 2 * num_cus() / ngroups);  // ~2 resident blocks per CU
    want = std::min(want, a->nchunks);
    a->per_slice = ceil_div(a->nchunks, want);
    a->ntslice = ceil_div(a->nchunks, a->per_slice);
    a->nslice = a->ntslice;
    return true;
}

int launch_wgrad_s(int pro, WgradArgs a, hipStream_t s) {
    const int TMW = a.NPM, NB = 32 * TMW, v = a.VX;
    PCX_CHECK_ARG(a.MT == 16 && (TMW == 1 || TMW == 2), "wgrad_s: bad tile split %d", TMW);
    PCX_CHECK_ARG(a.cout % NB == 0 && a.cin % 32 == 0, "wgrad_s: channels (%d,%d) vs block %dx32", a.cout, a.cin, NB);
    PCX_CHECK_ARG((int64_t)a.cout * a.H * a.W < ((int64_t)1 << 29) && (int64_t)a.cin * a.H * a.W < ((int64_t)1 << 29),
                  "wgrad_s: sample block too large");
    PCX_CHECK_ARG(a.nslice == a.ntslice && a.CW % 8 == 0 && a.W % v == 0, "wgrad_s: slices / strip %d", a.CW);
    SLayout L;
    PCX_CHECK_ARG((v == 1 || v == 2 || v == 4) && s_layout(a.W, a.CW, v, NB, &L), "wgrad_s: strip %d does not fit",
                  a.CW);
    PCX_CHECK_ARG(L.R == a.R0 && L.DCS == a.DCS && L.XCS == a.XCS && a.nvd == s_nd(v) * (256 / NB) &&
                      a.nvx == s_nx(v) * 8,
                  "wgrad_s: geometry mismatch");
    const size_t smem = L.lds;
    dim3 grid((unsigned)(((a.ntslice + 7) / 8) * 8 * ((a.cout / NB) * (a.cin / 32))));
#define PCX_WS(P_, V_, T_)                                                                            \
    if (pro == P_ && v == V_ && TMW == T_) {                                                          \
        (void)hipFuncSetAttribute((const void*)wgrad_s_kernel<P_, V_, T_>,                            \
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);             \
        wgrad_s_kernel<P_, V_, T_><<<grid, 256, smem, s>>>(a);                                        \
        PCX_LAUNCH_CHECK("wgrad_s_kernel");                                                           \
        return PCX_OK;                                                                                \
    }
#define PCX_WS_V(P_) PCX_WS(P_, 4, 1) PCX_WS(P_, 4, 2) PCX_WS(P_, 2, 1) PCX_WS(P_, 2, 2) PCX_WS(P_, 1, 1) \
    PCX_WS(P_, 1, 2)
    PCX_WS_V(PRO_RAW)
    PCX_WS_V(PRO_BNRELU)
#undef PCX_WS_V
#undef PCX_WS
    set_error("wgrad_s: unsupported combination (pro %d vec %d tiles %d)", pro, v, TMW);
    return PCX_EINVAL;
}

}  // namespace pcx
