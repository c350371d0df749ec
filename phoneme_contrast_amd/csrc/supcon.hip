// Supervised-contrastive loss (SupCon) forward + closed-form backward on fp32 MFMA.
//
// Replaces SupervisedContrastiveLoss.forward (reference src/training/losses.py:41-86) and the
// autograd graph behind it.  S = F F^T is never materialised: every kernel recomputes its
// 32x32 tiles of S with v_mfma_f32_32x32x2_f32 (exact f32) from the L2-resident features.
//
// The tile is computed TRANSPOSED, C'[j][i] = S_ij with A = F_j, B = F_i, so each lane owns one
// anchor row i (its MFMA column) and 16 candidate columns j in its accumulator registers:
// the per-anchor reductions (max, sum-exp, positive sums) are in-lane plus one half swap, and
// the same registers are directly the A operand of the gradient product dF_i = sum_j H_ij F_j.
//
// Numerics follow the reference exactly: row max over ALL j (diagonal included, detached),
// den_i = sum_{j != i} exp(S_ij/T - m_i) + 1e-6, rows without positives divide by 1 and still
// count in the mean, loss scaled by T / base_T.
#include "pcx_common.h"

namespace pcx {
namespace {

constexpr int TILE = 32;
constexpr int WAVES = 4;

struct RowPart {  // online log-sum-exp partial for one anchor row
    float m, s, pos, msum;
};

__device__ __forceinline__ RowPart merge(RowPart a, RowPart b) {
    RowPart r;
    r.m = fmaxf(a.m, b.m);
    float ea = (a.m == -INFINITY) ? 0.f : expf(a.m - r.m);
    float eb = (b.m == -INFINITY) ? 0.f : expf(b.m - r.m);
    r.s = a.s * ea + b.s * eb;
    r.pos = a.pos + b.pos;
    r.msum = a.msum + b.msum;
    return r;
}

// 32x32 tile C'[j][i] = sum_k F[rj][k] F[ri][k] for this lane's rows rj (A side) and ri (B side).
// Lane half h supplies features k = 8s + 4h + t at MFMA step (s, t); both operands are streamed
// from the (L2-resident) feature matrix as float4, 4 MFMAs per load pair.
template <int D>
__device__ __forceinline__ f32x16 tile_s(const float* __restrict__ F, int64_t rj, int64_t ri,
                                         int64_t B, int h) {
    f32x16 acc = {0.f};
    const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
    const float* pa = F + rj * D + 4 * h;
    const float* pb = F + ri * D + 4 * h;
    const bool va = rj < B, vb = ri < B;
#pragma unroll 4
    for (int s = 0; s < D / 8; ++s) {
        float4 a = va ? ld4(pa + 8 * s) : z;
        float4 b = vb ? ld4(pb + 8 * s) : z;
        acc = mfma32(a.x, b.x, acc);
        acc = mfma32(a.y, b.y, acc);
        acc = mfma32(a.z, b.z, acc);
        acc = mfma32(a.w, b.w, acc);
    }
    return acc;
}

// the same tile with the anchor row's B fragments held in registers (loaded once per kernel instead of once per
// tile: D <= 128, 16 float4 per lane)
template <int D>
struct AnchorFrag {
    float4 b[D / 8];
    __device__ __forceinline__ void load(const float* __restrict__ F, int64_t ri, int64_t B, int h) {
        const float* pb = F + ri * D + 4 * h;
#pragma unroll
        for (int s = 0; s < D / 8; ++s) b[s] = ri < B ? ld4(pb + 8 * s) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
};
template <int D>
__device__ __forceinline__ f32x16 tile_s_frag(const float* __restrict__ F, int64_t rj, const AnchorFrag<D>& fi,
                                              int64_t B, int h) {
    f32x16 acc = {0.f};
    const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
    const float* pa = F + rj * D + 4 * h;
    const bool va = rj < B;
#pragma unroll
    for (int s = 0; s < D / 8; ++s) {
        const float4 a = va ? ld4(pa + 8 * s) : z;
        acc = mfma32(a.x, fi.b[s].x, acc);
        acc = mfma32(a.y, fi.b[s].y, acc);
        acc = mfma32(a.z, fi.b[s].z, acc);
        acc = mfma32(a.w, fi.b[s].w, acc);
    }
    return acc;
}
// anchor fragments in registers where they fit, in the gradient kernel (PCX_AB_SUPCON_NOFRAG: reload per tile;
// 143 -> 136 us at B = 4096, profiles/r6s2_supcon.txt)
template <int D>
constexpr bool kFrag = D <= 128 && !PCX_AB_SUPCON_NOFRAG;

__device__ __forceinline__ float pos_weight(const int64_t* __restrict__ labels,
                                            const float* __restrict__ mask, int64_t B, int64_t i,
                                            int64_t j, int64_t li) {
    if (labels) return (labels[j] == li) ? 1.f : 0.f;
    return mask[i * B + j];
}

// ---------------------------------------------------------------- forward: row partials
template <int D>
__global__ __launch_bounds__(256) void supcon_rows_partial(
    const float* __restrict__ F, const int64_t* __restrict__ labels, const float* __restrict__ mask,
    int64_t B, int64_t row0, int64_t nrows, float inv_t, int jblk_per_split, RowPart* __restrict__ part) {
    const int lane = lane_id(), wave = threadIdx.x >> 6, h = lane >> 5;
    const int64_t il = (int64_t)blockIdx.x * TILE + (lane & 31);  // anchor row within the range
    const bool ivalid = il < nrows;
    const int64_t i = row0 + il;                                    // its column index in F
    const int64_t nj = (B + TILE - 1) / TILE;
    const int64_t li = (labels && ivalid) ? labels[i] : 0;

    RowPart p = {-INFINITY, 0.f, 0.f, 0.f};
    const int64_t jb0 = (int64_t)blockIdx.y * jblk_per_split;
    const int64_t jb1 = min(nj, jb0 + jblk_per_split);
    // (anchor fragments reloaded per tile here: held in registers this kernel measured 74 -> 78 us at B = 4096)
    for (int64_t jb = jb0 + wave; jb < jb1; jb += WAVES) {
        f32x16 acc = tile_s<D>(F, jb * TILE + (lane & 31), i, B, h);
        if (ivalid) {
            float mb = -INFINITY;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                int64_t j = jb * TILE + acc_row(r, h);
                if (j < B) mb = fmaxf(mb, acc[r] * inv_t);
            }
            float mn = fmaxf(p.m, mb);
            float s = (p.m == -INFINITY) ? 0.f : p.s * expf(p.m - mn);
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                int64_t j = jb * TILE + acc_row(r, h);
                if (j < B && j != i) {
                    float v = acc[r] * inv_t;
                    s += expf(v - mn);
                    float w = pos_weight(labels, mask, B, i, j, li);
                    p.pos += w * v;
                    p.msum += w;
                }
            }
            p.m = mn;
            p.s = s;
        }
    }
    // merge the two row-halves of each column, then the 4 waves
    RowPart o;
    o.m = __shfl_xor(p.m, 32, 64);
    o.s = __shfl_xor(p.s, 32, 64);
    o.pos = __shfl_xor(p.pos, 32, 64);
    o.msum = __shfl_xor(p.msum, 32, 64);
    p = merge(p, o);
    __shared__ RowPart red[WAVES][TILE];
    if (h == 0) red[wave][lane] = p;
    __syncthreads();
    if (threadIdx.x < TILE) {
        RowPart q = red[0][threadIdx.x];
#pragma unroll
        for (int w = 1; w < WAVES; ++w) q = merge(q, red[w][threadIdx.x]);
        int64_t row = (int64_t)blockIdx.x * TILE + threadIdx.x;
        if (row < nrows) part[(int64_t)blockIdx.y * nrows + row] = q;
    }
}

// ---------------------------------------------------------------- forward: finalize
// rowstats[i] = {m_i, den_i, msum_i, loss_i} for the nrows anchors of the range; loss_out reduced
// per `reduction` over the range, the mean taken over all B anchors of the batch (a range's value
// is its share of the batch mean; the shares of a partition sum to the mean).
// (one block of FIN_T threads: the loss is one fixed-order tree sum; 1024 threads instead of 256 cut the
// per-thread chain of row merges 4x, 44 -> ~15 us at B = 4096)
constexpr int FIN_T = 1024;
__global__ __launch_bounds__(FIN_T) void supcon_rows_finalize(const RowPart* __restrict__ part,
                                                             int nsplit, int64_t B, int64_t nrows,
                                                             float t_over_bt, int reduction,
                                                             float4* __restrict__ rowstats,
                                                             float* __restrict__ loss_out) {
    __shared__ float red[FIN_T];
    float acc = 0.f;
    for (int64_t i = threadIdx.x; i < nrows; i += FIN_T) {
        RowPart q = part[i];
        for (int sp = 1; sp < nsplit; ++sp) q = merge(q, part[(int64_t)sp * nrows + i]);
        float den = q.s + 1e-6f;
        float P = (q.msum == 0.f) ? 1.f : q.msum;
        float mlpp = (q.pos - q.msum * q.m - q.msum * logf(den)) / P;
        float li = -t_over_bt * mlpp;
        rowstats[i] = make_float4(q.m, den, q.msum, li);
        if (reduction == PCX_REDUCTION_NONE) loss_out[i] = li;
        acc += li;
    }
    red[threadIdx.x] = acc;
    __syncthreads();
    for (int o = FIN_T / 2; o > 0; o >>= 1) {
        if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
        __syncthreads();
    }
    if (threadIdx.x == 0 && reduction != PCX_REDUCTION_NONE)
        loss_out[0] = (reduction == PCX_REDUCTION_MEAN) ? red[0] / (float)B : red[0];
}

// ---------------------------------------------------------------- backward: row coefficients
// G_ij = a_i M_ij - b_i exp(S_ij/T - m_i), a_i = -w_i/(base_T P_i), b_i = a_i msum_i / den_i
// (rows of one range; the mean's 1/B is over the whole batch as in the forward)
__global__ void supcon_coef(const float4* __restrict__ rowstats, const float* __restrict__ grad_out,
                            int64_t B, int64_t nrows, float inv_bt, int reduction,
                            float4* __restrict__ coef) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nrows) return;
    float4 st = rowstats[i];
    float w = (reduction == PCX_REDUCTION_NONE) ? grad_out[i]
              : (reduction == PCX_REDUCTION_MEAN ? grad_out[0] / (float)B : grad_out[0]);
    float P = (st.z == 0.f) ? 1.f : st.z;
    float a = -w * inv_bt / P;
    coef[i] = make_float4(a, a * st.z / st.y, st.x, 0.f);
}

// ---------------------------------------------------------------- backward: dF partials
template <int D>
__global__ __launch_bounds__(256) void supcon_grad_partial(
    const float* __restrict__ F, const int64_t* __restrict__ labels, const float* __restrict__ mask,
    const float4* __restrict__ coef, int64_t B, int64_t row0, int64_t nrows, float inv_t,
    int jblk_per_split, float* __restrict__ part) {
    constexpr int NQ = D / 32;  // 32-wide feature sub-tiles of dF
    const int lane = lane_id(), wave = threadIdx.x >> 6, h = lane >> 5;
    const int64_t il = (int64_t)blockIdx.x * TILE + (lane & 31);
    const int64_t i = row0 + il;
    const int64_t nj = (B + TILE - 1) / TILE;
    const bool ivalid = il < nrows;
    const int64_t li = (labels && ivalid) ? labels[i] : 0;
    const float4 ci = ivalid ? coef[i] : make_float4(0.f, 0.f, 0.f, 0.f);

    f32x16 acc[NQ];
#pragma unroll
    for (int q = 0; q < NQ; ++q) acc[q] = f32x16{0.f};

    const int64_t jb0 = (int64_t)blockIdx.y * jblk_per_split;
    const int64_t jb1 = min(nj, jb0 + jblk_per_split);
    AnchorFrag<kFrag<D> ? D : 8> fi;
    if constexpr (kFrag<D>) fi.load(F, i, B, h);
    for (int64_t jb = jb0 + wave; jb < jb1; jb += WAVES) {
        f32x16 s;
        if constexpr (kFrag<D>) s = tile_s_frag<D>(F, jb * TILE + (lane & 31), fi, B, h);
        else s = tile_s<D>(F, jb * TILE + (lane & 31), i, B, h);
        float hv[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            int64_t j = jb * TILE + acc_row(r, h);
            float v = 0.f;
            if (ivalid && j < B && j != i) {
                float4 cj = coef[j];
                float zs = s[r] * inv_t;
                float mij = pos_weight(labels, mask, B, i, j, li);
                float mji = labels ? mij : mask[j * B + i];
                v = ci.x * mij + cj.x * mji - ci.y * expf(zs - ci.z) - cj.y * expf(zs - cj.z);
            }
            hv[r] = v;
        }
        // dF_i += sum_j H_ij F_j : A = H (lane = anchor i, k = j of register r), B = F_j rows
        // (accumulator column n of sub-tile q is feature NQ n + q: the lane's NQ B values of a row are
        // consecutive floats, one 8- / 16-byte load per row instead of NQ dword loads; PCX_AB_SUPCON_DWORD:
        // feature 32 q + n, dword loads)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            int64_t j = jb * TILE + acc_row(r, h);
            bool jv = j < B;
            if constexpr (PCX_AB_SUPCON_DWORD) {
                const float* fj = F + j * D + (lane & 31);
#pragma unroll
                for (int q = 0; q < NQ; ++q) {
                    float b = jv ? fj[32 * q] : 0.f;
                    acc[q] = mfma32(hv[r], b, acc[q]);
                }
            } else {
                const float* fj = F + j * D + NQ * (lane & 31);
                float b[NQ];
#pragma unroll
                for (int q4 = 0; q4 < NQ; q4 += 4) {
                    if constexpr (NQ == 2) {
                        const float2 v = jv ? *reinterpret_cast<const float2*>(fj) : make_float2(0.f, 0.f);
                        b[0] = v.x;
                        b[1] = v.y;
                    } else {
                        const float4 v = jv ? ld4(fj + q4) : make_float4(0.f, 0.f, 0.f, 0.f);
                        b[q4] = v.x;
                        b[q4 + 1] = v.y;
                        b[q4 + 2] = v.z;
                        b[q4 + 3] = v.w;
                    }
                }
#pragma unroll
                for (int q = 0; q < NQ; ++q) acc[q] = mfma32(hv[r], b[q], acc[q]);
            }
        }
    }
    // reduce the 4 waves through LDS: out tile rows = anchors (acc_row), cols = features
    __shared__ float red[TILE][D + 1];
    for (int w = 0; w < WAVES; ++w) {
        if (wave == w) {
#pragma unroll
            for (int q = 0; q < NQ; ++q)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    float* dst = &red[acc_row(r, h)][PCX_AB_SUPCON_DWORD ? 32 * q + (lane & 31) : NQ * (lane & 31) + q];
                    *dst = (w == 0) ? acc[q][r] : *dst + acc[q][r];
                }
        }
        __syncthreads();
    }
    for (int e = threadIdx.x; e < TILE * D; e += blockDim.x) {
        int rr = e / D, cc = e % D;
        int64_t row = (int64_t)blockIdx.x * TILE + rr;
        if (row < nrows) part[((int64_t)blockIdx.y * nrows + row) * D + cc] = red[rr][cc];
    }
}

__global__ void sum_splits(const float* __restrict__ part, int nsplit, int64_t n,
                           float* __restrict__ out) {
    int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= n) return;
    float a = part[e];
    for (int s = 1; s < nsplit; ++s) a += part[(int64_t)s * n + e];
    out[e] = a;
}

struct Geo {
    int nib, nsplit, per;
};

// anchor-row blocks over the range x column splits over the whole batch
Geo geometry(int64_t B, int64_t nrows) {
    Geo g;
    g.nib = ceil_div(nrows, TILE);
    int64_t nj = ceil_div(B, TILE);
    int64_t want = nj / (WAVES * 4);  // aim for >= 4 j-blocks per wave
    g.nsplit = (int)(want < 1 ? 1 : (want > 16 ? 16 : want));
    g.per = ceil_div(nj, g.nsplit);
    g.nsplit = ceil_div(nj, g.per);
    return g;
}

int check_common(const float* F, const int64_t* labels, const float* mask, int64_t B, int64_t D,
                 float temperature, float base_temperature, int reduction) {
    PCX_CHECK_ARG(F != nullptr, "supcon: features is NULL");
    PCX_CHECK_ARG((labels != nullptr) != (mask != nullptr), "supcon: give exactly one of labels/mask");
    PCX_CHECK_ARG(B > 1, "Batch size must be greater than 1 for contrastive loss");
    PCX_CHECK_ARG(D == 64 || D == 128 || D == 256, "supcon: embedding dim %lld unsupported (64/128/256)",
                  (long long)D);
    PCX_CHECK_ARG(temperature > 0.f && base_temperature > 0.f, "supcon: temperatures must be > 0");
    PCX_CHECK_ARG(reduction >= 0 && reduction <= 2, "supcon: bad reduction %d", reduction);
    PCX_CHECK_ARG(((uintptr_t)F & 15) == 0, "supcon: features must be 16-byte aligned");
    return PCX_OK;
}

int check_range(int64_t B, int64_t row0, int64_t nrows) {
    PCX_CHECK_ARG(row0 >= 0 && nrows >= 1 && row0 + nrows <= B,
                  "supcon: anchor rows [%lld, %lld) outside the batch of %lld", (long long)row0,
                  (long long)(row0 + nrows), (long long)B);
    return PCX_OK;
}

size_t ws_bytes_rows(int64_t B, int64_t D, int64_t nrows, bool with_coef) {
    Geo g = geometry(B, nrows);
    size_t fwd = (size_t)g.nsplit * nrows * sizeof(RowPart);
    size_t bwd = (size_t)g.nsplit * nrows * D * sizeof(float) + (with_coef ? (size_t)B * sizeof(float4) : 0);
    size_t n = fwd > bwd ? fwd : bwd;
    return (n + 255) / 256 * 256;
}

void launch_rows_partial(const float* F, const int64_t* labels, const float* mask, int64_t B, int64_t D,
                         int64_t row0, int64_t nrows, float temperature, RowPart* part, const Geo& g,
                         hipStream_t stream) {
    dim3 grid(g.nib, g.nsplit);
    float inv_t = 1.0f / temperature;
    if (D == 64)
        supcon_rows_partial<64><<<grid, 256, 0, stream>>>(F, labels, mask, B, row0, nrows, inv_t, g.per, part);
    else if (D == 128)
        supcon_rows_partial<128><<<grid, 256, 0, stream>>>(F, labels, mask, B, row0, nrows, inv_t, g.per, part);
    else
        supcon_rows_partial<256><<<grid, 256, 0, stream>>>(F, labels, mask, B, row0, nrows, inv_t, g.per, part);
}

void launch_grad(const float* F, const int64_t* labels, const float* mask, int64_t B, int64_t D,
                 int64_t row0, int64_t nrows, float temperature, const float4* coef, float* part,
                 float* dF, const Geo& g, hipStream_t stream) {
    dim3 grid(g.nib, g.nsplit);
    float inv_t = 1.0f / temperature;
    if (D == 64)
        supcon_grad_partial<64><<<grid, 256, 0, stream>>>(F, labels, mask, coef, B, row0, nrows, inv_t, g.per, part);
    else if (D == 128)
        supcon_grad_partial<128><<<grid, 256, 0, stream>>>(F, labels, mask, coef, B, row0, nrows, inv_t, g.per, part);
    else
        supcon_grad_partial<256><<<grid, 256, 0, stream>>>(F, labels, mask, coef, B, row0, nrows, inv_t, g.per, part);
}

}  // namespace
}  // namespace pcx

using namespace pcx;

extern "C" size_t pcx_supcon_workspace_bytes(int64_t B, int64_t D) {
    if (B < 2) return 0;
    return ws_bytes_rows(B, D, B, true);
}

extern "C" size_t pcx_supcon_rows_workspace_bytes(int64_t B, int64_t D, int64_t nrows) {
    if (B < 2 || nrows < 1) return 0;
    return ws_bytes_rows(B, D, nrows, false);
}

extern "C" int pcx_supcon_forward_rows(const float* F, const int64_t* labels, const float* mask,
                                       int64_t B, int64_t D, int64_t row0, int64_t nrows,
                                       float temperature, float base_temperature, int reduction,
                                       float* loss_out, float* rowstats, void* ws, size_t ws_bytes,
                                       hipStream_t stream) {
    int rc = check_common(F, labels, mask, B, D, temperature, base_temperature, reduction);
    if (rc) return rc;
    if ((rc = check_range(B, row0, nrows))) return rc;
    PCX_CHECK_ARG(loss_out && rowstats, "supcon: NULL output");
    if (ws_bytes < ws_bytes_rows(B, D, nrows, false)) {
        set_error("supcon: workspace too small");
        return PCX_EWORKSPACE;
    }
    Geo g = geometry(B, nrows);
    RowPart* part = static_cast<RowPart*>(ws);
    launch_rows_partial(F, labels, mask, B, D, row0, nrows, temperature, part, g, stream);
    PCX_LAUNCH_CHECK("supcon_rows_partial");
    supcon_rows_finalize<<<1, FIN_T, 0, stream>>>(part, g.nsplit, B, nrows, temperature / base_temperature,
                                                 reduction, reinterpret_cast<float4*>(rowstats), loss_out);
    PCX_LAUNCH_CHECK("supcon_rows_finalize");
    return PCX_OK;
}

extern "C" int pcx_supcon_forward(const float* F, const int64_t* labels, const float* mask, int64_t B,
                                  int64_t D, float temperature, float base_temperature, int reduction,
                                  float* loss_out, float* rowstats, void* ws, size_t ws_bytes,
                                  hipStream_t stream) {
    return pcx_supcon_forward_rows(F, labels, mask, B, D, 0, B, temperature, base_temperature, reduction,
                                   loss_out, rowstats, ws, ws_bytes, stream);
}

extern "C" int pcx_supcon_coef_rows(const float* rowstats, const float* grad_out, int64_t B, int64_t nrows,
                                    float base_temperature, int reduction, float* coef, hipStream_t stream) {
    PCX_CHECK_ARG(rowstats && grad_out && coef, "supcon: NULL argument");
    PCX_CHECK_ARG(nrows >= 1 && nrows <= B, "supcon: bad row count %lld of %lld", (long long)nrows,
                  (long long)B);
    PCX_CHECK_ARG(base_temperature > 0.f, "supcon: temperatures must be > 0");
    PCX_CHECK_ARG(reduction >= 0 && reduction <= 2, "supcon: bad reduction %d", reduction);
    supcon_coef<<<ceil_div(nrows, 256), 256, 0, stream>>>(reinterpret_cast<const float4*>(rowstats), grad_out,
                                                           B, nrows, 1.0f / base_temperature, reduction,
                                                           reinterpret_cast<float4*>(coef));
    PCX_LAUNCH_CHECK("supcon_coef");
    return PCX_OK;
}

extern "C" int pcx_supcon_backward_rows(const float* F, const int64_t* labels, const float* mask,
                                        int64_t B, int64_t D, int64_t row0, int64_t nrows,
                                        float temperature, float base_temperature, const float* coef,
                                        float* dF, void* ws, size_t ws_bytes, hipStream_t stream) {
    int rc = check_common(F, labels, mask, B, D, temperature, base_temperature, 0);
    if (rc) return rc;
    if ((rc = check_range(B, row0, nrows))) return rc;
    PCX_CHECK_ARG(coef && dF, "supcon: NULL argument");
    if (ws_bytes < ws_bytes_rows(B, D, nrows, false)) {
        set_error("supcon: workspace too small");
        return PCX_EWORKSPACE;
    }
    Geo g = geometry(B, nrows);
    float* part = static_cast<float*>(ws);
    launch_grad(F, labels, mask, B, D, row0, nrows, temperature, reinterpret_cast<const float4*>(coef), part,
                dF, g, stream);
    PCX_LAUNCH_CHECK("supcon_grad_partial");
    int64_t n = nrows * D;
    sum_splits<<<ceil_div(n, 256), 256, 0, stream>>>(part, g.nsplit, n, dF);
    PCX_LAUNCH_CHECK("sum_splits");
    return PCX_OK;
}

extern "C" int pcx_supcon_backward(const float* F, const int64_t* labels, const float* mask, int64_t B,
                                   int64_t D, float temperature, float base_temperature, int reduction,
                                   const float* grad_out, const float* rowstats, float* dF, void* ws,
                                   size_t ws_bytes, hipStream_t stream) {
    int rc = check_common(F, labels, mask, B, D, temperature, base_temperature, reduction);
    if (rc) return rc;
    PCX_CHECK_ARG(grad_out && rowstats && dF, "supcon: NULL argument");
    if (ws_bytes < pcx_supcon_workspace_bytes(B, D)) {
        set_error("supcon: workspace too small");
        return PCX_EWORKSPACE;
    }
    Geo g = geometry(B, B);
    float* part = static_cast<float*>(ws);
    float* coef = part + (size_t)g.nsplit * B * D;
    if ((rc = pcx_supcon_coef_rows(rowstats, grad_out, B, B, base_temperature, reduction, coef, stream)))
        return rc;
    launch_grad(F, labels, mask, B, D, 0, B, temperature, reinterpret_cast<const float4*>(coef), part, dF, g,
                stream);
    PCX_LAUNCH_CHECK("supcon_grad_partial");
    int64_t n = B * D;
    sum_splits<<<ceil_div(n, 256), 256, 0, stream>>>(part, g.nsplit, n, dF);
    PCX_LAUNCH_CHECK("sum_splits");
    return PCX_OK;
}
