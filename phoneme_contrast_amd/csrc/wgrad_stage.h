// Row staging of the sliding-row-window weight-gradient kernel (wgrad_w32.hip, 32 x 32 tiles):
// per-thread register prefetch of the next dz / y / x rows,
// BN backward / x prologue / zero padding, stores into the LDS row ring.
#pragma once
#include "kernels.h"

namespace pcx {
namespace {

template <int V>
using vecf = float __attribute__((ext_vector_type(V)));

// LDS: dy rows [2][NB][DS] | x rows [4][CB][XSP].  dy image column j = sample column w0 + j;
// x image column jj = sample column w0 - VX + jj (jj < CW + 2 VX; x is staged VX-wide, VX <= VEC,
// so that narrower halos can buy a wider strip).  Image row rho of x lives in
// slot (rho + 1) & 3, dy row rho in slot rho & 1.  DS and XSP are 2 * odd: the 16x16 operand reads
// (16 channels x 2 pixels per 32-lane group) are bank-conflict free and b64 stores stay aligned.
struct Geo {
    int CW, QD, QX, DS, XSP, nqd, nqx, dyslot, xslot, xbase;
};

__host__ __device__ inline int pad2odd(int n) {  // smallest m >= n with m = 2 * odd
    while ((n & 3) != 2) ++n;
    return n;
}

// Per-thread staging walk over the quads (VEC-vectors) of the flattened dy image [NB][QD] and x
// image [CB][QX]: quad e = tid + 256 i, advanced incrementally (no divisions in the row loop).
struct Walk {
    int n0, q0, dn, dq;   // dy
    int c0, qx0, dc, dqx; // x
};

// The walk offsets do not depend on the row: left alone, the compiler hoists all of them out of
// the row loop and spills.  An empty asm makes the walk start opaque per call.
__device__ __forceinline__ void opaque(int& x, int& y) { asm volatile("" : "+v"(x), "+v"(y)); }

template <int V>
__device__ __forceinline__ void lds_store(float* p, vecf<V> v) {
    if constexpr (V == 4) {  // 8-byte aligned (strides are 2 * odd)
        *reinterpret_cast<vecf<2>*>(p) = vecf<2>{v[0], v[1]};
        *reinterpret_cast<vecf<2>*>(p + 2) = vecf<2>{v[2], v[3]};
    } else {
        *reinterpret_cast<vecf<V>*>(p) = v;
    }
}

template <int PRO, int VEC, int VX, int NQDY, int NQX>
struct RowStage {
    vecf<VEC> dzv[NQDY], yv[NQDY];
    vecf<VX> xv[NQX];

    __device__ __forceinline__ void load_dy(const WgradArgs& a, const Geo& g, const Walk& wk, const float* dzb,
                                            const float* yb, int w0, int r, int NB) {
        const int HW = a.H * a.W, qlim = (a.W - VEC - w0) / VEC;  // last quad inside the sample
        int n = wk.n0, q = wk.q0;
        opaque(n, q);
        const float* dzr = dzb + r * a.W + w0;
        const float* yr = yb + r * a.W + w0;
#pragma unroll
        for (int i = 0; i < NQDY; ++i) {
            const int o = min(n, NB - 1) * HW + VEC * min(q, qlim);
            dzv[i] = *reinterpret_cast<const vecf<VEC>*>(dzr + o);
            yv[i] = *reinterpret_cast<const vecf<VEC>*>(yr + o);
            n += wk.dn;
            q += wk.dq;
            if (q >= g.QD) { q -= g.QD; ++n; }
        }
    }
    // values first (branch-free), then the LDS / HBM stores
    __device__ __forceinline__ void store_dy(const WgradArgs& a, const Geo& g, const Walk& wk, int tid, float* lds,
                                             const float4* cfd, float* dyo, int w0, int r, int slot, int NB) {
        const int HW = a.H * a.W, qlim = (a.W - VEC - w0) / VEC;
        int n = wk.n0, q = wk.q0;
        opaque(n, q);
#pragma unroll
        for (int i = 0; i < NQDY; ++i) {
            const float4 k = cfd[min(n, NB - 1)];
            vecf<VEC> v;
#pragma unroll
            for (int e = 0; e < VEC; ++e) v[e] = k.x * (dzv[i][e] - k.y - (yv[i][e] - k.w) * k.z);
            dzv[i] = q <= qlim ? v : vecf<VEC>(0.f);
            n += wk.dn;
            q += wk.dq;
            if (q >= g.QD) { q -= g.QD; ++n; }
        }
        n = wk.n0;
        q = wk.q0;
        opaque(n, q);
        float* dyr = dyo ? dyo + r * a.W + w0 : nullptr;
#pragma unroll
        for (int i = 0; i < NQDY; ++i) {
            if (tid + 256 * i < g.nqd) {
                lds_store<VEC>(lds + slot * g.dyslot + n * g.DS + VEC * q, dzv[i]);
                if (dyr && q <= qlim) *reinterpret_cast<vecf<VEC>*>(dyr + n * HW + VEC * q) = dzv[i];
            }
            n += wk.dn;
            q += wk.dq;
            if (q >= g.QD) { q -= g.QD; ++n; }
        }
    }
    __device__ __forceinline__ void load_x(const WgradArgs& a, const Geo& g, const Walk& wk, const float* xb,
                                           int w0, int rx, int CB) {
        const int HW = a.H * a.W;
        int c = wk.c0, q = wk.qx0;
        opaque(c, q);
        const float* xr = xb + rx * a.W;
#pragma unroll
        for (int i = 0; i < NQX; ++i) {
            const int w = min(max(w0 - VX + VX * q, 0), a.W - VX);
            xv[i] = *reinterpret_cast<const vecf<VX>*>(xr + min(c, CB - 1) * HW + w);
            c += wk.dc;
            q += wk.dqx;
            if (q >= g.QX) { q -= g.QX; ++c; }
        }
    }
    __device__ __forceinline__ void store_x(const WgradArgs& a, const Geo& g, const Walk& wk, int tid, float* lds,
                                            const float4* cfx, int w0, int slot, int CB) {
        int c = wk.c0, q = wk.qx0;
        opaque(c, q);
#pragma unroll
        for (int i = 0; i < NQX; ++i) {
            const int w = w0 - VX + VX * q;
            vecf<VX> v = xv[i];
            if (PRO == PRO_BNRELU) {
                const float4 k = cfx[min(c, CB - 1)];
#pragma unroll
                for (int e = 0; e < VX; ++e) v[e] = fmaxf(fmaf(v[e], k.x, k.y), 0.f);
            }
            xv[i] = (w >= 0 && w < a.W) ? v : vecf<VX>(0.f);
            c += wk.dc;
            q += wk.dqx;
            if (q >= g.QX) { q -= g.QX; ++c; }
        }
        c = wk.c0;
        q = wk.qx0;
        opaque(c, q);
#pragma unroll
        for (int i = 0; i < NQX; ++i) {
            if (tid + 256 * i < g.nqx) lds_store<VX>(lds + g.xbase + slot * g.xslot + c * g.XSP + VX * q, xv[i]);
            c += wk.dc;
            q += wk.dqx;
            if (q >= g.QX) { q -= g.QX; ++c; }
        }
    }
};

inline size_t win_lds(int NB, int CB, int CW, int vx) {
    return ((size_t)2 * NB * pad2odd(CW) + (size_t)4 * CB * pad2odd(CW + 2 * vx) + 4 * (size_t)(NB + CB)) * 4;
}

inline int win_vec(int W) { return (W % 4 == 0) ? 4 : (W % 2 == 0) ? 2 : 1; }

}  // namespace
}  // namespace pcx
