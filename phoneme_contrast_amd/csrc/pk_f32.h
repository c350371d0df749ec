// Packed fp32 arithmetic for the Winograd transforms (v_pk_add_f32 / v_pk_fma_f32): beside fp32 MFMAs one
// packed instruction costs ~1.6x one v_add_f32 at two waves per SIMD and does two (tools/mfma_mix.hip,
// profiles/r6_mfma_mix_packed.txt).  Written as float2 vector arithmetic the compiler can see (not inline
// asm: it must insert the MFMA -> VALU wait states for reads of accumulators, which it does not do for an
// asm operand).  Subtractions are fma(b, -1, a) with the -1 an opaque scalar register: the compiler turns a
// plain float2 subtraction of accumulator halves into two v_sub_f32 (the v4f32 subtraction it first forms is
// scalarised), and would fold a literal -1 back into that subtraction.  Every lane's result is the scalar
// operation's, bit for bit: fma(b, -1, a) = round(a - b), fma(e, 1, f) = round(e + f).
#pragma once

namespace pcx {

typedef float pk_f2 __attribute__((ext_vector_type(2)));

struct PkK {
    pk_f2 m1;  // {-1, -1}
    pk_f2 pm;  // {1, -1}
};

__device__ __forceinline__ PkK pk_consts() {
    float p1, m1;
    asm("s_mov_b32 %0, 1.0" : "=s"(p1));
    asm("s_mov_b32 %0, -1.0" : "=s"(m1));
    return PkK{pk_f2{m1, m1}, pk_f2{p1, m1}};
}

__device__ __forceinline__ pk_f2 pk_sub(const PkK& k, pk_f2 a, pk_f2 b) {  // a - b
    return __builtin_elementwise_fma(b, k.m1, a);
}

// BN + ReLU of both lanes: max(fma(d, s, t), 0), st = {s, t}
__device__ __forceinline__ pk_f2 pk_bnrelu(pk_f2 d, pk_f2 st) {
    const pk_f2 y = __builtin_elementwise_fma(d, st.xx, st.yy);
    return pk_f2{fmaxf(y.x, 0.f), fmaxf(y.y, 0.f)};
}

// Winograd F(2x2, 3x3) input transform V = B^T d B of a 4x4 patch held as row pairs P[r][0] = d[r][0..1],
// P[r][1] = d[r][2..3]; v[16] in the scalar order v[4 r + c] (rows first, then columns):
//   rows:    e0 = d0 - d2, e1 = d1 + d2, e2 = d2 - d1, e3 = d1 - d3           (8 packed)
//   columns: {v0, v3} = {e0, e1} - {e2, e3},  {v1, v2} = fma({e1, e1}, {1, -1}, {e2, e2})   (8 packed)
__device__ __forceinline__ void pk_input_transform(const PkK& k, const pk_f2 (&P)[4][2], float (&v)[16]) {
    pk_f2 E[4][2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        E[0][h] = pk_sub(k, P[0][h], P[2][h]);
        E[1][h] = P[1][h] + P[2][h];
        E[2][h] = pk_sub(k, P[2][h], P[1][h]);
        E[3][h] = pk_sub(k, P[1][h], P[3][h]);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const pk_f2 a = E[r][0], b = E[r][1];
        const pk_f2 c03 = pk_sub(k, a, b);
        const pk_f2 c12 = __builtin_elementwise_fma(a.yy, k.pm, b.xx);
        v[4 * r + 0] = c03.x;
        v[4 * r + 3] = c03.y;
        v[4 * r + 1] = c12.x;
        v[4 * r + 2] = c12.y;
    }
}

}  // namespace pcx
