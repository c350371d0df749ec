// Semantics probe of the packed fp32 forms the Winograd transforms use (gfx950): operand selects, negations,
// broadcast, and the destination overlapping a source.  Prints per form the number of lanes that differ from
// the scalar expression.   hipcc -O3 --offload-arch=gfx950 tools/pk_probe.hip -o tools/pk_probe && tools/pk_probe
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f2 __attribute__((ext_vector_type(2)));

__global__ void probe(const float* in, int* bad) {
    const int l = threadIdx.x;
    const f2 a = {in[4 * l], in[4 * l + 1]}, b = {in[4 * l + 2], in[4 * l + 3]};
    f2 r, want;
    int k = 0;
#define CHECK(expr_x, expr_y) want = f2{expr_x, expr_y}; if (r.x != want.x || r.y != want.y) atomicAdd(bad + k, 1); ++k;
    asm volatile("v_pk_add_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    CHECK(a.x + b.x, a.y + b.y)
    asm volatile("v_pk_add_f32 %0, %1, %2 neg_lo:[0,1] neg_hi:[0,1]" : "=v"(r) : "v"(a), "v"(b));
    CHECK(a.x - b.x, a.y - b.y)
    asm volatile("v_pk_add_f32 %0, %1, %2 op_sel_hi:[1,0] neg_lo:[0,1]" : "=v"(r) : "v"(a), "v"(b));
    CHECK(a.x - b.x, a.y + b.x)
    asm volatile("v_pk_add_f32 %0, %1, %2 op_sel:[1,0] neg_lo:[1,0] neg_hi:[0,1]" : "=v"(r) : "v"(a), "v"(b));
    CHECK(b.x - a.y, a.y - b.y)
    asm volatile("v_pk_fma_f32 %0, %1, %2, %2 op_sel:[0,0,1] op_sel_hi:[1,0,1]" : "=v"(r) : "v"(a), "v"(b));
    CHECK(fmaf(a.x, b.x, b.y), fmaf(a.y, b.x, b.y))
    // destination = src1 / src0 (forced overlap)
    r = b;
    asm volatile("v_pk_add_f32 %0, %1, %0 op_sel_hi:[1,0] neg_lo:[0,1]" : "+v"(r) : "v"(a));
    CHECK(a.x - b.x, a.y + b.x)
    r = a;
    asm volatile("v_pk_add_f32 %0, %0, %1 op_sel:[1,0] neg_lo:[1,0] neg_hi:[0,1]" : "+v"(r) : "v"(b));
    CHECK(b.x - a.y, a.y - b.y)
    r = a;
    asm volatile("v_pk_fma_f32 %0, %0, %1, %1 op_sel:[0,0,1] op_sel_hi:[1,0,1]" : "+v"(r) : "v"(b));
    CHECK(fmaf(a.x, b.x, b.y), fmaf(a.y, b.x, b.y))
    r = b;
    asm volatile("v_pk_fma_f32 %0, %1, %0, %0 op_sel:[0,0,1] op_sel_hi:[1,0,1]" : "+v"(r) : "v"(a));
    CHECK(fmaf(a.x, b.x, b.y), fmaf(a.y, b.x, b.y))
    r = b;
    asm volatile("v_pk_add_f32 %0, %1, %0 neg_lo:[0,1] neg_hi:[0,1]" : "+v"(r) : "v"(a));
    CHECK(a.x - b.x, a.y - b.y)
}

int main2();
int main() {
    const int r2 = main2();
    const int n = 64;
    float h[4 * n];
    for (int i = 0; i < 4 * n; ++i) h[i] = (float)((i * 7919) % 1000) * 0.01f - 5.f + 0.001f * i;
    float* d;
    int* bad;
    (void)hipMalloc(&d, sizeof h);
    (void)hipMalloc(&bad, 64);
    (void)hipMemcpy(d, h, sizeof h, hipMemcpyHostToDevice);
    (void)hipMemset(bad, 0, 64);
    probe<<<1, n>>>(d, bad);
    int hb[16];
    (void)hipMemcpy(hb, bad, 64, hipMemcpyDeviceToHost);
    const char* names[] = {"add", "sub", "col01", "col23", "bn", "col01 dst=src1", "col23 dst=src0", "bn dst=src0",
                           "bn dst=src1,2", "sub dst=src1"};
    int tot = 0;
    for (int i = 0; i < 10; ++i) { printf("%-16s %d lanes wrong\n", names[i], hb[i]); tot += hb[i]; }
    return tot || r2 ? 1 : 0;
}

// ---- the engines' whole transforms through the shared helpers (csrc/pk_f32.h), against the scalar forms (bitwise)
#include "../phoneme_contrast_amd/csrc/pk_f32.h"
using pcx::pk_f2;

__global__ void transforms(const float* in, int* bad) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    const float* p = in + 36 * t;
    const pk_f2 st = {p[32], p[33]};
    // input transform of a 4x4 patch with BN + ReLU (conv_wino K-step)
    pk_f2 P[4][2];
    float d[4][4];
    for (int r = 0; r < 4; ++r) {
        P[r][0] = pk_f2{p[4 * r], p[4 * r + 1]};
        P[r][1] = pk_f2{p[4 * r + 2], p[4 * r + 3]};
        for (int c = 0; c < 4; ++c) d[r][c] = fmaxf(fmaf(p[4 * r + c], st.x, st.y), 0.f);
    }
    const pcx::PkK K = pcx::pk_consts();
    for (int r = 0; r < 4; ++r)
        for (int k = 0; k < 2; ++k) P[r][k] = pcx::pk_bnrelu(P[r][k], st);
    float g[16];
    pcx::pk_input_transform(K, P, g);
    float e_[4][4], v[16];
    for (int c = 0; c < 4; ++c) {
        e_[0][c] = d[0][c] - d[2][c];
        e_[1][c] = d[1][c] + d[2][c];
        e_[2][c] = d[2][c] - d[1][c];
        e_[3][c] = d[1][c] - d[3][c];
    }
    for (int r = 0; r < 4; ++r) {
        v[4 * r + 0] = e_[r][0] - e_[r][2];
        v[4 * r + 1] = e_[r][1] + e_[r][2];
        v[4 * r + 2] = e_[r][2] - e_[r][1];
        v[4 * r + 3] = e_[r][1] - e_[r][3];
    }
    int nb = 0;
    for (int x = 0; x < 16; ++x) nb += g[x] != v[x];
    if (nb) atomicAdd(bad + 10, 1);
    // output transform over channel pairs (acc[x] = 16 values x 2 channels)
    pk_f2 A[16];
    for (int x = 0; x < 16; ++x) A[x] = pk_f2{p[x] * 1.5f + st.x, p[(x * 5) & 31] - st.y};
    pk_f2 s0[4], s1[4];
    for (int c = 0; c < 4; ++c) {
        s0[c] = A[c] + A[4 + c] + A[8 + c];
        s1[c] = pcx::pk_sub(K, pcx::pk_sub(K, A[4 + c], A[8 + c]), A[12 + c]);
    }
    const pk_f2 y0 = s0[0] + s0[1] + s0[2];
    const pk_f2 y1 = pcx::pk_sub(K, pcx::pk_sub(K, s0[1], s0[2]), s0[3]);
    const pk_f2 y2 = s1[0] + s1[1] + s1[2];
    const pk_f2 y3 = pcx::pk_sub(K, pcx::pk_sub(K, s1[1], s1[2]), s1[3]);
    int ob = 0;
    for (int h = 0; h < 2; ++h) {
        float a0[16];
        for (int x = 0; x < 16; ++x) a0[x] = h ? A[x].y : A[x].x;
        float q0[4], q1[4];
        for (int c = 0; c < 4; ++c) {
            q0[c] = a0[c] + a0[4 + c] + a0[8 + c];
            q1[c] = a0[4 + c] - a0[8 + c] - a0[12 + c];
        }
        const float z0 = q0[0] + q0[1] + q0[2], z1 = q0[1] - q0[2] - q0[3];
        const float z2 = q1[0] + q1[1] + q1[2], z3 = q1[1] - q1[2] - q1[3];
        ob += (z0 != (h ? y0.y : y0.x)) + (z1 != (h ? y1.y : y1.x)) + (z2 != (h ? y2.y : y2.x)) + (z3 != (h ? y3.y : y3.x));
    }
    if (ob) atomicAdd(bad + 11, 1);
}

int main2() {
    const int n = 1 << 16;
    float* h = new float[36 * n];
    unsigned s = 12345;
    for (int i = 0; i < 36 * n; ++i) { s = s * 1664525u + 1013904223u; h[i] = (float)(s >> 8) / (1 << 24) * 8.f - 4.f; }
    float* d;
    int* bad;
    (void)hipMalloc(&d, 36 * (size_t)n * 4);
    (void)hipMalloc(&bad, 64);
    (void)hipMemcpy(d, h, 36 * (size_t)n * 4, hipMemcpyHostToDevice);
    (void)hipMemset(bad, 0, 64);
    transforms<<<n / 256, 256>>>(d, bad);
    int hb[16];
    (void)hipMemcpy(hb, bad, 64, hipMemcpyDeviceToHost);
    printf("input transform (BN + ReLU, packed): %d of %d threads differ\n", hb[10], n);
    printf("output transform (packed pairs):     %d of %d threads differ\n", hb[11], n);
    delete[] h;
    return hb[10] + hb[11] ? 1 : 0;
}
