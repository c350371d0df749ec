// What does non-MFMA work cost beside a stream of fp32 v_mfma_f32_16x16x4_f32 on gfx950 (analysis aid for
// the Winograd engines' design)?  Each wave runs ITERS x 8 independent MFMAs (8 accumulators) and, per MFMA,
// N filler instructions of one kind:
//   kind 0 none, 1 v_fma_f32 (independent), 2 ds_read_b128 (results kept live, consumed at the end),
//   3 buffer_load_dwordx4 ... lds (1 KiB LDS-DMA per wave-instruction, L2-resident source; vmcnt bounded),
//   4 buffer_load_dword ... lds (256 B), 5 ds_read_b64, 6 v_add_f32 (inline asm, independent), 7 v_pk_add_f32
//   (two f32 adds per lane), 8 v_pk_fma_f32, 9 v_max_f32 (inline asm, independent), 10 global_load_lds_dwordx4
//   (saddr + voffset LDS-DMA, 1 KiB), 11 global_load_dwordx4 to VGPRs, 12 buffer_load_dwordx4 to VGPRs,
//   13 ds_write_b128
// at 1 wave per SIMD (256-thread blocks) and 2 waves per SIMD (512), one block per CU.  Prints cycles per
// MFMA at the measured clock-free rate (ms) and the extra time per filler instruction.
//   hipcc -O3 --offload-arch=gfx950 tools/mfma_mix.hip -o tools/mfma_mix && tools/mfma_mix
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void;

template <int KIND, int N>
__global__ __launch_bounds__(512) void mix(const float* __restrict__ src, float* out, int iters, float a, float b) {
    __shared__ __attribute__((aligned(16))) float sh[16384];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    for (int i = tid; i < 16384; i += blockDim.x) sh[i] = (float)i * 1e-3f;
    __syncthreads();
    f32x4 acc[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    float v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = tid * 1e-3f + i;
    typedef float f2v __attribute__((ext_vector_type(2)));
    f2v p2[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) p2[i] = f2v{tid * 1e-3f + i, tid * 2e-3f - i};
    const f2v ka = f2v{a, b}, kb = f2v{b, a};
    f32x4 r4[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) r4[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(src), (short)0, 1 << 22, 0x00020000);
    const unsigned ldsb = (unsigned)(uintptr_t)(lds_void*)sh + 1024u * (unsigned)wave;
    float aa = a + lane * 1e-6f, bb = b;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(aa, bb, acc[j], 0, 0, 0);
#pragma unroll
            for (int q = 0; q < N; ++q) {
                if constexpr (KIND == 1) v[q & 7] = fmaf(v[q & 7], a, b);
                if constexpr (KIND == 2) {  // (inline asm: no add, no compiler wait; drained at the end)
                    const unsigned ad = ldsb + 16u * lane + 1024u * (unsigned)((j * N + q) & 7);
                    asm volatile("ds_read_b128 %0, %1" : "=v"(r4[(j * N + q) & 7]) : "v"(ad) : "memory");
                }
                if constexpr (KIND == 6)
                    asm volatile("v_add_f32 %0, %0, %1" : "+v"(v[(j * N + q) & 7]) : "v"(aa));
                if constexpr (KIND == 7)
                    asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(p2[(j * N + q) & 7]) : "v"(ka));
                if constexpr (KIND == 8)
                    asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(p2[(j * N + q) & 7]) : "v"(ka), "v"(kb));
                if constexpr (KIND == 9)
                    asm volatile("v_max_f32 %0, %0, %1" : "+v"(v[(j * N + q) & 7]) : "v"(aa));
                if constexpr (KIND == 10) {
                    const unsigned m0 = __builtin_amdgcn_readfirstlane(ldsb + 8192u * (unsigned)((j * N + q) & 1));
                    const unsigned voff = (unsigned)((lane * 16 + 1024 * ((it * 8 + j) * N + q)) & ((1 << 22) - 1));
                    asm volatile("s_nop 0\n\tglobal_load_lds_dwordx4 %0, %1" :: "v"(voff), "s"(src), "{m0}"(m0) : "memory");
                }
                if constexpr (KIND == 11) {
                    const unsigned voff = (unsigned)((lane * 16 + 1024 * ((it * 8 + j) * N + q)) & ((1 << 22) - 1));
                    asm volatile("global_load_dwordx4 %0, %1, %2" : "=v"(r4[(j * N + q) & 7]) : "v"(voff), "s"(src) : "memory");
                }
                if constexpr (KIND == 12) {
                    const unsigned voff = (unsigned)((lane * 16 + 1024 * ((it * 8 + j) * N + q)) & ((1 << 22) - 1));
                    asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen" : "=v"(r4[(j * N + q) & 7]) : "v"(voff), "s"(rs) : "memory");
                }
                if constexpr (KIND == 13) {
                    const unsigned ad = ldsb + 16u * lane + 1024u * (unsigned)((j * N + q) & 7);
                    asm volatile("ds_write_b128 %0, %1" :: "v"(ad), "v"(r4[(j * N + q) & 7]) : "memory");
                }
                if constexpr (KIND == 5) {
                    const unsigned ad = ldsb + 8u * lane + 1024u * (unsigned)((j * N + q) & 7);
                    float2 t;
                    asm volatile("ds_read_b64 %0, %1" : "=v"(t) : "v"(ad) : "memory");
                    v[q & 7] = t.x;
                }
                if constexpr (KIND == 3 || KIND == 4) {
                    const unsigned m0 = __builtin_amdgcn_readfirstlane(ldsb + (KIND == 3 ? 8192u : 8192u) * (unsigned)((j * N + q) & 1));
                    const unsigned voff = (unsigned)((lane * (KIND == 3 ? 16 : 4) + 1024 * ((it * 8 + j) * N + q)) & ((1 << 22) - 1));
                    if constexpr (KIND == 3)
                        asm volatile("s_nop 0\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds" :: "v"(voff), "s"(rs), "{m0}"(m0) : "memory");
                    else
                        asm volatile("s_nop 0\n\tbuffer_load_dword %0, %1, 0 offen lds" :: "v"(voff), "s"(rs), "{m0}"(m0) : "memory");
                }
            }
        }
        if constexpr (KIND == 3 || KIND == 4 || KIND >= 10) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    }
    if constexpr (KIND == 3 || KIND == 4 || KIND >= 10) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3] + v[i] + r4[i][0] + r4[i][3] + p2[i][0] + p2[i][1];
    if (s == 1234.5f) out[tid] = s + sh[tid];
}

template <int KIND, int N>
float run(const float* src, int threads, int iters) {
    float* d;
    (void)hipMalloc(&d, 4096 * 4);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    mix<KIND, N><<<256, threads>>>(src, d, iters, 1.0001f, 0.0001f);
    (void)hipEventRecord(e0);
    for (int r = 0; r < 3; ++r) mix<KIND, N><<<256, threads>>>(src, d, iters, 1.0001f, 0.0001f);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    (void)hipFree(d);
    return ms / 3;
}

int main() {
    float* src;
    (void)hipMalloc(&src, 1 << 22);
    (void)hipMemset(src, 0, 1 << 22);
    const int iters = 4000;
    for (int threads : {256, 512}) {
        const double nm = (double)iters * 8;  // MFMAs per wave
        const float t0 = run<0, 0>(src, threads, iters);
        const double cyc = 32.0;  // SIMD cycles per MFMA at full rate: extra SIMD cycles per filler = frac x 32 / n
        printf("waves/SIMD %d: bare MFMA %.3f ms (%.1f TF/s)\n", threads / 256, t0,
               256.0 * threads / 64 * nm * 2048 / (t0 * 1e9));
        auto rep = [&](const char* what, int n, float t) {
            // extra time per filler, in units of one MFMA's share of the bare time
            printf("  %-28s x%d/MFMA: %.3f ms  +%.1f%%  = %.1f MFMA-cycles per filler\n", what, n, t, 100 * (t / t0 - 1),
                   (t / t0 - 1) * cyc / n);
        };
        rep("v_fma_f32", 1, run<1, 1>(src, threads, iters));
        rep("v_fma_f32", 2, run<1, 2>(src, threads, iters));
        rep("v_fma_f32", 4, run<1, 4>(src, threads, iters));
        rep("v_add_f32 (asm)", 2, run<6, 2>(src, threads, iters));
        rep("v_add_f32 (asm)", 4, run<6, 4>(src, threads, iters));
        rep("v_pk_add_f32", 1, run<7, 1>(src, threads, iters));
        rep("v_pk_add_f32", 2, run<7, 2>(src, threads, iters));
        rep("v_pk_add_f32", 4, run<7, 4>(src, threads, iters));
        rep("v_pk_fma_f32", 2, run<8, 2>(src, threads, iters));
        rep("v_pk_fma_f32", 4, run<8, 4>(src, threads, iters));
        rep("v_max_f32 (asm)", 4, run<9, 4>(src, threads, iters));
        rep("ds_read_b128", 1, run<2, 1>(src, threads, iters));
        rep("ds_read_b128", 2, run<2, 2>(src, threads, iters));
        rep("ds_read_b64", 1, run<5, 1>(src, threads, iters));
        rep("buffer_load_dwordx4 lds", 1, run<3, 1>(src, threads, iters));
        rep("buffer_load_dwordx4 lds", 2, run<3, 2>(src, threads, iters));
        rep("buffer_load_dword lds", 1, run<4, 1>(src, threads, iters));
        rep("global_load_lds_dwordx4", 1, run<10, 1>(src, threads, iters));
        rep("global_load_dwordx4 (VGPR)", 1, run<11, 1>(src, threads, iters));
        rep("buffer_load_dwordx4 (VGPR)", 1, run<12, 1>(src, threads, iters));
        rep("ds_write_b128", 1, run<13, 1>(src, threads, iters));
        rep("ds_write_b128", 2, run<13, 2>(src, threads, iters));
    }
    return 0;
}
