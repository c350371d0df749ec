// Does VALU work overlap v_mfma_f32_32x32x2_f32 on gfx950?  Times (a) MFMA-only waves, (b) MFMA +
// n VALU fma per MFMA in the same wave, (c) MFMA-only and VALU-only waves side by side on a SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int NV, int MODE>
__global__ __launch_bounds__(512) void k(float* out, int iters, float a, float b) {
    __shared__ float sh[2048];
    sh[threadIdx.x] = threadIdx.x;
    __syncthreads();
    f32x16 acc[4];
    for (int i = 0; i < 4; ++i) acc[i] = f32x16{0.f};
    float v[8];
    for (int i = 0; i < 8; ++i) v[i] = threadIdx.x * 0.001f + i;
    const int wave = threadIdx.x >> 6;
    const bool do_mfma = MODE == 0 || MODE == 2 || (MODE == 1 && (wave & 1) == 0);
    const bool do_valu = MODE == 0 || (MODE == 1 && (wave & 1) == 1);
    for (int it = 0; it < iters; ++it) {
        if (do_mfma) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[j], 0, 0, 0);
                if (do_valu && MODE != 2) {
#pragma unroll
                    for (int q = 0; q < NV; ++q) v[q & 7] = fmaf(v[q & 7], a, b);
                }
                if (MODE == 2) {
#pragma unroll
                    for (int q = 0; q < NV; ++q) v[q & 7] += sh[(threadIdx.x + 64 * q + it) & 2047];
                }
            }
        } else if (do_valu) {
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int q = 0; q < NV; ++q) v[q & 7] = fmaf(v[q & 7], a, b);
        }
    }
    float s = 0.f;
    for (int i = 0; i < 4; ++i) for (int r = 0; r < 16; ++r) s += acc[i][r];
    for (int i = 0; i < 8; ++i) s += v[i];
    if (s == 1234.5f) out[threadIdx.x] = s;
}

template <int NV, int MODE>
float run(int blocks, int threads, int iters) {
    float* d; hipMalloc(&d, 4096);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    k<NV, MODE><<<blocks, threads>>>(d, iters, 1.0001f, 0.0001f);
    hipEventRecord(e0);
    k<NV, MODE><<<blocks, threads>>>(d, iters, 1.0001f, 0.0001f);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    hipFree(d);
    return ms;
}

int main() {
    const int iters = 20000;
    // one block of 256 threads (4 waves, 1 per SIMD) per CU, or 512 threads (2 waves per SIMD)
    for (int threads : {256, 512}) {
        const int blocks = 256;
        double mf = (double)blocks * (threads / 64) * iters * 4 * 32 * 32 * 2 * 2;
        printf("threads %d\n", threads);
        float t0 = run<0, 0>(blocks, threads, iters);
        printf("  mfma only          %.3f ms  %.1f TF/s\n", t0, mf / t0 / 1e9);
        float t1 = run<4, 0>(blocks, threads, iters);
        printf("  mfma+4 fma/mfma    %.3f ms  (+%.1f%%)\n", t1, 100 * (t1 / t0 - 1));
        float t2 = run<8, 0>(blocks, threads, iters);
        printf("  mfma+8 fma/mfma    %.3f ms  (+%.1f%%)\n", t2, 100 * (t2 / t0 - 1));
        float t3 = run<16, 0>(blocks, threads, iters);
        printf("  mfma+16 fma/mfma   %.3f ms  (+%.1f%%)\n", t3, 100 * (t3 / t0 - 1));
        float t6 = run<4, 2>(blocks, threads, iters);
        printf("  mfma+4 lds(+add)/mfma %.3f ms  (+%.1f%%)\n", t6, 100 * (t6 / t0 - 1));
        float t7 = run<8, 2>(blocks, threads, iters);
        printf("  mfma+8 lds(+add)/mfma %.3f ms  (+%.1f%%)\n", t7, 100 * (t7 / t0 - 1));
        if (threads == 512) {
            float t4 = run<16, 1>(blocks, threads, iters);
            printf("  split: mfma waves | 16-fma waves  %.3f ms (mfma-only half would be %.3f)\n", t4, t0 / 2);
            float t5 = run<32, 1>(blocks, threads, iters);
            printf("  split: mfma waves | 32-fma waves  %.3f ms\n", t5);
        }
    }
    return 0;
}
