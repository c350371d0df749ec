// Shared device/host helpers for libpcx (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "pcx.h"

namespace pcx {

// ---------------------------------------------------------------- error state (host)
void set_error(const char* fmt, ...);
int hip_status(hipError_t e, const char* what);
int num_cus();  // compute units of the current device

#define PCX_CHECK_ARG(cond, ...)                  \
    do {                                          \
        if (!(cond)) {                            \
            ::pcx::set_error(__VA_ARGS__);        \
            return PCX_EINVAL;                    \
        }                                         \
    } while (0)

#define PCX_LAUNCH_CHECK(what)                                            \
    do {                                                                  \
        hipError_t _e = hipGetLastError();                                \
        if (_e != hipSuccess) return ::pcx::hip_status(_e, what);         \
    } while (0)

// ---------------------------------------------------------------- device helpers
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int WAVE = 64;

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }

// D = A(32x2) * B(2x32) + C, exact f32 (v_mfma_f32_32x32x2_f32).
// lane l supplies A[i=l&31][k=l>>5] and B[k=l>>5][j=l&31];
// C/D register r of lane l holds (row (r&3)+8*(r>>2)+4*(l>>5), col l&31).
__device__ __forceinline__ f32x16 mfma32(float a, float b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

// row of accumulator register r for lane half h (32x32 C/D layout)
__device__ __forceinline__ int acc_row(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}
// combine lanes l and l^32 (the two row-halves of a 32x32 accumulator column)
__device__ __forceinline__ float half_sum(float v) { return v + __shfl_xor(v, 32, 64); }
__device__ __forceinline__ float half_max(float v) { return fmaxf(v, __shfl_xor(v, 32, 64)); }

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ void st4(float* p, float4 v) { *reinterpret_cast<float4*>(p) = v; }

inline int ceil_div(int64_t a, int64_t b) { return (int)((a + b - 1) / b); }

}  // namespace pcx

// nonnegative n / d in 32 bits, for index arithmetic whose operands the launcher has checked to be < 2^31 (round 6:
// an int64 division compiles to ~100 scalar or ~60 vector instructions; convg / convg_bf16 did several per block and
// per K-chunk and lane)
namespace pcx {
__host__ __device__ __forceinline__ int64_t udiv32(int64_t n, int64_t d) { return (int64_t)((unsigned)n / (unsigned)d); }
}  // namespace pcx

// ---------------------------------------------------------------- A/B alternates (analysis builds only)
// The measured-and-superseded alternates of the product kernels (the round-4/5 A/B comparisons in DESIGN.md)
// are compile-time switches: `make AB="-DPCX_AB_NO_WGBD=1"` builds a library that takes the old path.  The
// shipped libpcx.so is built with every one at its default and reads no environment variable that selects a
// kernel or changes numerics (PCX_ROCTX only names profiler ranges).
#ifndef PCX_AB_WINO_SLOT          // 1: static blockIdx unit order in conv_wino (no XCD-contiguous slots)
#define PCX_AB_WINO_SLOT 0
#endif
#ifndef PCX_AB_NO_WINO_X4         // 1: dword operand copies instead of 16-byte LDS-DMA in conv_wino
#define PCX_AB_NO_WINO_X4 0
#endif
#ifndef PCX_AB_NO_WINO_QUEUE      // 1: static unit order instead of the per-XCD work queue
#define PCX_AB_NO_WINO_QUEUE 0
#endif
#ifndef PCX_AB_NO_POOLSEL         // 1: pooled data gradients re-read the producer's full-resolution windows
#define PCX_AB_NO_POOLSEL 0
#endif
#ifndef PCX_AB_NO_POOLDZ          // 1: no pooled gradient hand-over to layers 2 / 4 (dz written at full size)
#define PCX_AB_NO_POOLDZ 0
#endif
#ifndef PCX_AB_NO_WGBD            // 1: layer 2's weight and data gradients as two kernels
#define PCX_AB_NO_WGBD 0
#endif
#ifndef PCX_AB_WGBD_UNPAIRED      // 1: wgbd blocks walk their own task runs (no XCD-paired strips)
#define PCX_AB_WGBD_UNPAIRED 0
#endif
#ifndef PCX_AB_POOL_NI            // pixel quads per thread and pass in bn_relu_pool
#define PCX_AB_POOL_NI 2
#endif
#ifndef PCX_AB_NHWC_ROWS1         // 1: the channel-last writer steps one image row at a time
#define PCX_AB_NHWC_ROWS1 0
#endif
#ifndef PCX_AB_NO_CONVN_HALO      // 1: per-tap channel-last bf16 conv instead of the halo-staged one
#define PCX_AB_NO_CONVN_HALO 0
#endif
#ifndef PCX_AB_CONVN_NW           // 4 / 8: force the halo kernel's waves per block (0: by shape)
#define PCX_AB_CONVN_NW 0
#endif
#ifndef PCX_AB_CHAN_TARGET        // blocks of the channel-reduction passes
#define PCX_AB_CHAN_TARGET 16384
#endif
#ifndef PCX_AB_BN_ROWTILE         // 1: BN apply passes as row tiles instead of flat 16-byte streams
#define PCX_AB_BN_ROWTILE 0
#endif
#ifndef PCX_AB_NO_WINO_SPAN       // 1: narrow cnn_deep blocks on the direct conv (no batch-spanning Winograd)
#define PCX_AB_NO_WINO_SPAN 0
#endif
#ifndef PCX_AB_NO_EPSUMS          // 1: the BN-backward sums of the channel-last data gradient as a separate pass
#define PCX_AB_NO_EPSUMS 0
#endif
#ifndef PCX_AB_WW_NH1             // 1: Winograd weight gradient blocks of 32 input channels only (no 8-wave NH = 2)
#define PCX_AB_WW_NH1 0
#endif
#ifndef PCX_AB_NO_PSEL            // 1: block tails by bn_relu_pool (no pool selection in the producer's epilogue)
#define PCX_AB_NO_PSEL 0
#endif
#ifndef PCX_AB_WW_ODD_ALL         // 1: odd-width Winograd weight gradients at any tile coverage (analysis builds)
#define PCX_AB_WW_ODD_ALL 0
#endif
#ifndef PCX_AB_WINO_X4_RAWFWD     // 1: 16-byte operand copies for the raw-input Winograd forward too (layers 3 / 5)
#define PCX_AB_WINO_X4_RAWFWD 0
#endif
#ifndef PCX_AB_NO_NT_STORES       // 1: plain (not streaming) output stores in conv_wino / wgrad_wino / wgbd_wino (nt measured 2 % slower)
#define PCX_AB_NO_NT_STORES 1
#endif
#ifndef PCX_AB_SUPCON_DWORD       // 1: SupCon gradient B operands by dword loads (feature 32 q + n)
#define PCX_AB_SUPCON_DWORD 0
#endif
#ifndef PCX_AB_SUPCON_NOFRAG      // 1: SupCon kernels reload the anchor rows' B fragments per tile
#define PCX_AB_SUPCON_NOFRAG 0
#endif
#ifndef PCX_AB_BN_NO_SPLIT        // 1: one block per channel in the BN finalisers (no split + merge)
#define PCX_AB_BN_NO_SPLIT 0
#endif
