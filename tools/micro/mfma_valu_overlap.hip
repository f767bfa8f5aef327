// Micro-benchmark: can one SIMD run an MFMA-only wave and a VALU-only wave at
// the same time?  One block of 8 waves per CU (2 per SIMD; a 96 KB LDS
// allocation keeps it to one block), 256 blocks.  Waves 0-3 (one per SIMD)
// run `m` rounds of v_mfma_f32_32x32x16_f16 on 4 independent accumulators;
// waves 4-7 run `v` rounds of 8 independent v_pk_fma_f32.  Cases: MFMA only,
// VALU only, both (concurrent), and both in one wave (interleaved).  The
// question behind it: the f16x3 actor (policy_mlp.hip) spends as long as its
// VALU and MFMA issue times added up, not the longer of the two.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x)                                                                         \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                  \
        }                                                                             \
    } while (0)

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ void mfma_work(int m, float* sink, int lane) {
    f16x8 a = {(_Float16)1, (_Float16)lane, 0, 0, 0, 0, 0, (_Float16)0.5f};
    f16x8 b = a;
    f32x16 acc[4] = {};
    for (int i = 0; i < m; ++i) {
#pragma unroll
        for (int t = 0; t < 4; ++t) acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, acc[t], 0, 0, 0);
    }
    float s = 0.f;
#pragma unroll
    for (int t = 0; t < 4; ++t) s += acc[t][0] + acc[t][15];
    if (s == 1234.5f) sink[lane] = s;
}

__device__ __forceinline__ void valu_work(int v, float* sink, int lane) {
    f32x2 x[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] = f32x2{(float)lane * 1e-3f + j, 1.0f - j};
    const f32x2 c = {0.999f, 0.999f}, d = {1e-4f, 2e-4f};
    for (int i = 0; i < v; ++i) {
#pragma unroll
        for (int j = 0; j < 8; ++j) x[j] = __builtin_elementwise_fma(x[j], c, d);
    }
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) s += x[j].x + x[j].y;
    if (s == 1234.5f) sink[lane] = s;
}

// mfma_work with s_nops between the MFMAs (each MFMA issues to an idle pipe:
// does a wave stalled on a busy matrix pipe block the SIMD's issue for its
// partner wave?).
template <int NOPS>
__device__ __forceinline__ void mfma_gap_work(int m, float* sink, int lane) {
    f16x8 a = {(_Float16)1, (_Float16)lane, 0, 0, 0, 0, 0, (_Float16)0.5f};
    f16x8 b = a;
    f32x16 acc[4] = {};
    for (int i = 0; i < m; ++i) {
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, acc[t], 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (NOPS >= 1) asm volatile("s_nop 7");
            if constexpr (NOPS >= 2) asm volatile("s_nop 7");
            if constexpr (NOPS >= 3) asm volatile("s_nop 7");
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    float s = 0.f;
#pragma unroll
    for (int t = 0; t < 4; ++t) s += acc[t][0] + acc[t][15];
    if (s == 1234.5f) sink[lane] = s;
}

// The same VALU work as 16 independent scalar v_fma_f32 chains.
__device__ __forceinline__ void valu_scalar_work(int v, float* sink, int lane) {
    float x[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) x[j] = (float)lane * 1e-3f + j;
    for (int i = 0; i < v; ++i) {
#pragma unroll
        for (int j = 0; j < 16; ++j) x[j] = __builtin_fmaf(x[j], 0.999f, (j & 1) ? 2e-4f : 1e-4f);
    }
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < 16; ++j) s += x[j];
    if (s == 1234.5f) sink[lane] = s;
}

// The MFMA and VALU work of one wave in one loop: each round 4 independent
// MFMAs with vpr x 8 independent packed FMAs placed between them
// (sched_group_barrier: 1 MFMA, 2 * vpr VALU, four times).
template <int VPR>
__device__ __forceinline__ void mixed_work(int m, float* sink, int lane) {
    f16x8 a = {(_Float16)1, (_Float16)lane, 0, 0, 0, 0, 0, (_Float16)0.5f};
    f16x8 b = a;
    f32x16 acc[4] = {};
    f32x2 x[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] = f32x2{(float)lane * 1e-3f + j, 1.0f - j};
    const f32x2 c = {0.999f, 0.999f}, d = {1e-4f, 2e-4f};
    for (int i = 0; i < m; ++i) {
#pragma unroll
        for (int t = 0; t < 4; ++t) acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, acc[t], 0, 0, 0);
#pragma unroll
        for (int q = 0; q < VPR; ++q) {
#pragma unroll
            for (int j = 0; j < 8; ++j) x[j] = __builtin_elementwise_fma(x[j], c, d);
        }
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);        // one MFMA
            __builtin_amdgcn_sched_group_barrier(0x002, 2 * VPR, 0);  // its share of the VALU
        }
    }
    float s = 0.f;
#pragma unroll
    for (int t = 0; t < 4; ++t) s += acc[t][0] + acc[t][15];
#pragma unroll
    for (int j = 0; j < 8; ++j) s += x[j].x + x[j].y;
    if (s == 1234.5f) sink[lane] = s;
}

// mode 0: MFMA waves only; 1: VALU waves only; 2: both, in different waves;
// 3: both in the same waves (waves 0-3 do MFMA then VALU in one stream);
// 4: VALU waves only, as scalar v_fma_f32; 5 / 6: packed / scalar VALU in all 8 waves;
// 7 / 8: interleaved (packed) in one wave / both waves of a SIMD;
// 9: MFMA waves and scalar-VALU waves (different waves of a SIMD: does
// scalar f32 VALU, unlike packed, run beside another wave's MFMAs?);
// 10: mfma_gap_work<3> waves alone; 11: mfma_gap_work<3> waves and scalar-VALU waves;
// 12 / 13: the same with one s_nop 7 per MFMA (the pipe stays about busy)
__global__ __launch_bounds__(512) void k(int mode, int m, int v, float* sink) {
    extern __shared__ float big[];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (m < 0) big[threadIdx.x] = 1.f;  // the LDS allocation is what matters
    if (wave < 4) {
        if (mode == 0 || mode == 2 || mode == 3) mfma_work(m, sink, lane);
        if (mode == 3) valu_work(v, sink, lane);
    } else {
        if (mode == 1 || mode == 2) valu_work(v, sink, lane);
        if (mode == 4) valu_scalar_work(v, sink, lane);
        if (mode == 5) valu_work(v, sink, lane);
        if (mode == 9 || mode == 11 || mode == 13) valu_scalar_work(v, sink, lane);
    }
    if (mode == 9 && wave < 4) mfma_work(m, sink, lane);
    if ((mode == 10 || mode == 11) && wave < 4) mfma_gap_work<3>(m, sink, lane);
    if ((mode == 12 || mode == 13) && wave < 4) mfma_gap_work<1>(m, sink, lane);
    if (mode == 5 && wave < 4) valu_work(v, sink, lane);   // packed, both waves of a SIMD
    if (mode == 6) valu_scalar_work(v, sink, lane);         // scalar, both waves of a SIMD
    if ((mode == 7 && wave < 4) || mode == 8) {  // interleaved in one wave (7) / in both waves of a SIMD (8)
        if (v == m) mixed_work<1>(m, sink, lane);
        else if (v == 2 * m) mixed_work<2>(m, sink, lane);
        else mixed_work<4>(m, sink, lane);
    }
}

int main() {
    float* sink;
    CK(hipMalloc(&sink, 4096));
    CK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int m = 2000, vs[] = {2000, 4000, 8000};
    for (int vi = 0; vi < 3; ++vi) {
        const int v = vs[vi];
        for (int mode = 0; mode < 14; ++mode) {
            float best = 1e30f;
            for (int r = 0; r < 5; ++r) {
                CK(hipEventRecord(e0));
                hipLaunchKernelGGL(k, dim3(256), dim3(512), 96 * 1024, 0, mode, m, v, sink);
                CK(hipEventRecord(e1));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                best = ms < best ? ms : best;
            }
            printf("{\"mode\": %d, \"mfma_rounds\": %d, \"valu_rounds\": %d, \"us\": %.2f}\n", mode,
                   mode == 1 ? 0 : m, mode == 0 ? 0 : v, best * 1e3f);
        }
    }
    return 0;
}
