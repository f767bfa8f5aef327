// Micro-benchmark: what one instruction costs a LONE wave on its SIMD (the
// config-5 rollout's situation: 65,536 drones = one wave per SIMD), by
// instruction, for independent streams (8 accumulators, issue cost) and for
// one dependent chain (latency).  One 256-thread block per CU = one wave per
// SIMD; every block runs `iters` x 16 copies of the instruction.  The row
// "v_add_u32" is the 1-issue-slot reference; costs print as ns and as slots
// relative to it (so the clock drops out).
//
//   hipcc --offload-arch=gfx950 -O3 -o valu_cost valu_cost.hip && ./valu_cost
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

// independent: 8 registers, each op reads and writes its own
#define K_IND(name, T, ASM, CONS, ...)                                                             \
    __global__ void name(T* out, int iters) {                                                 \
        T r0 = (T)threadIdx.x, r1 = r0 + 1, r2 = r0 + 2, r3 = r0 + 3, r4 = r0 + 4, r5 = r0 + 5, \
          r6 = r0 + 6, r7 = r0 + 7;                                                           \
        const T c = (T)3;                                                                     \
        for (int i = 0; i < iters; ++i) {                                                     \
            _Pragma("unroll") for (int k = 0; k < 2; ++k) {                                   \
                asm volatile(ASM : "+" CONS(r0) : CONS(c) __VA_ARGS__);                                   \
                asm volatile(ASM : "+" CONS(r1) : CONS(c) __VA_ARGS__);                                   \
                asm volatile(ASM : "+" CONS(r2) : CONS(c) __VA_ARGS__);                                   \
                asm volatile(ASM : "+" CONS(r3) : CONS(c) __VA_ARGS__);                                   \
                asm volatile(ASM : "+" CONS(r4) : CONS(c) __VA_ARGS__);                                   \
                asm volatile(ASM : "+" CONS(r5) : CONS(c) __VA_ARGS__);                                   \
                asm volatile(ASM : "+" CONS(r6) : CONS(c) __VA_ARGS__);                                   \
                asm volatile(ASM : "+" CONS(r7) : CONS(c) __VA_ARGS__);                                   \
            }                                                                                 \
        }                                                                                     \
        out[blockIdx.x * blockDim.x + threadIdx.x] = r0 + r1 + r2 + r3 + r4 + r5 + r6 + r7;   \
    }
// dependent: one register, 16 ops in a chain
#define K_DEP(name, T, ASM, CONS, ...)                                            \
    __global__ void name(T* out, int iters) {                                \
        T r0 = (T)threadIdx.x;                                               \
        const T c = (T)3;                                                    \
        for (int i = 0; i < iters; ++i) {                                    \
            _Pragma("unroll") for (int k = 0; k < 16; ++k) asm volatile(ASM : "+" CONS(r0) : CONS(c) __VA_ARGS__); \
        }                                                                    \
        out[blockIdx.x * blockDim.x + threadIdx.x] = r0;                     \
    }

#define V(x) "v"(x)
#define S(x) "s"(x)

K_IND(i_add_u32, uint32_t, "v_add_u32 %0, %0, %1", V)
K_IND(i_and_b32, uint32_t, "v_and_b32 %0, %0, %1", V)
K_IND(i_bfe_u32, uint32_t, "v_bfe_u32 %0, %0, %1, 3", V)
K_IND(i_add_f32, float, "v_add_f32 %0, %0, %1", V)
K_IND(i_fma_f32, float, "v_fma_f32 %0, %0, %1, %1", V)
K_IND(i_cnd_b32, uint32_t, "v_cndmask_b32 %0, %0, %1, vcc", V)
K_IND(i_cnd_e64_s, uint32_t, "v_cndmask_b32_e64 %0, %0, %1, s[2:3]", V, : "s2", "s3")
K_IND(i_cnd_k, uint32_t, "v_cndmask_b32 %0, 0, %0, vcc", V)
K_IND(i_cmp_cnd, uint32_t, "v_cmp_lt_u32 vcc, %0, %1\n v_cndmask_b32 %0, %0, %1, vcc", V, : "vcc")
K_IND(i_cmp_u32, uint32_t, "v_cmp_lt_u32 vcc, %0, %1", V, : "vcc")
K_IND(i_cmp_e64, uint32_t, "v_cmp_lt_u32_e64 s[2:3], %0, %1", V, : "s2", "s3")
K_IND(i_bfi_b32, uint32_t, "v_bfi_b32 %0, %1, %0, %1", V)
// a predicate and the double select it drives, as the frame's code has them
// (32-bit halves as separate registers: lo = %0, hi = %1, other = %2 / %3)
#define K_PAIR(name, ASM, ...)                                                                \
    __global__ void name(uint32_t* out, int iters) {                                          \
        uint32_t l[8], h[8];                                                                  \
        _Pragma("unroll") for (int j = 0; j < 8; ++j) { l[j] = threadIdx.x + j; h[j] = j; }   \
        const uint32_t cl = 3, ch = 5;                                                        \
        for (int i = 0; i < iters; ++i) {                                                     \
            _Pragma("unroll") for (int k = 0; k < 2; ++k) {                                   \
                _Pragma("unroll") for (int j = 0; j < 8; ++j)                                 \
                    asm volatile(ASM : "+v"(l[j]), "+v"(h[j]) : "v"(cl), "v"(ch) __VA_ARGS__);  \
            }                                                                                 \
        }                                                                                     \
        uint32_t t = 0;                                                                       \
        _Pragma("unroll") for (int j = 0; j < 8; ++j) t += l[j] ^ h[j];                       \
        out[blockIdx.x * blockDim.x + threadIdx.x] = t;                                       \
    }
K_PAIR(p_cmp_cnd2_vcc, "v_cmp_lt_u32 vcc, %0, %2\n v_cndmask_b32 %0, %0, %2, vcc\n v_cndmask_b32 %1, %1, %3, vcc", : "vcc")
K_PAIR(p_cmp_cnd2_s, "v_cmp_lt_u32_e64 s[4:5], %0, %2\n v_cndmask_b32_e64 %0, %0, %2, s[4:5]\n v_cndmask_b32_e64 %1, %1, %3, s[4:5]", : "s4", "s5")
K_PAIR(p_cmp_cnd4_vcc, "v_cmp_lt_u32 vcc, %0, %2\n v_cndmask_b32 %0, %0, %2, vcc\n v_cndmask_b32 %1, %1, %3, vcc\n v_cndmask_b32 %0, %2, %0, vcc\n v_cndmask_b32 %1, %3, %1, vcc", : "vcc")
K_PAIR(p_cmp_cnd4_s, "v_cmp_lt_u32_e64 s[4:5], %0, %2\n v_cndmask_b32_e64 %0, %0, %2, s[4:5]\n v_cndmask_b32_e64 %1, %1, %3, s[4:5]\n v_cndmask_b32_e64 %0, %2, %0, s[4:5]\n v_cndmask_b32_e64 %1, %3, %1, s[4:5]", : "s4", "s5")
K_PAIR(p_mask_bfi2, "v_cmp_lt_u32 vcc, %0, %2\n v_cndmask_b32 v250, 0, -1, vcc\n v_bfi_b32 %0, v250, %0, %2\n v_bfi_b32 %1, v250, %1, %3", : "vcc", "v250")
K_PAIR(p_and2, "v_cmp_lt_u32 vcc, %0, %2\n v_cndmask_b32 v250, 0, -1, vcc\n v_and_b32 %0, v250, %0\n v_and_b32 %1, v250, %1", : "vcc", "v250")
K_PAIR(p_sub_mask_and2, "v_sub_u32 v250, %0, %2\n v_ashrrev_i32 v250, 31, v250\n v_and_b32 %0, v250, %0\n v_and_b32 %1, v250, %1", : "v250")
K_IND(i_mov_b32, uint32_t, "v_mov_b32 %0, %1", V)
K_IND(i_xor_b32, uint32_t, "v_xor_b32 %0, %0, %1", V)
K_IND(i_lshl_b32, uint32_t, "v_lshlrev_b32 %0, 3, %0", V)
K_IND(i_med3_f32, float, "v_med3_f32 %0, %0, %1, %1", V)
K_IND(i_readlane, uint32_t, "v_readlane_b32 s2, %0, 5\n v_add_u32 %0, s2, %0", V, : "s2")
K_IND(i_mul_hi_u32, uint32_t, "v_mul_hi_u32 %0, %0, %1", V)
K_IND(i_fma_f64, double, "v_fma_f64 %0, %0, %1, %1", V)
K_IND(i_add_f64, double, "v_add_f64 %0, %0, %1", V)
K_IND(i_mul_f64, double, "v_mul_f64 %0, %0, %1", V)
K_IND(i_min_f64, double, "v_min_f64 %0, %0, %1", V)
K_IND(i_ldexp_f64, double, "v_ldexp_f64 %0, %0, 1", V)
K_IND(i_rndne_f64, double, "v_rndne_f64 %0, %0", V)
K_IND(i_cvt_f32_f64, double, "v_cvt_f32_f64 v250, %0\n v_cvt_f64_f32 %0, v250", V, : "v250")  // the pair (quantize)
K_IND(i_cvt_f64_f32_only, float, "v_cvt_f64_f32 v[250:251], %0", V, : "v250", "v251")
K_IND(i_cvt_f32_f64_only, double, "v_cvt_f32_f64 v250, %0", V, : "v250")
K_IND(i_cvt_i32_f64, double, "v_cvt_i32_f64 v250, %0", V, : "v250")
K_IND(i_fmac_lit, double, "v_fmac_f64 %0, 0x40490000, %1", V)
K_IND(i_class_f64, double, "v_cmp_class_f64 vcc, %0, 3", V, : "vcc")
K_IND(i_rsq_f64, double, "v_rsq_f64 %0, %0", V)
K_IND(i_cmp_f64, double, "v_cmp_lt_f64 vcc, %0, %1", V, : "vcc")
K_IND(i_mad_u64_u32, uint64_t, "v_mad_u64_u32 %0, vcc, 3, 5, %0", V, : "vcc")
K_IND(i_pk_fma_f32, double, "v_pk_fma_f32 %0, %0, %1, %1", V)
// scalar: the same shape on SGPRs (uniform values)
#define K_SCA(name, ASM)                                                                      \
    __global__ void name(uint32_t* out, int iters) {                                          \
        uint32_t r0 = blockIdx.x, r1 = r0 + 1, r2 = r0 + 2, r3 = r0 + 3;                      \
        for (int i = 0; i < iters; ++i) {                                                     \
            _Pragma("unroll") for (int k = 0; k < 4; ++k) {                                   \
                asm volatile(ASM : "+s"(r0));                                                 \
                asm volatile(ASM : "+s"(r1));                                                 \
                asm volatile(ASM : "+s"(r2));                                                 \
                asm volatile(ASM : "+s"(r3));                                                 \
            }                                                                                 \
        }                                                                                     \
        out[blockIdx.x * blockDim.x + threadIdx.x] = r0 + r1 + r2 + r3;                       \
    }
K_SCA(i_s_mov, "s_mov_b32 %0, 0x12345")
K_SCA(i_s_add, "s_bitset1_b32 %0, 5")
K_SCA(i_s_nop, "s_nop 0")
K_DEP(d_add_u32, uint32_t, "v_add_u32 %0, %0, %1", V)
K_DEP(d_add_f32, float, "v_add_f32 %0, %0, %1", V)
K_DEP(d_fma_f64, double, "v_fma_f64 %0, %0, %1, %1", V)
K_DEP(d_add_f64, double, "v_add_f64 %0, %0, %1", V)
K_DEP(d_mul_f64, double, "v_mul_f64 %0, %0, %1", V)
K_DEP(d_cvt_pair, double, "v_cvt_f32_f64 v250, %0\n v_cvt_f64_f32 %0, v250", V, : "v250")
K_DEP(d_rsq_f64, double, "v_rsq_f64 %0, %0", V)

template <typename T>
float run(void (*k)(T*, int), int iters, int threads) {
    T* out;
    hipMalloc(&out, 256 * 1024 * sizeof(T));
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipLaunchKernelGGL(k, dim3(256), dim3(threads), 0, 0, out, iters);
    hipDeviceSynchronize();
    float best = 1e30f;
    for (int rep = 0; rep < 3; ++rep) {
        hipEventRecord(e0);
        hipLaunchKernelGGL(k, dim3(256), dim3(threads), 0, 0, out, iters);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        best = ms < best ? ms : best;
    }
    hipFree(out);
    return best;
}

int main() {
    const int iters = 20000;
    struct Row { const char* name; float ms1, ms2; int per_op; };
    double ref = 0;
#define RUN(k, T, n)                                                                                 \
    {                                                                                                \
        const float a = run<T>(k, iters, 256), b = run<T>(k, iters, 512);                            \
        const double ns = a * 1e6 / (iters * 16.0 * (n));                                            \
        const double ns2 = b * 1e6 / (iters * 16.0 * (n) * 2);                                      \
        if (ref == 0) ref = ns;                                                                      \
        printf("{\"op\": \"%s\", \"ns_per_op_1wave\": %.4f, \"slots_vs_add_u32\": %.3f, "           \
               "\"ns_per_op_per_simd_2waves\": %.4f}\n", #k, ns, ns / ref, ns2);                     \
    }
    RUN(i_add_u32, uint32_t, 1)
    RUN(i_and_b32, uint32_t, 1)
    RUN(i_bfe_u32, uint32_t, 1)
    RUN(i_add_f32, float, 1)
    RUN(i_fma_f32, float, 1)
    RUN(i_cnd_b32, uint32_t, 1)
    RUN(i_cnd_e64_s, uint32_t, 1)
    RUN(i_cnd_k, uint32_t, 1)
    RUN(i_cmp_cnd, uint32_t, 2)
    RUN(i_cmp_u32, uint32_t, 1)
    RUN(i_cmp_e64, uint32_t, 1)
    RUN(i_bfi_b32, uint32_t, 1)
    RUN(p_cmp_cnd2_vcc, uint32_t, 3)
    RUN(p_cmp_cnd2_s, uint32_t, 3)
    RUN(p_cmp_cnd4_vcc, uint32_t, 5)
    RUN(p_cmp_cnd4_s, uint32_t, 5)
    RUN(p_mask_bfi2, uint32_t, 4)
    RUN(p_and2, uint32_t, 4)
    RUN(p_sub_mask_and2, uint32_t, 4)
    RUN(i_mov_b32, uint32_t, 1)
    RUN(i_xor_b32, uint32_t, 1)
    RUN(i_lshl_b32, uint32_t, 1)
    RUN(i_med3_f32, float, 1)
    RUN(i_readlane, uint32_t, 2)
    RUN(i_mul_hi_u32, uint32_t, 1)
    RUN(i_fma_f64, double, 1)
    RUN(i_add_f64, double, 1)
    RUN(i_mul_f64, double, 1)
    RUN(i_min_f64, double, 1)
    RUN(i_ldexp_f64, double, 1)
    RUN(i_rndne_f64, double, 1)
    RUN(i_cvt_f32_f64, double, 2)
    RUN(i_cvt_f64_f32_only, float, 1)
    RUN(i_cvt_f32_f64_only, double, 1)
    RUN(i_cvt_i32_f64, double, 1)
    RUN(i_fmac_lit, double, 1)
    RUN(i_class_f64, double, 1)
    RUN(i_rsq_f64, double, 1)
    RUN(i_cmp_f64, double, 1)
    RUN(i_mad_u64_u32, uint64_t, 1)
    RUN(i_pk_fma_f32, double, 1)
    RUN(i_s_mov, uint32_t, 1)
    RUN(i_s_add, uint32_t, 1)
    RUN(i_s_nop, uint32_t, 1)
    RUN(d_add_u32, uint32_t, 1)
    RUN(d_add_f32, float, 1)
    RUN(d_fma_f64, double, 1)
    RUN(d_add_f64, double, 1)
    RUN(d_mul_f64, double, 1)
    RUN(d_cvt_pair, double, 2)
    RUN(d_rsq_f64, double, 1)
    return 0;
}
