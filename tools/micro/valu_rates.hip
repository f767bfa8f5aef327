// Micro-benchmark: issue cost of the VALU instructions the drone frame and
// its re-spawn are made of, on gfx950.  Each kernel runs R rounds of 8
// independent chains per lane of ONE instruction kind (inline asm, so the
// compiler neither folds nor reorders it), at 4 waves per SIMD (the config-3
// step's occupancy) and at 8; the time per round per wave, divided by 8,
// is the instruction's issue cost in SIMD cycles (clock from hipDeviceProp).
//   f64fma  v_fma_f64            (the frame's arithmetic)
//   f64mul  v_mul_f64
//   f32fma  v_fma_f32            (for scale)
//   mad64   v_mad_u64_u32        (Philox rounds: 2 per round)
//   mulhi   v_mul_hi_u32         (draw_range)
//   xor     v_xor_b32            (Philox rounds: 4 per round)
//   cvt     v_cvt_f32_f64        (stores, observation columns)
//   rsq     v_rsq_f64            (square roots)
// Output: one JSON line per (kind, waves per SIMD).
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

enum Kind { F64FMA, F64MUL, F32FMA, MAD64, MULHI, XOR, CVT, RSQ, NKIND };
static const char* kNames[NKIND] = {"f64fma", "f64mul", "f32fma", "mad64", "mulhi", "xor", "cvt", "rsq"};

template <int K>
__global__ __launch_bounds__(256) void bench(int rounds, uint64_t* sink) {
    double d[8];
    float f[8];
    uint32_t u[8];
    uint64_t w[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) {
        d[c] = 1.0 + 1e-3 * (threadIdx.x + c);
        f[c] = 1.0f + 1e-3f * (threadIdx.x + c);
        u[c] = 0x9E3779B9u * (threadIdx.x + c + 1);
        w[c] = u[c];
    }
    const double a = 0.999, b = 1e-4;
    const float af = 0.999f, bf = 1e-4f;
    const uint32_t m = 0xD2511F53u;
    for (int r = 0; r < rounds; ++r) {
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            if constexpr (K == F64FMA) asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(d[c]) : "v"(a), "v"(b));
            if constexpr (K == F64MUL) asm volatile("v_mul_f64 %0, %0, %1" : "+v"(d[c]) : "v"(a));
            if constexpr (K == F32FMA) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(f[c]) : "v"(af), "v"(bf));
            if constexpr (K == MAD64)
                asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(w[c]) : "v"(u[c]), "v"(m) : "vcc");
            if constexpr (K == MULHI) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(u[c]) : "v"(m));
            if constexpr (K == XOR) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(u[c]) : "v"(m));
            if constexpr (K == CVT) {
                float t;
                asm volatile("v_cvt_f32_f64 %0, %1" : "=v"(t) : "v"(d[c]));
                asm volatile("v_cvt_f64_f32 %0, %1" : "=v"(d[c]) : "v"(t));
            }
            if constexpr (K == RSQ) asm volatile("v_rsq_f64 %0, %0" : "+v"(d[c]));
        }
    }
    uint64_t s = 0;
#pragma unroll
    for (int c = 0; c < 8; ++c) s += __double_as_longlong(d[c]) ^ __float_as_uint(f[c]) ^ u[c] ^ w[c];
    if (s == 0x1234567) sink[threadIdx.x] = s;
}

template <int K>
static float run(int waves_per_simd, int rounds, uint64_t* sink, int cus) {
    const int blocks = cus * waves_per_simd;  // 4 waves per block: one per SIMD
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    bench<K><<<blocks, 256>>>(rounds, sink);
    CK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int rep = 0; rep < 5; ++rep) {
        CK(hipEventRecord(e0));
        bench<K><<<blocks, 256>>>(rounds, sink);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        best = ms < best ? ms : best;
    }
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
    return best;
}

int main() {
    hipDeviceProp_t p;
    CK(hipGetDeviceProperties(&p, 0));
    const int cus = p.multiProcessorCount;
    const double ghz = p.clockRate / 1e6;
    uint64_t* sink;
    CK(hipMalloc(&sink, 256 * sizeof(uint64_t)));
    const int rounds = 20000;
    float (*fns[NKIND])(int, int, uint64_t*, int) = {run<F64FMA>, run<F64MUL>, run<F32FMA>, run<MAD64>,
                                                     run<MULHI>,  run<XOR>,    run<CVT>,    run<RSQ>};
    for (int k = 0; k < NKIND; ++k) {
        for (int wps : {4, 8}) {
            const float ms = fns[k](wps, rounds, sink, cus);
            // per SIMD: wps waves x rounds x 8 instructions (CVT: 2 per chain step)
            const double instr = (double)wps * rounds * 8 * (k == CVT ? 2 : 1);
            const double cyc = ms * 1e-3 * ghz * 1e9 / instr;
            printf("{\"kind\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.4f, \"cycles_per_instr_per_simd\": %.3f, "
                   "\"clock_ghz_nominal\": %.3f}\n",
                   kNames[k], wps, ms, cyc, ghz);
        }
    }
    CK(hipFree(sink));
    return 0;
}
