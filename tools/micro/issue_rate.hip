// Micro-benchmark: VALU issue rate of one vs two (vs four) waves per SIMD,
// for f64 FMA, f32 FMA and int adds, independent chains (8 accumulators).
// Answers: does a lone wave issue f64 at the full SIMD rate?
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

template <typename T, int OP>
__global__ void k(T* out, int iters, T a, T b) {
    T acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = (T)(threadIdx.x + j);
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            if constexpr (OP == 0) acc[j] = acc[j] * a + b;      // fma (contracted)
            else acc[j] = acc[j] + b;                             // add
        }
    }
    T s = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) s += acc[j];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <typename T, int OP>
float run(int threads, int iters) {
    T* out;
    hipMalloc(&out, 256 * 1024 * sizeof(T));
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    hipLaunchKernelGGL((k<T, OP>), dim3(256), dim3(threads), 0, 0, out, iters, (T)0.999, (T)1e-3);
    hipDeviceSynchronize();
    hipEventRecord(e0);
    hipLaunchKernelGGL((k<T, OP>), dim3(256), dim3(threads), 0, 0, out, iters, (T)0.999, (T)1e-3);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    hipFree(out);
    return ms;
}

int main() {
    const int iters = 20000;
    const char* names[] = {"f64 fma", "f32 fma", "i32 add", "f64 add"};
    for (int t = 0; t < 4; ++t) {
        for (int threads : {256, 512, 1024}) {  // 1, 2, 4 waves per SIMD (256 blocks: one per CU)
            float ms = t == 0 ? run<double, 0>(threads, iters) : t == 1 ? run<float, 0>(threads, iters)
                     : t == 2 ? run<int, 1>(threads, iters) : run<double, 1>(threads, iters);
            const double waves_per_simd = threads / 256.0;
            const double insts = (double)iters * 8 * waves_per_simd;  // per SIMD
            printf("{\"op\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.4f, \"ns_per_inst_per_simd\": %.4f}\n",
                   names[t], (int)waves_per_simd, ms, ms * 1e6 / insts);
        }
    }
    return 0;
}
