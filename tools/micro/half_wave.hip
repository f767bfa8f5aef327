// Micro-benchmark: does a wave64 VALU instruction with only half of its lanes
// enabled cost less than a full one on gfx950, and what does a lone wave per
// SIMD lose to issue latency?  Dependent f64 FMA chains (CH independent chains
// per lane, R rounds), 256-lane blocks.
//   full1  : 1,024 waves (one per SIMD), 64 lanes active
//   half1  : 1,024 waves, lanes 0-31 active (exec half)
//   half2  : 2,048 waves (two per SIMD), lanes 0-31 active: full1's lane-work
//   full2  : 2,048 waves, 64 lanes active
// Question behind it: dd_rollout at 65,536 drones is one wave per SIMD; would
// 32 drones per wave (twice the waves) run faster?
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

template <typename T, int CH>
__global__ __launch_bounds__(256) void chains(int rounds, int active_lanes, T* sink) {
    const int lane = threadIdx.x & 63;
    if (lane >= active_lanes) return;
    T v[CH];
#pragma unroll
    for (int c = 0; c < CH; ++c) v[c] = (T)(threadIdx.x + c) * (T)1e-3;
    const T a = (T)0.999, b = (T)1e-4;
    for (int r = 0; r < rounds; ++r) {
#pragma unroll
        for (int c = 0; c < CH; ++c) v[c] = v[c] * a + b;
    }
    T s = 0;
#pragma unroll
    for (int c = 0; c < CH; ++c) s += v[c];
    if (s == (T)12345) sink[threadIdx.x] = s;
}

template <typename K>
static float time_it(K launch) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    float best = 1e30f;
    for (int r = 0; r < 7; ++r) {
        CK(hipEventRecord(e0, 0));
        launch();
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (r >= 2 && ms < best) best = ms;
    }
    return best * 1e3f;
}

template <typename T, int CH>
static void run(const char* dt) {
    T* sink;
    CK(hipMalloc(&sink, 4096 * sizeof(T)));
    const int R = 4000;
    struct C { const char* name; int waves, lanes; } cs[] = {
        {"full1", 1024, 64}, {"half1", 1024, 32}, {"half2", 2048, 32}, {"full2", 2048, 64}, {"half4", 4096, 32}, {"full4", 4096, 64}};
    for (auto& c : cs) {
        const float us = time_it([&] { hipLaunchKernelGGL((chains<T, CH>), dim3(c.waves / 4), dim3(256), 0, 0, R, c.lanes, sink); });
        printf("{\"dtype\": \"%s\", \"chains\": %d, \"case\": \"%s\", \"waves\": %d, \"lanes\": %d, \"rounds\": %d, \"us\": %.2f, "
               "\"ns_per_fma_per_wave\": %.3f}\n", dt, CH, c.name, c.waves, c.lanes, R, us, us * 1e3f / (R * CH));
        fflush(stdout);
    }
    CK(hipFree(sink));
}

int main() {
    run<double, 1>("f64");
    run<double, 4>("f64");
    run<float, 1>("f32");
    run<float, 4>("f32");
    return 0;
}
