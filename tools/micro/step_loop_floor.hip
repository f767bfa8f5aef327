// Micro-benchmark: the floor of config 5 variant (a) (bench.py step_loop_point:
// one dd_step launch per frame into the [T, N] rollout buffers, 256 launches
// in one hipGraph) — the same launches and bytes with no frame arithmetic.
// Launch f of 256, N lanes (65,536), 256-lane blocks:
//   reads : 10 f32 state fields + status (u8) + steps (i32), in place, and
//           the frame's action byte acts[f][i]                   (46 B)
//   writes: 7 dynamics fields + total + steps (in place), reward[f][i] (f32),
//           done[f][i] (u8), obs[f][i][15] staged through a per-wave LDS
//           slice and stored as 16-byte non-temporal rows          (101 B)
// 147 B per lane-frame, as dd_step with obs.  Prints one JSON line per
// repetition: us per launch (graph replays timed with HIP events).
//   ./step_loop_floor [lanes=65536] [frames=256] [reps=5]
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

typedef float f32x4 __attribute__((ext_vector_type(4)));

struct State {
    float* f[10];  // x y vx vy angle omega fuel px py total
    uint8_t* status;
    int32_t* steps;
};

__global__ __launch_bounds__(256) void frame_copy(State s, const uint8_t* act, float* reward, uint8_t* done,
                                                  float* obs, uint32_t n) {
    __shared__ __attribute__((aligned(16))) float tile[256 * 15];
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    const int lane = threadIdx.x & 63, w0 = threadIdx.x & ~63;
    float v[10];
    uint32_t a = 0, st = 0;
    int32_t steps = 0;
    if (i < n) {
        a = act[i];
#pragma unroll
        for (int k = 0; k < 10; ++k) v[k] = s.f[k][i];
        st = s.status[i];
        steps = s.steps[i];
    }
    float acc = (float)(a + st);
#pragma unroll
    for (int k = 0; k < 10; ++k) acc += v[k];
    if (i < n) {
#pragma unroll
        for (int k = 0; k < 7; ++k) s.f[k][i] = v[k] + 1e-7f * acc;  // the 7 dynamics fields
        s.f[9][i] = v[9] + acc;                                       // total
        s.steps[i] = steps + 1;
        __builtin_nontemporal_store(acc, &reward[i]);
        __builtin_nontemporal_store((uint8_t)(st & 1u), &done[i]);
    }
    float* row = tile + threadIdx.x * 15;
#pragma unroll
    for (int k = 0; k < 15; ++k) row[k] = acc * (float)k;
    __syncwarp();
    const uint32_t wrow0 = blockIdx.x * 256 + w0;
    if (wrow0 < n) {
        const int rows = (int)min(64u, n - wrow0);
        const int nv = rows * 15 / 4;
        const f32x4* src = reinterpret_cast<const f32x4*>(tile + w0 * 15);
        f32x4* dst = reinterpret_cast<f32x4*>(obs + (size_t)wrow0 * 15);
        for (int k = lane; k < nv; k += 64) __builtin_nontemporal_store(src[k], &dst[k]);
    }
}

int main(int argc, char** argv) {
    const uint32_t n = argc > 1 ? (uint32_t)atoi(argv[1]) : 65536u;
    const int frames = argc > 2 ? atoi(argv[2]) : 256;
    const int reps = argc > 3 ? atoi(argv[3]) : 5;
    if (n == 0 || n % 64 || frames <= 0) {
        fprintf(stderr, "lanes must be a positive multiple of 64, frames positive\n");
        return 2;
    }
    State s;
    for (int k = 0; k < 10; ++k) {
        CK(hipMalloc(&s.f[k], n * 4));
        CK(hipMemset(s.f[k], 0, n * 4));
    }
    CK(hipMalloc(&s.status, n));
    CK(hipMemset(s.status, 0, n));
    CK(hipMalloc(&s.steps, n * 4));
    CK(hipMemset(s.steps, 0, n * 4));
    uint8_t *act, *done;
    float *reward, *obs;
    CK(hipMalloc(&act, (size_t)frames * n));
    CK(hipMemset(act, 3, (size_t)frames * n));
    CK(hipMalloc(&done, (size_t)frames * n));
    CK(hipMalloc(&reward, (size_t)frames * n * 4));
    CK(hipMalloc(&obs, (size_t)frames * n * 60));
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
    for (int f = 0; f < frames; ++f)
        hipLaunchKernelGGL(frame_copy, dim3(n / 256 + (n % 256 ? 1 : 0)), dim3(256), 0, st, s, act + (size_t)f * n,
                           reward + (size_t)f * n, done + (size_t)f * n, obs + (size_t)f * n * 15, n);
    CK(hipStreamEndCapture(st, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipGraphLaunch(ge, st));
    CK(hipStreamSynchronize(st));
    for (int r = 0; r < reps; ++r) {
        CK(hipEventRecord(e0, st));
        CK(hipGraphLaunch(ge, st));
        CK(hipEventRecord(e1, st));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        const double us = ms * 1e3 / frames;
        printf("{\"case\": \"step_loop_floor\", \"lanes\": %u, \"frames\": %d, \"rep\": %d, \"us_per_launch\": %.3f, "
               "\"bytes_per_lane_frame\": 147, \"GB_per_s\": %.1f}\n",
               n, frames, r, us, 147.0 * n / (us * 1e-6) / 1e9);
        fflush(stdout);
    }
    return 0;
}
