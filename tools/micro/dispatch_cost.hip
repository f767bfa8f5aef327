// Micro-benchmark: what a kernel's resources add to a dependent launch at
// config 3's shape (1,024 workgroups of 256 lanes, hipGraph of 100 launches).
//   empty            : no LDS, 4-byte kernarg
//   empty_lds        : + a 15,360-byte LDS tile (the step kernel's obs tile)
//   empty_karg       : + a 640-byte kernarg struct (the step kernel's StepArgs + Soa)
//   empty_lds_karg   : both
//   copy / copy_lds  : the step's byte pattern (12 dword loads, 10 dword + 15 obs
//                      floats stored), obs rows as strided dwords or staged
//                      through the LDS tile and stored as 16-byte rows
//   *_stamped        : the copy with per-wave entry/exit stamps (span vs outside),
//                      with nt / plain state-like stores, into separate arrays or in place
// Answers: does the obs tile's LDS allocation (or the big kernarg) cost launch
// time, i.e. is the step kernel's ~3 us outside its waves' span the launch?
// (No: it is the kernel-end drain of an in-place update)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <utility>

#define CK(x)                                                                             \
    do {                                                                                  \
        hipError_t e_ = (x);                                                              \
        if (e_ != hipSuccess) {                                                           \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));     \
            exit(1);                                                                      \
        }                                                                                 \
    } while (0)

struct Big {
    uint64_t w[80];  // 640 B
};

__global__ __launch_bounds__(256) void empty_kernel(int n) {
    if (n < 0) __builtin_trap();
}

__global__ __launch_bounds__(256) void empty_lds(int n, float* sink) {
    __shared__ float tile[256 * 15];
    if (n < 0) {
        tile[threadIdx.x] = 1.0f;
        __syncthreads();
        sink[threadIdx.x] = tile[255 - threadIdx.x];
    }
}

__global__ __launch_bounds__(256) void empty_karg(int n, Big b) {
    if (n < 0 && b.w[79] == 7) __builtin_trap();
}

__global__ __launch_bounds__(256) void empty_lds_karg(int n, Big b, float* sink) {
    __shared__ float tile[256 * 15];
    if (n < 0 && b.w[79] == 7) {
        tile[threadIdx.x] = 1.0f;
        __syncthreads();
        sink[threadIdx.x] = tile[255 - threadIdx.x];
    }
}

struct Arrs {
    const float* in[12];
    float* out[10];
    float* obs;
    uint8_t* done;
};

typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ uint64_t tl_buf[4096 * 2];

// kMix: 0 = every store nt (the copy floor); 1 = + a uint8 done stream (nt byte
// stores); 2 = the step kernel's mix: 9 state-like dword streams plain (kept
// dirty in L2), 1 nt, + the nt byte stream
template <bool kLds, bool kStamp = false, int kMix = 0>
__global__ __launch_bounds__(256) void copy_kernel(Arrs a, uint32_t n) {
    __shared__ __attribute__((aligned(16))) float tile[kLds ? 256 * 15 : 4];
    const uint64_t t_entry = kStamp ? __builtin_amdgcn_s_memrealtime() : 0;
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= n) return;
    float v[12];
#pragma unroll
    for (int r = 0; r < 12; ++r) v[r] = a.in[r][i];
    float s = 0.f;
#pragma unroll
    for (int r = 0; r < 12; ++r) s += v[r];
#pragma unroll
    for (int w = 0; w < 10; ++w) {
        if (kMix == 2 && w < 9) a.out[w][i] = s + (float)w;
        else __builtin_nontemporal_store(s + (float)w, &a.out[w][i]);
    }
    if (kMix >= 1) __builtin_nontemporal_store((uint8_t)(s > 1.0f), &a.done[i]);
    if constexpr (kLds) {
        float* row = tile + threadIdx.x * 15;
#pragma unroll
        for (int k = 0; k < 15; ++k) row[k] = s * (float)k;
        __builtin_amdgcn_wave_barrier();
        const int lane = threadIdx.x & 63;
        const uint32_t w0 = blockIdx.x * 256u + (threadIdx.x & ~63u);
        const f32x4* src = reinterpret_cast<const f32x4*>(tile + (threadIdx.x & ~63u) * 15);
        f32x4* dst = reinterpret_cast<f32x4*>(a.obs + (size_t)w0 * 15);
        for (int k = lane; k < 240; k += 64) __builtin_nontemporal_store(src[k], &dst[k]);
    } else {
#pragma unroll
        for (int k = 0; k < 15; ++k) __builtin_nontemporal_store(s * (float)k, &a.obs[(size_t)i * 15 + k]);
    }
    if constexpr (kStamp) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const uint64_t t_exit = __builtin_amdgcn_s_memrealtime();
        const uint32_t w = i / 64;
        if ((threadIdx.x & 63) == 0 && w < 4096) { tl_buf[2 * w] = t_entry; tl_buf[2 * w + 1] = t_exit; }
    }
}

template <typename F>
static float time_graph(hipStream_t st, int launches, F launch) {
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
    for (int k = 0; k < launches; ++k) launch();
    CK(hipStreamEndCapture(st, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    float sum = 0.f;
    const int reps = 12;
    for (int r = 0; r < reps + 2; ++r) {
        CK(hipEventRecord(e0, st));
        CK(hipGraphLaunch(ge, st));
        CK(hipEventRecord(e1, st));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (r >= 2) sum += ms;
    }
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
    return sum / reps * 1e3f / launches;
}

int main(int argc, char** argv) {
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    const int G = 1024;
    float* sink;
    CK(hipMalloc(&sink, 4096));
    Big b{};
    for (int rep = 0; rep < 2; ++rep) {
        printf("{\"case\": \"empty\", \"us\": %.3f}\n",
               time_graph(st, 100, [&] { hipLaunchKernelGGL(empty_kernel, dim3(G), dim3(256), 0, st, G); }));
        printf("{\"case\": \"empty_lds\", \"us\": %.3f}\n",
               time_graph(st, 100, [&] { hipLaunchKernelGGL(empty_lds, dim3(G), dim3(256), 0, st, G, sink); }));
        printf("{\"case\": \"empty_karg\", \"us\": %.3f}\n",
               time_graph(st, 100, [&] { hipLaunchKernelGGL(empty_karg, dim3(G), dim3(256), 0, st, G, b); }));
        printf("{\"case\": \"empty_lds_karg\", \"us\": %.3f}\n",
               time_graph(st, 100, [&] { hipLaunchKernelGGL(empty_lds_karg, dim3(G), dim3(256), 0, st, G, b, sink); }));
        fflush(stdout);
    }
    const uint32_t n = argc > 1 ? (uint32_t)atoi(argv[1]) : 262144u;  // drones (the copy cases)
    const int G2 = (int)(n / 256);
    Arrs a;
    for (int r = 0; r < 12; ++r) {
        float* p;
        CK(hipMalloc(&p, n * 4));
        CK(hipMemset(p, 0, n * 4));
        a.in[r] = p;
    }
    for (int w = 0; w < 10; ++w) CK(hipMalloc(&a.out[w], n * 4));
    CK(hipMalloc(&a.obs, (size_t)n * 60));
    CK(hipMalloc(&a.done, n));
    for (int rep = 0; rep < 2; ++rep) {
        printf("{\"case\": \"copy_strided_obs\", \"us\": %.3f}\n",
               time_graph(st, 100, [&] { hipLaunchKernelGGL((copy_kernel<false>), dim3(G2), dim3(256), 0, st, a, n); }));
        printf("{\"case\": \"copy_lds_obs\", \"us\": %.3f}\n",
               time_graph(st, 100, [&] { hipLaunchKernelGGL((copy_kernel<true>), dim3(G2), dim3(256), 0, st, a, n); }));
        auto stamped = [&](const char* name, auto kern) {
            if (n != 262144u) {  // the stamp buffer covers config 3's 4,096 waves
                printf("{\"case\": \"%s\", \"n\": %u, \"us\": %.3f}\n", name, n,
                       time_graph(st, 20, [&] { hipLaunchKernelGGL(kern, dim3(G2), dim3(256), 0, st, a, n); }));
                fflush(stdout);
                return;
            }
            const float us = time_graph(st, 100, [&] { hipLaunchKernelGGL(kern, dim3(G2), dim3(256), 0, st, a, n); });
            uint64_t tl[4096 * 2];
            CK(hipMemcpyFromSymbol(tl, HIP_SYMBOL(tl_buf), sizeof(tl), 0, hipMemcpyDeviceToHost));
            uint64_t lo = ~0ull, hi = 0;
            for (int w = 0; w < 4096; ++w) {
                lo = tl[2 * w] < lo ? tl[2 * w] : lo;
                hi = tl[2 * w + 1] > hi ? tl[2 * w + 1] : hi;
            }
            const double span = (double)(hi - lo) * 0.01;
            printf("{\"case\": \"%s\", \"us\": %.3f, \"span_us\": %.3f, \"outside_us\": %.3f}\n", name, us,
                   span, us - span);
            fflush(stdout);
        };
        stamped("copy_lds_obs_stamped", copy_kernel<true, true, 0>);
        stamped("copy_lds_obs_done_stamped", copy_kernel<true, true, 1>);
        stamped("copy_lds_obs_stepmix_stamped", copy_kernel<true, true, 2>);
        // in place, as the step is: the 9 state-like streams write the lines they read
        Arrs ip = a;
        for (int w = 0; w < 9; ++w) ip.out[w] = const_cast<float*>(a.in[w]);
        std::swap(a, ip);
        stamped("inplace_nt_stamped", copy_kernel<true, true, 1>);
        stamped("inplace_stepmix_stamped", copy_kernel<true, true, 2>);
        std::swap(a, ip);
        printf("{\"case\": \"copy_lds_obs_stepmix\", \"us\": %.3f}\n",
               time_graph(st, 100, [&] { hipLaunchKernelGGL((copy_kernel<true, false, 2>), dim3(G2), dim3(256), 0, st, a, n); }));
        fflush(stdout);
    }
    return 0;
}
