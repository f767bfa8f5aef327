// clock_probe.hip — the shader clock at one moment of a stream, for labs that
// ask whether a kernel's time moves with the chip's clock (DVFS) rather than
// with its own work (MI355X_MICROARCH "DVFS give-back", item 6).  One wave
// runs a fixed chain of dependent f32 FMAs between two stamps of the shader
// clock (s_memtime) and the 100 MHz real-time clock (s_memrealtime); the
// clock is their ratio x 100 MHz.  Launched between the kernels under test
// (same stream), it measures the clock the chip holds there.
//   hipcc --offload-arch=gfx950 -O3 -shared -fPIC -o tools/micro/libclock_probe.so tools/micro/clock_probe.hip
#include <hip/hip_runtime.h>
#include <stdint.h>

__global__ void clock_probe_kernel(uint64_t* out, int iters) {
    float x = (float)threadIdx.x;
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    const uint64_t r0 = __builtin_amdgcn_s_memrealtime();
    for (int i = 0; i < iters; ++i) asm volatile("v_fma_f32 %0, %0, %0, %0" : "+v"(x));
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    const uint64_t r1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) {
        out[0] = t1 - t0;
        out[1] = r1 - r0;
        out[2] = (uint64_t)__float_as_uint(x);
    }
}

extern "C" int clock_probe(void* out, int iters, void* stream) {
    hipLaunchKernelGGL(clock_probe_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, (uint64_t*)out, iters);
    return (int)hipGetLastError();
}
