// Device memory for an env's arrays (dronestep.h dd_device_alloc /
// dd_device_free): host code only.  VecDroneEnv(memory="contiguous") carves
// its SoA fields and per-step outputs from one such range.
#include <hip/hip_runtime.h>

#include "dronestep.h"

extern "C" {

int dd_device_alloc(void** ptr, uint64_t bytes, int32_t flags) {
    if (!ptr || bytes == 0) return hipErrorInvalidValue;
    *ptr = nullptr;
    switch (flags) {
        case DD_MEM_DEFAULT: return (int)hipMalloc(ptr, (size_t)bytes);
        case DD_MEM_CONTIGUOUS: return (int)hipExtMallocWithFlags(ptr, (size_t)bytes, hipDeviceMallocContiguous);
        default: return hipErrorInvalidValue;
    }
}

int dd_device_free(void* ptr) { return ptr ? (int)hipFree(ptr) : 0; }

}  // extern "C"
