// philox.h — Philox4x32 (Salmon et al., SC'11), the counter-based
// generator behind every random draw on the device: spawns (7 rounds, since
// round 6) are keyed by (seed; global env id, episode, 0), in-kernel random
// actions (10 rounds) by
// (seed; env id, step >> 5, 0xA5A5A5A5 ^ (step >> 5)_hi), one block per 32
// steps (drone_step.hip rollout_action), policy samples by
// (seed; env id, step, 0x5A5A5A5A ^ step_hi) (10 rounds).  Keyed by the global env id, a
// lane's draws do not depend on sharding or launch geometry.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dd {

// Philox4x32-R; R = 10 is Random123's default.  kR = 7 (philox4x32_7) is the
// fewest rounds Salmon et al. found Crush-resistant (BigCrush passes with 7,
// fails with 6; 10 keeps a margin of 3): the re-spawn stream, whose four draws
// per (env, episode) sit in the step kernel's rarest but costliest branch.
template <int kR>
__device__ __forceinline__ void philox4x32_r(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0,
                                             uint32_t k1, uint32_t out[4]) {
#pragma unroll
    for (int r = 0; r < kR; ++r) {
        const uint64_t p0 = (uint64_t)0xD2511F53u * c0;
        const uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
        const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
        const uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
        c1 = (uint32_t)p1;
        c3 = (uint32_t)p0;
        c0 = n0;
        c2 = n2;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

__device__ __forceinline__ void philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0,
                                              uint32_t k1, uint32_t out[4]) {
    philox4x32_r<10>(c0, c1, c2, c3, k0, k1, out);
}

__device__ __forceinline__ void philox4x32_7(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0,
                                             uint32_t k1, uint32_t out[4]) {
    philox4x32_r<7>(c0, c1, c2, c3, k0, k1, out);
}

}  // namespace dd
