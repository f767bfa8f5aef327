// policy_rollout.hip — collect_episodes_ppo (reference Actor_Critic_PPO.ipynb:
// 797-917) with the actor in the loop, as ONE launch for `frames` frames:
//
//   for each frame k:   obs[k] = observation (policy input)
//                       probs  = actor(obs[k])                   :851-855
//                       a, lp  = Bernoulli(probs).sample / .log_prob(a).sum   :857-859
//                       reward[k], done[k] = DroneGame.step(a)   (game_engine.py:95-138,
//                                            notebook reward + max_steps optional:
//                                            PPO's, or REINFORCE's for collect_episodes,
//                                            Policy_Gradients.ipynb:528-598)
//
// The two kernels it replaces (dd_mlp_forward + dd_step per frame) each pay a
// launch, the actor re-reads its 111 KB of packed parameters into every CU's
// LDS per call, and the observation makes an HBM round trip between them.
// Here a block of 8 waves (2 per SIMD, one block per CU: the parameters fill
// 111 KB of the 160 KB LDS) loads the parameters once and each wave carries
// its 32 drones through every frame with their state in registers:
//
//   * the network is mlp_core.h's mlp_body, the exact code of dd_mlp_forward,
//     so probabilities, samples and log-probabilities are bit-identical;
//   * the frame is frame.h's, the exact code of dd_step / dd_rollout, rounded
//     to the storage width after every frame as dd_step stores it;
//   * a wave tile is 32 drones (the MFMA's N) on 64 lanes: lane (c, h) holds
//     drone c in both halves h.  Both halves step the drone (the same
//     instructions either way) and each keeps the 8 observation columns that
//     are its B operands of the next frame's first layer, so the observation
//     never leaves the registers between frames; the [32, 15] rows a frame
//     records leave through a 1.9 KB LDS slice per wave as 16-byte stores.
//
// Bytes per drone-frame: obs 60 + action 1 + log-prob 4 + reward 4 + done 1
// (the state is read and written once per launch).  The work is the actor's
// (26.7k multiply-adds per drone-frame on the MFMA + LayerNorm on the VALU,
// which a gfx950 SIMD does not overlap); the frame adds ~3 % to a wave's
// cycles (SQ counters).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dronestep.h"
#include "frame.h"
#include "mlp_core.h"

namespace dd {
namespace prl {

using mlp::kCols;
using mlp::kPacked;
using mlp::kThreads;
using mlp::kWaves;
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kRowFloats = kCols * DD_OBS_DIM;  // one wave's [32, 15] observation slice: 480 floats
constexpr size_t kLdsBytes = (size_t)(kPacked + kWaves * kRowFloats) * sizeof(float);
static_assert(kPacked % 4 == 0 && kRowFloats % 4 == 0, "16-byte aligned LDS slices");

struct Args {
    Consts k;              // runtime constants (switches, spawn; physics when !kRef)
    const float* obs0;
    float* obs_final;
    float* obs;
    uint8_t* actions;
    float* log_prob;
    char* reward;          // [frames][n] of T
    uint8_t* done;
    double* shaped_hist;   // [2][n] (notebook reward mode) or null
    char* engine_reward;
    uint8_t* engine_done;
    uint64_t seed;
    int64_t step;
    int64_t n;
    int32_t frames;
    int32_t max_steps;
    int32_t shape;         // kShapeNone / kShapePpo / kShapeReinforce (frame.h)
    int32_t rows_aligned;  // every frame's obs rows start 16-byte aligned (obs aligned, n % 4 == 0)
    int32_t final_aligned; // obs_final 16-byte aligned
};

// Observation column `col` of layer 1's B operand for lane half h: column
// 8h + q (f16x3: one k-step of 16) or 2q + h (f32: k-steps of 2).
template <bool kSplit>
__device__ __forceinline__ constexpr int in_col(int q, int h) {
    return kSplit ? 8 * h + q : 2 * q + h;
}

// A wave's [rows, 15] observation slice, assembled in LDS from the lanes'
// columns, stored at dst (16-byte stores when aligned).
template <bool kSplit>
__device__ __forceinline__ void store_rows(float* slice, const float (&x)[8], int c, int h, int rows, float* dst,
                                           bool aligned) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        const int col = in_col<kSplit>(q, h);
        if (col < DD_OBS_DIM) slice[c * DD_OBS_DIM + col] = x[q];
    }
    __syncwarp();
    const int nf = rows * DD_OBS_DIM;
    if (aligned) {
        const int nv = nf >> 2;
        const f32x4* src4 = reinterpret_cast<const f32x4*>(slice);
        f32x4* dst4 = reinterpret_cast<f32x4*>(dst);
        for (int k = lane; k < nv; k += 64) __builtin_nontemporal_store(src4[k], &dst4[k]);
        for (int k = (nv << 2) + lane; k < nf; k += 64) __builtin_nontemporal_store(slice[k], &dst[k]);
    } else {
        for (int k = lane; k < nf; k += 64) __builtin_nontemporal_store(slice[k], &dst[k]);
    }
    __syncwarp();  // the slice is rewritten next frame
}

// The next frame's policy input: observation row of the frame's (unrounded)
// state as dd_step writes it, this lane half's 8 columns of it.
template <bool kRef, bool kGuard, bool kSplit>
__device__ __forceinline__ void next_input(const Consts& k, const Lane& s, int h, float (&x)[8]) {
    double v[13];
    observe_values<kGuard>(k, s, v);
    float o[16];
#pragma unroll
    for (int j = 0; j < 13; ++j) o[j] = (float)v[j];
    o[13] = (s.status & DD_ST_LANDED) ? 1.0f : 0.0f;
    o[14] = (s.status & DD_ST_CRASHED) ? 1.0f : 0.0f;
    o[15] = 0.0f;
#pragma unroll
    for (int q = 0; q < 8; ++q) x[q] = h ? o[in_col<kSplit>(q, 1)] : o[in_col<kSplit>(q, 0)];
}

template <typename T, bool kSplit, bool kRef>
__global__ __launch_bounds__(kThreads) void policy_rollout_kernel(const float* __restrict__ packed, Args p,
                                                                  Soa<T> a) {
    extern __shared__ f32x4 lds4[];
    float* lds = reinterpret_cast<float*>(lds4);
    for (int i = threadIdx.x; i < kPacked / 4; i += kThreads)
        lds4[i] = mlp::packed_fragment(reinterpret_cast<const f32x4*>(packed), i,
                                       mlp::pack_tag(kSplit ? DD_MLP_F16X3 : DD_MLP_F32, 3));
    __syncthreads();  // the only block barrier: waves run their frames independently

    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, h = lane >> 5, c = lane & 31;
    const int64_t d0 = ((int64_t)blockIdx.x * kWaves + wave) * kCols;
    if (d0 >= p.n) return;
    const int rows = (int)min((int64_t)kCols, p.n - d0);
    const bool live = c < rows;
    const bool writer = live && h == 0;  // one lane per drone stores its per-frame outputs
    const int64_t d = live ? d0 + c : p.n - 1;  // lanes past n shadow the last drone
    float* slice = lds + kPacked + wave * kRowFloats;
    const DDConfig& sw = p.k.c;
    const Consts& k = kRef ? kRefConsts : p.k;
    constexpr bool kGuard = !kRef && std::is_same<T, double>::value;
    const bool shaped = p.shape != kShapeNone;
    const bool ppo = p.shape == kShapePpo;
    const int64_t env = a.env_id_base + d;

    Lane s;
    s.x = a.x[d]; s.y = a.y[d]; s.vx = a.vx[d]; s.vy = a.vy[d]; s.angle = a.angle[d]; s.omega = a.omega[d];
    s.fuel = a.fuel[d]; s.px = a.px[d]; s.py = a.py[d]; s.total = a.total[d];
    s.status = a.status[d]; s.steps = a.steps[d]; s.episode = a.episode[d];
    double h0 = 0.0, h1 = 0.0;  // the notebook reward's two-frame distance history
    if (ppo) { h0 = p.shaped_hist[d]; h1 = p.shaped_hist[p.n + d]; }
    float x[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        const int col = in_col<kSplit>(q, h);
        x[q] = col < DD_OBS_DIM ? p.obs0[d * DD_OBS_DIM + col] : 0.0f;
    }

    for (int f = 0; f < p.frames; ++f) {
        const int64_t fo = (int64_t)f * p.n;  // frame offset of [frames][n] buffers
        if (p.obs) store_rows<kSplit>(slice, x, c, h, rows, p.obs + (fo + d0) * DD_OBS_DIM, p.rows_aligned);

        // the actor and the collection loop's sampling (dd_mlp_forward)
        float z[3];
        mlp::mlp_body<3, kSplit, false>(lds, lane, x, z);  // serial schedule: the frame holds the registers
        float prob[3];
        mlp::actor_probs(z, prob);
        uint32_t act;
        float lp;
        mlp::actor_sample(prob, (uint64_t)env, (uint64_t)(p.step + f), p.seed, act, lp);
        if (writer) {
            if (p.actions) __builtin_nontemporal_store((uint8_t)act, &p.actions[fo + d]);
            if (p.log_prob) __builtin_nontemporal_store(lp, &p.log_prob[fo + d]);
        }

        // the frame (dd_step / dd_rollout)
        const bool was_done = (s.status & DD_ST_DONE) != 0;
        double reward;
        if (sw.auto_reset) {  // next-step reset: the frame's result is discarded for a done lane
            reward = frame_checked<kRef, true>(k, sw, act, s);
            if (__ballot(was_done)) {
                if (was_done) {
                    spawn(sw, k.c.max_fuel, env, s);
                    reward = 0.0;
                }
            }
        } else if (was_done) {  // sticky done (game_engine.py:107-111)
            measure(s);
            reward = 0.0;
        } else {
            reward = frame_checked<kRef, true>(k, sw, act, s);
        }
        T* rew = reinterpret_cast<T*>(p.reward) + fo + d;
        uint8_t* dn = p.done + fo + d;
        if (shaped) {  // dd_step's notebook path (PPO: the history in h0 / h1)
            double v[13];
            observe_values<kGuard, true>(k, s, v);  // the notebook reward's doubles: exact quotients
            double sr = 0.0;
            bool sd;
            if (sw.auto_reset && was_done) {  // re-spawned: prev_state None
                h0 = v[9];
                h1 = __builtin_nan("");
                sd = false;
            } else if (was_done) {
                sd = true;
            } else {
                if (ppo) {
                    const bool odd = (s.steps & 1) != 0;
                    sr = notebook_reward(v, s.status, odd ? h1 : h0);
                    h1 = odd ? v[9] : h1;
                    h0 = odd ? h0 : v[9];
                } else {
                    sr = reinforce_reward(v, s.status);
                }
                sd = (s.status & DD_ST_DONE) != 0;
                if (p.max_steps > 0 && s.steps >= p.max_steps) {  // the collection loops' timeout
                    sr = (s.status & DD_ST_LANDED) ? sr : sr - 500;
                    sd = true;
                    s.status |= DD_ST_DONE;
                }
            }
            if (writer) {
                __builtin_nontemporal_store((T)sr, rew);
                __builtin_nontemporal_store((uint8_t)(sd ? 1 : 0), dn);
                if (p.engine_reward) {
                    __builtin_nontemporal_store((T)reward, reinterpret_cast<T*>(p.engine_reward) + fo + d);
                    __builtin_nontemporal_store((uint8_t)((s.status & DD_ST_DONE) ? 1 : 0), p.engine_done + fo + d);
                }
            }
        } else if (writer) {
            __builtin_nontemporal_store((T)reward, rew);
            __builtin_nontemporal_store((uint8_t)((s.status & DD_ST_DONE) ? 1 : 0), dn);
        }
        next_input<kRef, kGuard, kSplit>(k, s, h, x);  // from the unrounded frame, like dd_step's obs
        quantize<T, kRef>(s);
    }

    if (p.obs_final) store_rows<kSplit>(slice, x, c, h, rows, p.obs_final + d0 * DD_OBS_DIM, p.final_aligned);
    if (writer) {
        a.x[d] = (T)s.x; a.y[d] = (T)s.y; a.vx[d] = (T)s.vx; a.vy[d] = (T)s.vy; a.angle[d] = (T)s.angle;
        a.omega[d] = (T)s.omega; a.fuel[d] = (T)s.fuel; a.px[d] = (T)s.px; a.py[d] = (T)s.py;
        a.total[d] = (T)s.total; a.status[d] = (uint8_t)s.status; a.steps[d] = s.steps; a.episode[d] = s.episode;
        if (ppo) { p.shaped_hist[d] = h0; p.shaped_hist[p.n + d] = h1; }
    }
}

template <typename T, bool kSplit, bool kRef>
hipError_t launch(const float* packed, const Args& p, const Soa<T>& a, hipStream_t s) {
    // the LDS image exceeds the 64 KB default; per device, so set on every launch
    const hipError_t e = hipFuncSetAttribute((const void*)policy_rollout_kernel<T, kSplit, kRef>,
                                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)kLdsBytes);
    if (e != hipSuccess) return e;
    const int64_t tiles = (p.n + kCols - 1) / kCols;
    const unsigned blocks = (unsigned)((tiles + kWaves - 1) / kWaves);  // one wave per 32-drone tile
    hipLaunchKernelGGL((policy_rollout_kernel<T, kSplit, kRef>), dim3(blocks), dim3(kThreads), kLdsBytes, s, packed,
                       p, a);
    return hipGetLastError();
}

template <typename T, bool kSplit>
hipError_t launch_ref(bool ref, const float* packed, const Args& p, const Soa<T>& a, hipStream_t s) {
    return ref ? launch<T, kSplit, true>(packed, p, a, s) : launch<T, kSplit, false>(packed, p, a, s);
}

}  // namespace prl
}  // namespace dd

extern "C" int dd_policy_rollout(const DDConfig* cfg, const DDState* st, const float* packed, int32_t compute,
                                 const DDPolicyRolloutIO* io, int64_t n, void* stream) {
    if (!cfg || !io || !dd::state_ok(st) || n < 0 || io->frames < 0) return hipErrorInvalidValue;
    if (compute != DD_MLP_F32 && compute != DD_MLP_F16X3) return hipErrorInvalidValue;
    if ((io->engine_reward == nullptr) != (io->engine_done == nullptr)) return hipErrorInvalidValue;
    if (io->shaped_mode != DD_SHAPED_PPO && io->shaped_mode != DD_SHAPED_REINFORCE) return hipErrorInvalidValue;
    const int shape = io->shaped_mode == DD_SHAPED_REINFORCE ? dd::kShapeReinforce
                      : io->shaped_hist ? dd::kShapePpo : dd::kShapeNone;
    if (io->engine_reward && shape == dd::kShapeNone) return hipErrorInvalidValue;
    if (n == 0) return hipSuccess;
    if (!packed || !io->obs0 || (io->frames > 0 && (!io->reward || !io->done))) return hipErrorInvalidValue;
    if (reinterpret_cast<uintptr_t>(packed) & 15u) return hipErrorInvalidValue;  // read as 16-byte fragments
    if (io->frames == 0 && io->obs_final == nullptr) return hipSuccess;
    dd::prl::Args p{};
    p.k = dd::make_consts(*cfg);
    p.obs0 = io->obs0;
    p.obs_final = io->obs_final;
    p.obs = io->obs;
    p.actions = io->actions;
    p.log_prob = io->log_prob;
    p.reward = static_cast<char*>(io->reward);
    p.done = io->done;
    p.shaped_hist = io->shaped_hist;
    p.engine_reward = static_cast<char*>(io->engine_reward);
    p.engine_done = io->engine_done;
    p.seed = io->seed;
    p.step = io->step;
    p.n = n;
    p.frames = io->frames;
    p.max_steps = io->max_steps;
    p.shape = shape;
    p.rows_aligned = (reinterpret_cast<uintptr_t>(io->obs) & 15u) == 0 && (n & 3) == 0;
    p.final_aligned = (reinterpret_cast<uintptr_t>(io->obs_final) & 15u) == 0;
    const bool ref = dd::uses_reference_physics(*cfg);
    const hipStream_t s = (hipStream_t)stream;
    hipError_t e;
    if (st->precision == DD_F64) {
        const dd::Soa<double> a = dd::soa_of<double>(*st, 0);
        e = compute == DD_MLP_F16X3 ? dd::prl::launch_ref<double, true>(ref, packed, p, a, s)
                                    : dd::prl::launch_ref<double, false>(ref, packed, p, a, s);
    } else {
        const dd::Soa<float> a = dd::soa_of<float>(*st, 0);
        e = compute == DD_MLP_F16X3 ? dd::prl::launch_ref<float, true>(ref, packed, p, a, s)
                                    : dd::prl::launch_ref<float, false>(ref, packed, p, a, s);
    }
    return (int)e;
}
