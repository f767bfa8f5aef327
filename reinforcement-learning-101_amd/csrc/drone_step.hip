// drone_step.hip — MI355X (gfx950) kernels behind include/dronestep.h.
//
// One lane = one drone.  The frame of DroneGame.step (reference
// delivery_drone/game/game_engine.py:95-138) is evaluated in IEEE double in
// registers, in the reference's operation order, and rounded once on store
// (DD_F32) or not at all (DD_F64).  The path moves ~147 B per drone-frame for
// ~220 double ops, so the kernel is shaped for bytes and for VALU issue:
//   * SoA dword loads/stores, coalesced per wave64, addressed as a wave-uniform
//     SGPR base + one 32-bit lane offset (launches are chunked so offsets fit);
//   * the reference's world constants (config.py) folded into the instruction
//     stream when the run uses them (the usual case), kernarg otherwise;
//   * observation rows staged through LDS so each [256, 15] tile leaves as
//     contiguous 16-byte non-temporal stores;
//   * done-lane compaction by wave ballots, one atomic per wave.
//
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -fPIC -shared
// (-ffp-contract=off keeps every a*b+c as the reference's two roundings.)

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <type_traits>

#include "dronestep.h"
#include "frame.h"
#include "philox.h"
#include "trig.h"

namespace dd {

constexpr int kBlock = 256;  // 4 waves; one obs tile = 256 rows
constexpr int kWave = 64;
// Lanes per launch: keeps every byte offset (lane x 8 B) below 2^31.
constexpr int64_t kChunk = int64_t(1) << 28;
typedef float f32x4 __attribute__((ext_vector_type(4)));

// ---------------------------------------------------------------------------
// SoA access: wave-uniform base pointers (SGPRs) + one 32-bit byte offset per
// lane, so every load/store is `global_load_dword v, v_off, s[base]`.
// ---------------------------------------------------------------------------

// Store cache policies (gfx950), measured per stream: the
// SoA state is stored plainly (write-back into the XCD's L2; the next step
// reads it there), the output streams this kernel never re-reads (reward,
// done, observation rows) with the non-temporal hint (+2-6 % at 262,144 and
// 16.8M lanes).  Write-through (sc1) state stores made the next step's loads
// miss L2 (0.5 -> 1.35 us), non-temporal state stores / loads were slower.
template <typename E>
__device__ __forceinline__ void store_nt(E* base, uint32_t i, E v) {
    __builtin_nontemporal_store(v, &at(base, i));
}

typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// Output streams this kernel never re-reads (reward, done) are stored
// non-temporally, like the obs tile.
template <typename E>
__device__ __forceinline__ void put_out(E* base, uint32_t i, E v) {
    asm volatile("" : "+v"(i));  // keep the offset 32-bit and local: SGPR-base store
    store_nt(base, i, v);
}

template <typename T>
__device__ __forceinline__ void load_dynamics(const Soa<T>& a, uint32_t i, Lane& s) {
    s.x = at(a.x, i); s.y = at(a.y, i); s.vx = at(a.vx, i); s.vy = at(a.vy, i);
    s.angle = at(a.angle, i); s.omega = at(a.omega, i); s.fuel = at(a.fuel, i);
    s.px = at(a.px, i); s.py = at(a.py, i);
}

template <typename E>
__device__ __forceinline__ void put_state(E* base, uint32_t i, E v) {
    at(base, i) = v;
}

template <typename T>
__device__ __forceinline__ void store_dynamics(const Soa<T>& a, uint32_t i, const Lane& s) {
    put_state(a.x, i, (T)s.x); put_state(a.y, i, (T)s.y); put_state(a.vx, i, (T)s.vx);
    put_state(a.vy, i, (T)s.vy); put_state(a.angle, i, (T)s.angle); put_state(a.omega, i, (T)s.omega);
    put_state(a.fuel, i, (T)s.fuel);
}

template <typename T, bool kTotal = true>
__device__ __forceinline__ void store_spawn(const Soa<T>& a, uint32_t i, const Lane& s) {
    store_dynamics(a, i, s);
    at(a.px, i) = (T)s.px; at(a.py, i) = (T)s.py;
    if constexpr (kTotal) at(a.total, i) = (T)s.total;
    at(a.status, i) = (uint8_t)s.status;
    at(a.steps, i) = s.steps;
    at(a.episode, i) = s.episode;
}

// Writes a block's [rows, 15] observation tile from LDS to global memory as
// 16-byte stores (non-temporal: the rows are the step's output stream, read
// by the consumer, not by this kernel again).  dst = first row of the tile.
template <int NB = kBlock>
__device__ __forceinline__ void flush_obs_tile(const float* tile, float* dst, int rows) {
    const int nf = rows * DD_OBS_DIM;
    // tiles start at multiples of 256 rows (15360 B): dst is 16-B aligned iff obs is
    if ((reinterpret_cast<uintptr_t>(dst) & 15u) == 0) {
        const int nv = nf >> 2;
        const f32x4* src4 = reinterpret_cast<const f32x4*>(tile);
        f32x4* dst4 = reinterpret_cast<f32x4*>(dst);
        for (int k = threadIdx.x; k < nv; k += NB) __builtin_nontemporal_store(src4[k], &dst4[k]);
        for (int k = (nv << 2) + threadIdx.x; k < nf; k += NB) dst[k] = tile[k];
    } else {
        for (int k = threadIdx.x; k < nf; k += NB) dst[k] = tile[k];
    }
}

// The same for one wave's slice of the tile (rows <= 64, starting at the
// wave's first row): only this wave wrote and reads the slice, so a
// wave-level sync stands in for the block barrier and each wave's rows leave
// as soon as its own lanes are done.  dst + 64-row slices of 3840 B keep
// the 16-byte alignment of the tile.
__device__ __forceinline__ void flush_obs_wave(const float* wtile, float* dst, int rows) {
    __syncwarp();
    const int lane = threadIdx.x & (kWave - 1);
    const int nf = rows * DD_OBS_DIM;
    if ((reinterpret_cast<uintptr_t>(dst) & 15u) == 0) {
        const int nv = nf >> 2;
        const f32x4* src4 = reinterpret_cast<const f32x4*>(wtile);
        f32x4* dst4 = reinterpret_cast<f32x4*>(uniform_ptr(dst));
        for (int k = lane; k < nv; k += kWave) store_nt(dst4, (uint32_t)k, src4[k]);
        for (int k = (nv << 2) + lane; k < nf; k += kWave) dst[k] = wtile[k];
    } else {
        for (int k = lane; k < nf; k += kWave) dst[k] = wtile[k];
    }
    __syncwarp();  // the slice may be rewritten next (rollout frames)
}

template <int AFMT>
__device__ __forceinline__ uint32_t load_action(const void* actions, uint32_t i) {
    if constexpr (AFMT == DD_ACT_BITMASK) {
        return at(static_cast<const uint8_t*>(actions), i);
    } else if constexpr (AFMT == DD_ACT_F32X3) {
        const float* a = &at(static_cast<const float*>(actions), 3 * i);
        return (a[0] != 0.0f ? 1u : 0u) | (a[1] != 0.0f ? 2u : 0u) | (a[2] != 0.0f ? 4u : 0u);
    } else {
        const uint8_t* a = &at(static_cast<const uint8_t*>(actions), 3 * i);
        return (a[0] ? 1u : 0u) | (a[1] ? 2u : 0u) | (a[2] ? 4u : 0u);
    }
}

// ---------------------------------------------------------------------------
// dd_step kernel: one 256-lane tile per block, one chunk of lanes per launch.
// ---------------------------------------------------------------------------
struct StepArgs {
    Consts k;              // runtime constants (switches, spawn; physics when !kRef)
    const void* actions;   // chunk-relative
    void* reward;
    uint8_t* done;
    float* obs;
    int32_t* done_idx;
    int32_t* done_count;
    int32_t n;             // lanes in this chunk
    int32_t idx_base;      // chunk start, for done_idx entries
    double* shaped_hist;   // slot 0 of this chunk; slot 1 at + hist_stride
    int64_t hist_stride;
    void* shaped_reward;
    uint8_t* shaped_done;
    int32_t max_steps;
};

// 256 lanes per block: 128 / 512 / 1024 measured +0 / +4 / +14 % at 262,144
// drones; no occupancy floor (forcing 8 waves per SIMD spilled).
constexpr int kStepBlock = 256;

// A lane's inputs as loaded (storage width), before widening to double.
template <typename T>
struct Raw {
    T x, y, vx, vy, angle, omega, fuel, px, py, total;
    uint32_t status, act;
    int32_t steps;
};

template <typename T, int AFMT>
__device__ __forceinline__ void load_raw(const Soa<T>& a, const void* actions, uint32_t i, Raw<T>& r) {
    // The action is loaded first and pinned below: only the live branch reads
    // it, and left to itself the compiler sank its load into that branch,
    // i.e. behind the wait for the status byte: a second memory round trip.
    r.act = load_action<AFMT>(actions, i);
    r.x = at(a.x, i); r.y = at(a.y, i); r.vx = at(a.vx, i); r.vy = at(a.vy, i);
    r.angle = at(a.angle, i); r.omega = at(a.omega, i); r.fuel = at(a.fuel, i);
    r.px = at(a.px, i); r.py = at(a.py, i); r.total = at(a.total, i);
    r.status = at(a.status, i);
    r.steps = at(a.steps, i);
    asm volatile("" ::"v"(r.act));  // every load is issued; this waits for the oldest only
}

// Everything after the loads for one lane: the frame (or sticky done / auto
// reset), the state and output stores, the observation row into `orow`
// (LDS).  Returns whether the lane's episode ended in this call.  The fast
// frame may report the lane risky (frame.h): then, in a wave-uniform rare
// branch, the lane's frame is redone at once from its loaded inputs with
// kExact (glibc's sin, cos and pow), and the rest of the lane's work is
// shared.  (Until round 6 a second finish_lane pass over the risky lanes
// redid everything after the loads: the same results, but that copy of the
// observation, reward and store code cost config 3 1-2 % in time and ~110
// instruction-wait cycles per wave, profiles/r06/lab/step_inline_exact.jsonl.)
// kShape: the notebooks' reward fused (frame.h, kShapePpo / kShapeReinforce).
// kPP (ping-pong, DDStepIO.state_out): the nine per-frame fields (x y vx vy
// angle omega fuel total steps) go to `o`; px, py, status and episode always
// go to `a`.  In place (the usual case) the kernel has no `o` at all.
template <typename T, bool kRef, int kShape, bool kPP>
__device__ __forceinline__ bool finish_lane(const StepArgs& p, const Soa<T>& a, const Soa<T>& o, uint32_t i,
                                            const Raw<T>& r, float* orow) {
    const DDConfig& sw = p.k.c;
    const Consts& k = kRef ? kRefConsts : p.k;
    Lane s;
    s.x = r.x; s.y = r.y; s.vx = r.vx; s.vy = r.vy; s.angle = r.angle; s.omega = r.omega;
    s.fuel = r.fuel; s.px = r.px; s.py = r.py; s.total = r.total;
    s.status = r.status;
    s.steps = r.steps;
    bool ended = false;
    bool respawned = false;
    double reward;
    double shaped = 0.0;
    bool shaped_done = false;
    if (s.status & DD_ST_DONE) {
        reward = 0.0;
        if (sw.auto_reset) {  // next-step reset: fresh episode, reward 0, done 0
            s.episode = at(a.episode, i);
            spawn(sw, k.c.max_fuel, a.env_id_base + i, s);
            respawned = true;
            if constexpr (kShape == kShapePpo) {  // the notebook's history restarts: prev_state None
                at(p.shaped_hist, i) = trig::div_exact(s.dist, k.c.world_width, k.inv_w);
                at(p.shaped_hist + p.hist_stride, i) = __builtin_nan("");
            }
        } else {  // sticky done (game_engine.py:107-111): nothing changes
            measure(s);
            shaped_done = true;
        }
    } else {
        bool rk = false;
        reward = frame<kRef, false>(k, sw, r.act, s, &rk);
        if (__builtin_expect(__ballot(rk) != 0, 0)) {
            if (rk) {  // the frame again from the loaded state, the reference's functions (frame.h)
                s.x = r.x; s.y = r.y; s.vx = r.vx; s.vy = r.vy; s.angle = r.angle; s.omega = r.omega;
                s.fuel = r.fuel; s.px = r.px; s.py = r.py; s.total = r.total; s.status = r.status;
                s.steps = r.steps;
                reward = frame<kRef, false, true>(k, sw, r.act, s, nullptr);
            }
        }
        if constexpr (kShape != kShapeNone) {
            double v[13];
            observe_values<false, true>(k, s, v);  // the notebook reward's doubles: exact quotients
            if constexpr (kShape == kShapePpo) {
                double* slot = p.shaped_hist + (s.steps & 1) * p.hist_stride;  // two frames back
                shaped = notebook_reward(v, s.status, at(slot, i));
                at(slot, i) = v[9];
            } else {
                shaped = reinforce_reward(v, s.status);
            }
            shaped_done = (s.status & DD_ST_DONE) != 0;
            if (p.max_steps > 0 && s.steps >= p.max_steps) {  // the collection loops' timeout
                shaped = (s.status & DD_ST_LANDED) ? shaped : shaped - 500;
                shaped_done = true;
                s.status |= DD_ST_DONE;  // the episode ends here (TimeLimit)
            }
            if (p.obs) observe(k, s, orow);  // rows as every other path writes them
        }
        ended = (s.status & DD_ST_DONE) != 0;
    }
    // State stores after the branches merge, so each is one SGPR-base +
    // lane-offset store (stores inside the branches got 64-bit per-lane
    // addresses, 22 VGPRs live across the frame).  A sticky-done lane
    // writes nothing; status and px only change on the terminal frame, a
    // respawn or a moving platform; py and episode only on a respawn.
    // (with separate out arrays a sticky lane copies its fields across)
    const bool sticky = (r.status & DD_ST_DONE) && !respawned && !kPP;
    if (!sticky) {
        uint32_t j = i;
        asm volatile("" : "+v"(j));  // an offset defined in this block: isel folds it into saddr stores
        store_dynamics(o, j, s);
        put_state(o.steps, j, s.steps);
        put_state(o.total, j, (T)s.total);
        const bool moving = !kRef && sw.platform_moving;
        if (moving || respawned) put_state(a.px, j, (T)s.px);
        if (moving || ended || respawned) put_state(a.status, j, (uint8_t)s.status);
        if (respawned) { put_state(a.py, j, (T)s.py); put_state(a.episode, j, s.episode); }
    }
    put_out(static_cast<T*>(p.reward), i, (T)reward);
    put_out(p.done, i, (uint8_t)((s.status & DD_ST_DONE) ? 1 : 0));
    if constexpr (kShape != kShapeNone) {
        put_out(static_cast<T*>(p.shaped_reward), i, (T)shaped);
        put_out(p.shaped_done, i, (uint8_t)(shaped_done ? 1 : 0));
        if (p.obs && ((r.status & DD_ST_DONE) != 0)) observe(k, s, orow);  // the live path wrote its row
    } else {
        if (p.obs) observe(k, s, orow);
    }
    return ended;
}

// One step tile: one drone per lane, kStepBlock lanes.  `o` is `a` unless kPP.
template <typename T, int AFMT, bool kRef, int kShape, bool kPP>
__device__ __forceinline__ void step_tile(const StepArgs& p, const Soa<T>& a, const Soa<T>& o) {
    __shared__ __attribute__((aligned(16))) float tile[kStepBlock * DD_OBS_DIM];
    const uint32_t row0 = blockIdx.x * kStepBlock;
    const uint32_t i = row0 + threadIdx.x;
    // The load bases are wanted in SGPRs before the lane test: left to
    // itself the compiler sank their kernarg loads into the `i < n` branch,
    // one scalar-load latency later than the state loads could start.
    asm volatile("" ::"s"(a.x), "s"(a.y), "s"(a.vx), "s"(a.vy), "s"(a.angle), "s"(a.omega), "s"(a.fuel),
                 "s"(a.px), "s"(a.py), "s"(a.total), "s"(a.status), "s"(a.steps), "s"(p.actions));
    Raw<T> r;
    if (i < (uint32_t)p.n) load_raw<T, AFMT>(a, p.actions, i, r);
    const bool ended = i < (uint32_t)p.n &&
                       finish_lane<T, kRef, kShape, kPP>(p, a, o, i, r, tile + threadIdx.x * DD_OBS_DIM);
    if (p.done_idx) {  // wave-ballot compaction of the lanes that just ended
        const uint64_t m = __ballot(ended);
        if (m) {
            const int lane = threadIdx.x & (kWave - 1);
            const int leader = __ffsll((unsigned long long)m) - 1;
            const int before = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                         __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
            int b = 0;
            if (lane == leader) b = atomicAdd(p.done_count, __popcll(m));
            b = __shfl(b, leader);
            if (ended) p.done_idx[b + before] = p.idx_base + (int32_t)i;
        }
    }
    if (p.obs) {  // each wave's 64 rows leave as 16-byte stores
        const uint32_t wrow0 = row0 + (threadIdx.x & ~(kWave - 1));
        const int rows = (int)min((int64_t)kWave, max((int64_t)0, (int64_t)p.n - wrow0));
        flush_obs_wave(tile + (threadIdx.x & ~(kWave - 1)) * DD_OBS_DIM, p.obs + (size_t)wrow0 * DD_OBS_DIM, rows);
    }
}

// dd_step kernel, in place (the usual case: one set of state bases).
template <typename T, int AFMT, bool kRef, int kShape>
__global__ __launch_bounds__(kStepBlock) void step_kernel(StepArgs p, Soa<T> a) {
    step_tile<T, AFMT, kRef, kShape, false>(p, a, a);
}

// dd_step kernel with ping-pong state (DDStepIO.state_out): its own
// instantiation, so the in-place kernel carries none of its plumbing (the
// shared kernel's `if (!ping_pong) o = a` had cost config 3 ~0.1 us).
template <typename T, int AFMT, bool kRef, int kShape>
__global__ __launch_bounds__(kStepBlock) void step_pp_kernel(StepArgs p, Soa<T> a, Soa<T> o) {
    step_tile<T, AFMT, kRef, kShape, true>(p, a, o);
}

// ---------------------------------------------------------------------------
// dd_rollout kernel: `frames` consecutive frames per launch, the lane's state
// in registers between frames.  Per frame a lane reads its action (1 B, the
// next frame's prefetched) and writes reward, done and its obs row (through
// its wave's LDS slice; no block barrier, waves drift freely).  Same frame code as
// step_kernel, so a rollout equals `frames` dd_step calls bit for bit.
// ---------------------------------------------------------------------------
struct RolloutArgs {
    Consts k;
    const char* actions;      // frame 0, lane 0 of this chunk
    int64_t act_stride;       // bytes between frames (N x action width)
    uint32_t act_bytes;       // extent of the launch's action rows from `actions` (< 2^32, see rollout_chunks)
    char* reward;             // frame 0, lane 0 of this chunk
    int64_t reward_stride;    // bytes between frames
    uint8_t* done;
    float* obs;               // frame 0, row 0 of this chunk (nullable)
    int64_t n_total;          // N: frame stride in lanes for done / obs
    int32_t frames;
    int32_t n;                // lanes in this chunk
    uint64_t action_seed;
    int64_t action_step;
    // the notebooks' reward (kShape): reward / done above receive calc_reward
    // and the notebook's done; the engine's go to these (nullable)
    double* shaped_hist;      // kShapePpo: slot 0 of this chunk; slot 1 at + n_total
    char* engine_reward;      // frame 0, lane 0 of this chunk (reward_stride apart)
    uint8_t* engine_done;
    int32_t max_steps;
    int32_t spin_cap;         // kSplit: polls per hand-over wait before it is reported (DD_ERR_HANDOVER)
};

// DD_ACT_PHILOX: one Philox4x32-10 block (key = action_seed, ctr = {env,
// step >> 5, 0xA5A5A5A5 ^ (step >> 5)_hi}) serves 32 consecutive steps: nibble
// step & 31 of its 128 output bits, whose low 3 bits are the bitmask (uniform
// and independent per thruster).  Still a function of (seed, env, step) only,
// so any split of a rollout into launches draws the same actions; one block
// per 32 frames instead of one per frame took ~7 % off the config-5 rollout.
struct PhiloxActions {
    uint32_t w[4];
    int64_t blk = -1;
};

template <int AFMT>
__device__ __forceinline__ uint32_t rollout_action(const RolloutArgs& p, int64_t env, int f, uint32_t i,
                                                   PhiloxActions& pa) {
    if constexpr (AFMT == DD_ACT_PHILOX) {
        const uint64_t step = (uint64_t)(p.action_step + f);
        const int64_t blk = (int64_t)(step >> 5);
        if (blk != pa.blk) {  // wave-uniform: every 32nd frame
            philox4x32_10((uint32_t)env, (uint32_t)((uint64_t)env >> 32), (uint32_t)blk,
                          (uint32_t)((uint64_t)blk >> 32) ^ 0xA5A5A5A5u, (uint32_t)p.action_seed,
                          (uint32_t)(p.action_seed >> 32), pa.w);
            pa.blk = blk;
        }
        const uint32_t q = (uint32_t)(step >> 3) & 3u;
        const uint32_t word = q == 0 ? pa.w[0] : q == 1 ? pa.w[1] : q == 2 ? pa.w[2] : pa.w[3];
        return (word >> (4u * ((uint32_t)step & 7u))) & 7u;
    } else {
        return load_action<AFMT>(p.actions + f * p.act_stride, i);
    }
}

// A kernel's by-value Soa argument (placed after `Args` in the kernarg
// segment) read again through an opaque pointer.  The frame loop of
// rollout_kernel does not touch the state arrays, but with `a` itself used
// after the loop the compiler kept its 26 pointer SGPRs live across the loop
// and spilled them to VGPR lanes; the second read lets them die.
template <typename Args, typename T>
__device__ __forceinline__ Soa<T> reload_soa() {
#if defined(__HIP_DEVICE_COMPILE__)
    constexpr size_t off = (sizeof(Args) + alignof(Soa<T>) - 1) / alignof(Soa<T>) * alignof(Soa<T>);
    uint64_t kp = (uint64_t)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(kp));
    typedef const __attribute__((address_space(4))) Soa<T> KSoa;
    const KSoa* q = reinterpret_cast<KSoa*>(kp + off);
    Soa<T> r;
    r.x = q->x; r.y = q->y; r.vx = q->vx; r.vy = q->vy; r.angle = q->angle; r.omega = q->omega;
    r.fuel = q->fuel; r.px = q->px; r.py = q->py; r.total = q->total;
    r.status = q->status; r.steps = q->steps; r.episode = q->episode; r.env_id_base = q->env_id_base;
    return r;
#else
    return Soa<T>{};  // the host pass never runs device code
#endif
}

// Rollout observation staging.  kHeld (every frame row of the launch starts
// 16-byte aligned: obs aligned and N % 4 == 0, the usual case): two LDS
// slices per wave; frame f's rows go into slice f & 1 while frame f - 1's
// rows are read back into registers before frame f's arithmetic and stored
// after it, so the LDS round trip and the stores overlap the frame instead
// of following it (the rollout runs one wave per SIMD at 65,536 drones:
// nothing else hides latency).
// !kHeld: one slice per wave, flushed after each frame.
struct HeldObs {
    f32x4 v[4];  // a 64-row slice is 240 float4: 3.75 per lane
};

// Reads the whole 64-row slice at wtile (plus padding: the tile carries
// kHeldPad floats past its last slice), unconditionally so the four reads
// issue back to back; store_held_wave writes only the float4s that are rows.
constexpr int kHeldPad = 4 * kWave * 4 - kWave * DD_OBS_DIM;  // 256 float4 read vs 240 in a slice

__device__ __forceinline__ void hold_obs_wave(const float* wtile, HeldObs& h) {
    const int lane = threadIdx.x & (kWave - 1);
    const f32x4* src4 = reinterpret_cast<const f32x4*>(wtile);
#pragma unroll
    for (int j = 0; j < 4; ++j) h.v[j] = src4[lane + j * kWave];
}

// A raw buffer resource over [p, p + bytes): accesses at offsets >= bytes
// are dropped (stores) or read 0 (loads) by the hardware's range check.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_over(const void* p, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, (int)bytes, 0x00020000);
}

// The held slice leaves as four unconditional 16-byte non-temporal raw
// buffer stores over the wave's slice of one frame (`slice` covers its rows
// * 60 bytes): float4 lane + 64 j past the slice (lanes >= 48 of j = 3, all
// of a ragged wave's missing rows) is dropped by the range check.  No
// exec-mask branches, so every frame issues the same vector-memory
// instructions and the compiler's vmcnt waits for the action prefetch count
// exactly (with the branchy stores of rounds 1-3 it waited, at the end of
// every frame pair, for that pair's own reward / done / obs stores:
// SQ_WAIT_ANY 186 of 720 wave cycles per frame).  Under kHeld N % 4 == 0,
// so a wave's slice is whole float4s.
__device__ __forceinline__ void store_held_wave(const HeldObs& h, __amdgpu_buffer_rsrc_t slice) {
    const uint32_t lane = threadIdx.x & (kWave - 1);
#pragma unroll
    for (int j = 0; j < 4; ++j)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, h.v[j]), slice, (lane + j * kWave) * 16u, 0,
                                               2 /* nt */);
}

// One lane's action of one frame, by raw buffer loads over the launch's
// [frames][N] action rows (rollout_chunks keeps every consumed offset below
// 2^32): a prefetch past the last frame needs no clamp, the range check
// makes it read 0.
template <int AFMT>
__device__ __forceinline__ uint32_t buffer_action(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    if constexpr (AFMT == DD_ACT_BITMASK) {
        return __builtin_amdgcn_raw_buffer_load_b8(r, off, 0, 0);
    } else if constexpr (AFMT == DD_ACT_F32X3) {
        const float a0 = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0));
        const float a1 = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, off + 4u, 0, 0));
        const float a2 = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, off + 8u, 0, 0));
        return (a0 != 0.0f ? 1u : 0u) | (a1 != 0.0f ? 2u : 0u) | (a2 != 0.0f ? 4u : 0u);
    } else {
        const uint32_t a0 = __builtin_amdgcn_raw_buffer_load_b8(r, off, 0, 0);
        const uint32_t a1 = __builtin_amdgcn_raw_buffer_load_b8(r, off + 1u, 0, 0);
        const uint32_t a2 = __builtin_amdgcn_raw_buffer_load_b8(r, off + 2u, 0, 0);
        return (a0 ? 1u : 0u) | (a1 ? 2u : 0u) | (a2 ? 4u : 0u);
    }
}

// ---------------------------------------------------------------------------
// Split rollout (kSplit: kRef, unshaped, held obs, one block per CU).  A block
// is 8 waves: waves 0-3 step the drones (the "frame" waves), waves 4-7 write
// the frames' outputs (the "writer" waves), one writer per frame wave, which
// the dispatcher places on the same SIMD (wave w and w + 4 of a block).  At
// 65,536 drones the single-role kernel runs one wave per SIMD, which issues
// about one instruction per 2.5 ns — half the SIMD's rate; the writer's
// instructions (the observation's 13 quotients and conversions, the row
// staging, every output store and its waits) go into the other half.  A
// frame wave hands each frame over through LDS as 6 (float) or 7 (double)
// float4 per lane: the unrounded doubles the observation reads, the status
// and the reward as stored.
// Hand-over: two slots per pair, two counters in LDS.  produced[w] = frames
// the frame wave has written, consumed[w] = frames the writer has finished
// with.  LDS executes one wave's operations in issue order, so a counter
// written after the data (program order, a compiler barrier between) is seen
// only after the data is; no s_waitcnt is needed on either side.  The frame
// wave writes slot f & 1 once consumed >= f - 1 (the writer is done with
// frame f - 2; it reads that counter at the frame's start, so the wait at
// the end is normally already satisfied).  Deadlock-free: the writer only
// waits for frames the frame wave has produced, the frame wave only for the
// writer to finish frames it has produced.
// Every wait is bounded (spin_cap polls of ~64 clocks, 2^20 = ~30 ms): a
// wait that runs out sets DD_ERR_HANDOVER in the device error word
// (dd_device_errors) and the wave carries on, so a broken hand-over ends the
// kernel (never a wave that spins forever) and is reported, not silent.
constexpr int kSpinCap = 1 << 20;
constexpr int kStageQ = 5;

struct D2 {
    double a, b;
};

// (the value is a VGPR: readfirstlane it where it is tested, so a read issued
// early does not wait for the LDS at the read)
// Ordering, under the HIP memory model and not only because LDS executes one
// wave's operations in issue order: a counter store is preceded by a
// workgroup-scope release fence over LDS (the slot's data before the counter
// that publishes it), and a wait that has seen a counter is followed by the
// matching acquire fence (ctr_acquire).  On gfx950 each is an lgkmcnt(0)
// wait; the loads themselves stay relaxed so that the frame wave's early read
// of `consumed` does not wait for the LDS where it is issued.
__device__ __forceinline__ int ctr_load(const int* c) {
    return __hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void ctr_acquire() { __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local"); }
__device__ __forceinline__ void ctr_store(int* c, int v) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __hip_atomic_store(c, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// The device error word (dd_device_errors): sticky DD_ERR_* bits, one vector
// atomic from the first active lane of the wave that hits the condition.
__device__ uint32_t dd_error_bits;
__device__ __forceinline__ void raise_error(uint32_t bit) {
    if (__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0)) ==
        (uint32_t)__ffsll((unsigned long long)__ballot(1)) - 1)
        __hip_atomic_fetch_or(&dd_error_bits, bit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// slot: this wave's kStageQ x 64 float4 of one frame (float4 q of lane l at q * 64 + l).
// Never __builtin_bit_cast a vector ELEMENT (v[i], v.x): ROCm 7.2's clang
// bit-casts the vector's first element whatever the index (it takes the
// element's address as the vector's).  The first version of this hand-over
// bit-cast element 2 of the last float4 to read the status and got the
// speed's low word: every row's landed / crashed columns were wrong
// (tests/test_gpu_configs.py config 2 caught it; tests/test_source_lint.py
// now rejects the pattern).  Elements go through __uint_as_float / plain
// integer conversions.
__device__ __forceinline__ u32x4 words2(double a, double b) {
    const uint64_t x = __builtin_bit_cast(uint64_t, a), y = __builtin_bit_cast(uint64_t, b);
    return u32x4{(uint32_t)x, (uint32_t)(x >> 32), (uint32_t)y, (uint32_t)(y >> 32)};
}
__device__ __forceinline__ double word_pair(uint32_t lo, uint32_t hi) {
    return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ D2 unpack2(u32x4 w) { return D2{word_pair(w[0], w[1]), word_pair(w[2], w[3])}; }

// The frame's state as frame() leaves it under kDefer (unrounded), and the
// status word with kWasDone when the lane started the frame done: 5 float4.
constexpr uint32_t kWasDone = 1u << 8;
__device__ __forceinline__ void stage_put(f32x4* slot, uint32_t lane, const Lane& s, uint32_t status) {
    const auto put = [&](int q, u32x4 w) { slot[q * kWave + lane] = __builtin_bit_cast(f32x4, w); };
    put(0, words2(s.x, s.y));
    put(1, words2(s.vx, s.vy));
    put(2, words2(s.angle, s.omega));
    put(3, words2(s.fuel, s.px));
    const uint64_t py = __builtin_bit_cast(uint64_t, s.py);
    put(4, u32x4{(uint32_t)py, (uint32_t)(py >> 32), status, 0u});
}

__device__ __forceinline__ void stage_get(const f32x4* slot, uint32_t lane, Lane& s, uint32_t& status) {
    u32x4 q[kStageQ];
#pragma unroll
    for (int j = 0; j < kStageQ; ++j) q[j] = __builtin_bit_cast(u32x4, slot[j * kWave + lane]);
    D2 d = unpack2(q[0]);
    s.x = d.a, s.y = d.b;
    d = unpack2(q[1]);
    s.vx = d.a, s.vy = d.b;
    d = unpack2(q[2]);
    s.angle = d.a, s.omega = d.b;
    d = unpack2(q[3]);
    s.fuel = d.a, s.px = d.b;
    s.py = word_pair(q[4][0], q[4][1]);
    status = q[4][2];
}

// per SIMD: 2 keeps the kernel within 256 registers in all (1 let the Philox-action
// variant take 2 AGPRs on top of 256 VGPRs, one wave per SIMD at 262,144 drones:
// +38 %); 4 caps it at 128 VGPRs and spills (A/B: DESIGN.md section 4)
constexpr int kRollMinWaves = 2;
template <typename T, int AFMT, bool kRef, bool kHeld, int kShape, bool kSplit = false>
__global__ __launch_bounds__(kSplit ? 2 * kBlock : kBlock, kRollMinWaves) void rollout_kernel(RolloutArgs p,
                                                                                              Soa<T> a) {
    static_assert(!kSplit || (kRef && kHeld && kShape == kShapeNone),
                  "the split rollout covers the reference config's held path");
    // kSplit: the frame hand-over slots (the writer stages its rows in the
    // slot it has just read); otherwise the observation tile
    constexpr int kTileFloats = kSplit ? 4 : kBlock * DD_OBS_DIM + (kHeld ? kHeldPad : 0);
    __shared__ __attribute__((aligned(16))) float tile[kHeld && !kSplit ? 2 : 1][kTileFloats];
    __shared__ __attribute__((aligned(16))) f32x4 stage[kSplit ? kBlock / kWave : 1][2][kSplit ? kStageQ : 1]
                                                      [kSplit ? kWave : 1];
    __shared__ int ctr[2][kBlock / kWave];  // kSplit: produced, consumed
    if constexpr (kSplit) {
        if (threadIdx.x < 2 * (kBlock / kWave)) ctr[threadIdx.x >> 2][threadIdx.x & 3] = 0;
        __syncthreads();
        if (__builtin_amdgcn_readfirstlane(threadIdx.x) >= kBlock) {  // a writer wave
            const uint32_t ht = threadIdx.x - kBlock, lane = ht & (kWave - 1);
            const uint32_t wv = __builtin_amdgcn_readfirstlane(ht / kWave);  // uniform: SGPR store bases
            const uint32_t hrow0 = blockIdx.x * kBlock;
            const uint32_t hi = hrow0 + ht < (uint32_t)p.n ? hrow0 + ht : (uint32_t)p.n - 1;  // shadows, as below
            const uint32_t hw0 = hrow0 + wv * kWave;
            const int hrows = (int)min((int64_t)kWave, max((int64_t)0, (int64_t)p.n - hw0));
            const uint32_t hslice = (uint32_t)hrows * (DD_OBS_DIM * 4);
            char* rew_p = p.reward;
            uint8_t* done_p = p.done;
            const float* obs_f = p.obs + (int64_t)hw0 * DD_OBS_DIM;
            const bool auto_reset = p.k.c.auto_reset;
            double total = at(a.total, hi);  // the running total is the writer's (kDefer)
            for (int f = 0; f < p.frames; ++f) {
                int spin = 0;
                for (; __builtin_amdgcn_readfirstlane(ctr_load(&ctr[0][wv])) <= f; ++spin) {
                    if (spin >= p.spin_cap) {  // the frame wave never produced frame f
                        raise_error(DD_ERR_HANDOVER);
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                }
                ctr_acquire();
                f32x4* slot = &stage[wv][f & 1][0][0];
                Lane s;
                uint32_t word;
                stage_get(slot, lane, s, word);
                asm volatile("" ::: "memory");  // every lane's reads issue before any row write
                s.status = word & ~kWasDone;
                const double reward = finish_deferred<T>(s, (word & kWasDone) != 0, auto_reset, total);
                put_out(reinterpret_cast<T*>(rew_p), hi, (T)reward);
                put_out(done_p, hi, (uint8_t)((s.status & DD_ST_DONE) ? 1 : 0));
                // the rows go where the slot's data was (read above, in order)
                float* rows = reinterpret_cast<float*>(slot);
                observe<false>(kRefConsts, s, rows + lane * DD_OBS_DIM);
                __syncwarp();
                HeldObs h;
                hold_obs_wave(rows, h);
                ctr_store(&ctr[1][wv], f + 1);  // after the reads of the slot
                store_held_wave(h, rsrc_over(obs_f, hslice));
                obs_f += p.n_total * DD_OBS_DIM;
                rew_p += p.reward_stride;
                done_p += p.n_total;
            }
            if (hrow0 + ht < (uint32_t)p.n) at(a.total, hi) = (T)total;
            return;
        }
    }
    const DDConfig& sw = p.k.c;
    const Consts& k = kRef ? kRefConsts : p.k;
    const uint32_t row0 = blockIdx.x * kBlock;
    const bool live = row0 + threadIdx.x < (uint32_t)p.n;
    // Lanes past n shadow lane n - 1: they load its state and action and
    // compute its values, so its per-frame stores from them write the same
    // bytes.  The frame loop then has no `live` branch (one basic block per
    // frame on the common path); only the final state store is guarded.
    const uint32_t i = live ? row0 + threadIdx.x : (uint32_t)p.n - 1;
    // this wave's first row, its row count and slice offset: wave-uniform, in SGPRs
    const uint32_t wrow0 = __builtin_amdgcn_readfirstlane(row0 + (threadIdx.x & ~(kWave - 1)));
    const int wrows = (int)min((int64_t)kWave, max((int64_t)0, (int64_t)p.n - wrow0));
    const int woff = (int)__builtin_amdgcn_readfirstlane((threadIdx.x & ~(kWave - 1)) * DD_OBS_DIM);
    const int roff = threadIdx.x * DD_OBS_DIM;                   // the lane's row in a tile
    const int64_t env = a.env_id_base + i;
    constexpr bool kGuard = !kRef && std::is_same<T, double>::value;
    HeldObs held;
    Lane s;
    // kShapePpo: the notebook reward's two-frame distance history, in registers
    double h0 = 0.0, h1 = 0.0;
    if constexpr (kShape == kShapePpo) { h0 = at(p.shaped_hist, i); h1 = at(p.shaped_hist + p.n_total, i); }
    load_dynamics(a, i, s);
    s.total = at(a.total, i);
    s.status = at(a.status, i);
    s.steps = at(a.steps, i);
    s.episode = at(a.episode, i);
    // Output streams as wave-uniform cursors advanced once per frame (SGPR
    // pairs: two scalar adds each, where recomputing base + f * stride took
    // six and the frame loop's SGPRs spilled), every store an SGPR base + the
    // lane's 32-bit offset.  obs_prev: frame f - 1's slice of this wave (its
    // range is empty at f = 0).
    char* rew_p = p.reward;
    uint8_t* done_p = p.done;
    char* erew_p = p.engine_reward;  // (advanced every frame: test has_engine, not the pointer)
    uint8_t* edone_p = p.engine_done;
    const bool has_engine = p.engine_reward != nullptr;
    const float* obs_prev = p.obs + ((int64_t)wrow0 - p.n_total) * DD_OBS_DIM;
    const uint32_t slice_bytes = (uint32_t)wrows * (DD_OBS_DIM * 4);
    uint32_t prev_bytes = 0;
    // Actions: raw buffer loads (buffer_action), prefetched two frames ahead
    // into two registers used in turn (the loop is unrolled by two, so no
    // register copy of a pending load); act_next is the byte offset of the
    // frame the next prefetch reads.
    // kActDw (bitmask actions under kHeld, whose launch condition includes a
    // 4-byte aligned action buffer and N % 4 == 0): the lane loads the
    // aligned dword holding its byte and extracts it where the frame uses it.
    // The prefetched value is then a plain 32-bit register; a loaded byte
    // crosses the loop's back edge as a 16-bit value whose widening (a
    // v_and 0xffff) the compiler placed at the loop latch, right behind the
    // pair's stores, and waited there for the load.
    constexpr bool kActDw = kHeld && AFMT == DD_ACT_BITMASK;
    constexpr uint32_t act_w = AFMT == DD_ACT_F32X3 ? 12u : AFMT == DD_ACT_U8X3 ? 3u : 1u;
    const __amdgpu_buffer_rsrc_t act_r = rsrc_over(p.actions, AFMT == DD_ACT_PHILOX ? 0u : p.act_bytes);
    const uint32_t act_lane = kActDw ? (i & ~3u) : i * act_w;
    const uint32_t act_sh = (i & 3u) * 8u;
    const uint32_t act_stride = (uint32_t)p.act_stride;
    uint32_t act_next = 0;
    uint32_t act0 = 0, act1 = 0;
    PhiloxActions pa;
    if constexpr (AFMT == DD_ACT_PHILOX) {
        act0 = rollout_action<AFMT>(p, env, 0, i, pa);
        act1 = rollout_action<AFMT>(p, env, 1, i, pa);
    } else if constexpr (kActDw) {
        act0 = __builtin_amdgcn_raw_buffer_load_b32(act_r, act_lane, 0, 0);
        act1 = __builtin_amdgcn_raw_buffer_load_b32(act_r, act_lane + act_stride, 0, 0);
        act_next = 2u * act_stride;
    } else {
        act0 = buffer_action<AFMT>(act_r, act_lane);
        act1 = buffer_action<AFMT>(act_r, act_lane + act_stride);
        act_next = 2u * act_stride;
    }
    // every prologue load lands here, not at a wait inside the frame loop
    asm volatile("" ::"v"(s.x), "v"(s.y), "v"(s.vx), "v"(s.vy), "v"(s.angle), "v"(s.omega), "v"(s.fuel),
                 "v"(s.px), "v"(s.py), "v"(s.total), "v"(s.status), "v"(s.steps), "v"(s.episode), "v"(act0),
                 "v"(act1));
    // auto_reset: the next episode's Philox block per lane (frame.h).  Not with
    // the in-kernel Philox actions, whose own blocks it competes with for
    // registers: there it cost 2-3 % (65,536 and 262,144 x 256), where with
    // action buffers it took 65,536 x 256 from 0.330 to 0.303 ms
    // (profiles/r04/lab/roll_spawn_ahead.jsonl)
    constexpr bool kAhead = AFMT != DD_ACT_PHILOX;
    SpawnAhead ahead;
    ThrustTrig tt;  // the thrust's sin / cos of the lane's current angle (frame.h next_trig)
    // One frame; kObs and kAuto (auto_reset) are compile-time so the loop
    // body carries no uniform branch on them.
    auto run_frame = [&](const int f, uint32_t& slot, auto obs_c, auto auto_c) __attribute__((always_inline)) {
        constexpr bool kObs = decltype(obs_c)::value, kAuto = decltype(auto_c)::value;
        int consumed = 0;
        if constexpr (kSplit) {
            consumed = ctr_load(&ctr[1][threadIdx.x / kWave]);  // used at the hand-over, at the frame's end
        } else if (kHeld && kObs) {
            __syncwarp();  // frame f - 1's rows (other lanes of this wave) are in LDS
            hold_obs_wave(tile[(f - 1) & 1] + woff, held);
        }
        const uint32_t act = kActDw ? __builtin_amdgcn_ubfe(slot, act_sh, 3) : slot;
        if constexpr (AFMT == DD_ACT_PHILOX) {
            slot = rollout_action<AFMT>(p, env, f + 2, i, pa);
        } else if constexpr (kActDw) {
            slot = __builtin_amdgcn_raw_buffer_load_b32(act_r, act_lane + act_next, 0, 0);
            act_next += act_stride;
        } else {
            slot = buffer_action<AFMT>(act_r, act_lane + act_next);
            act_next += act_stride;
        }
        double reward;
        const bool was_done = (s.status & DD_ST_DONE) != 0;
        auto fast = [&]() __attribute__((always_inline)) {
            return frame_checked<kRef, true, kSplit, true, T>(k, sw, act, s, &tt);  // kSplit: the writer finishes it
        };
        if constexpr (kAuto) {
            // next-step reset, fixed up after the frame: every lane runs the
            // frame (a done lane's result is discarded), and a wave with a lane
            // to re-spawn takes the one branch
            reward = fast();
            if (__ballot(was_done)) {
                if (was_done) {
                    if constexpr (kAhead) ahead.respawn(sw, k.c.max_fuel, env, s);
                    else spawn(sw, k.c.max_fuel, env, s);
                    reward = 0.0;
                    tt.s = 0.0;  // sin / cos of the spawn angle 0, as next_trig gives them
                    tt.c = 1.0;
                }
            }
        } else if (was_done) {  // sticky done (game_engine.py:107-111)
            measure(s);
            reward = 0.0;
        } else {
            reward = fast();
        }
        if constexpr (kShape != kShapeNone) {
            // dd_step's notebook path (finish_lane); kShapePpo: the history in
            // h0 / h1, slot steps & 1 holds the distance two frames back
            double v[13];
            observe_values<kGuard, true>(k, s, v);  // the notebook reward's doubles: exact quotients
            double shaped = 0.0;
            bool shaped_done;
            if (kAuto && was_done) {  // re-spawned: the history restarts (prev_state None)
                if constexpr (kShape == kShapePpo) {
                    h0 = v[9];
                    h1 = __builtin_nan("");
                }
                shaped_done = false;
            } else if (was_done) {  // sticky done
                shaped_done = true;
            } else {
                if constexpr (kShape == kShapePpo) {
                    const bool odd = (s.steps & 1) != 0;
                    shaped = notebook_reward(v, s.status, odd ? h1 : h0);
                    h1 = odd ? v[9] : h1;
                    h0 = odd ? h0 : v[9];
                } else {
                    shaped = reinforce_reward(v, s.status);
                }
                shaped_done = (s.status & DD_ST_DONE) != 0;
                if (p.max_steps > 0 && s.steps >= p.max_steps) {  // the collection loops' timeout
                    shaped = (s.status & DD_ST_LANDED) ? shaped : shaped - 500;
                    shaped_done = true;
                    s.status |= DD_ST_DONE;
                }
            }
            put_out(reinterpret_cast<T*>(rew_p), i, (T)shaped);
            put_out(done_p, i, (uint8_t)(shaped_done ? 1 : 0));
            if (has_engine) {
                put_out(reinterpret_cast<T*>(erew_p), i, (T)reward);
                put_out(edone_p, i, (uint8_t)((s.status & DD_ST_DONE) ? 1 : 0));
            }
        } else if constexpr (kSplit) {
            // hand frame f to the writer (the unrounded frame, as the obs below)
            const int wv = threadIdx.x / kWave;
            // slot f & 1 still holds frame f - 2
            for (int spin = 0; __builtin_amdgcn_readfirstlane(consumed) < f - 1; ++spin) {
                if (spin >= p.spin_cap) {  // the writer never finished frame f - 2
                    raise_error(DD_ERR_HANDOVER);
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
                consumed = ctr_load(&ctr[1][wv]);
            }
            ctr_acquire();
            stage_put(&stage[wv][f & 1][0][0], threadIdx.x & (kWave - 1), s, s.status | (was_done ? kWasDone : 0u));
            ctr_store(&ctr[0][wv], f + 1);
        } else {
            put_out(reinterpret_cast<T*>(rew_p), i, (T)reward);
            put_out(done_p, i, (uint8_t)((s.status & DD_ST_DONE) ? 1 : 0));
        }
        if constexpr (kObs && !kSplit) observe<kGuard>(k, s, tile[kHeld ? (f & 1) : 0] + roff);
        // the obs above sees the unrounded frame, like dd_step's
        quantize<T, kRef>(s);
        if constexpr (kObs && !kSplit) {
            if constexpr (kHeld) {
                store_held_wave(held, rsrc_over(obs_prev, prev_bytes));  // frame f - 1's rows
                prev_bytes = slice_bytes;
                obs_prev += p.n_total * DD_OBS_DIM;
            } else {
                flush_obs_wave(tile[0] + woff, p.obs + ((size_t)f * p.n_total + wrow0) * DD_OBS_DIM, wrows);
            }
        }
        rew_p += p.reward_stride;
        done_p += p.n_total;
        if constexpr (kShape != kShapeNone) {
            erew_p += p.reward_stride;
            edone_p += p.n_total;
        }
        if constexpr (kAuto && kAhead) ahead.refill(sw, env, s.episode, f);
    };
    auto run = [&](auto obs_c, auto auto_c) __attribute__((always_inline)) {
        if constexpr (decltype(auto_c)::value && kAhead) ahead.init(sw, env, s.episode);
        next_trig(s, tt);
        // an odd count leaves the loop between the pair's frames (`break`, not
        // a skipped second frame): the loop latch is then reached from one
        // path only, and the vmcnt the compiler derives there for the
        // prefetched actions counts every store the pair issued
        for (int f = 0; f < p.frames; f += 2) {
            run_frame(f, act0, obs_c, auto_c);
            if (f + 1 >= p.frames) break;
            run_frame(f + 1, act1, obs_c, auto_c);
        }
    };
    using yes = std::true_type;
    using no = std::false_type;
    if (kSplit || p.obs) {  // (kSplit: launched with obs; the writers wait for every frame)
        if (sw.auto_reset) run(yes{}, yes{});
        else run(yes{}, no{});
    } else {
        if (sw.auto_reset) run(no{}, yes{});
        else run(no{}, no{});
    }
    if (!kSplit && kHeld && p.obs && p.frames > 0) {  // the last frame's slice
        const int f = p.frames - 1;
        __syncwarp();
        hold_obs_wave(tile[f & 1] + woff, held);
        store_held_wave(held, rsrc_over(obs_prev, slice_bytes));
    }
    if (live) {
        // every field (lanes may have re-spawned); kSplit: not the total, the writer's
        store_spawn<T, !kSplit>(reload_soa<RolloutArgs, T>(), i, s);
        if constexpr (kShape == kShapePpo) { at(p.shaped_hist, i) = h0; at(p.shaped_hist + p.n_total, i) = h1; }
    }
}

// dd_selftest_sqrt kernel: trig::sqrt_unscaled against the compiler's sqrt()
// on doubles from 2^-767 up, drawn with a uniform exponent (Philox bits: 11
// exponent bits folded into [255, 2047), 52 random mantissa bits), plus the
// integers 0..2^20 (spawn distances) at the start of the range; counts the
// inputs whose results differ in any bit.
__global__ __launch_bounds__(kBlock) void sqrt_selftest_kernel(uint64_t seed, uint64_t first, int64_t len,
                                                               unsigned long long* mismatches) {
    const uint64_t t = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    uint32_t r[4];
    philox4x32_10((uint32_t)(first + 4 * t), (uint32_t)((first + 4 * t) >> 32), 0x5a17u, 0u, (uint32_t)seed,
                  (uint32_t)(seed >> 32), r);
    int bad = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint64_t idx = 4 * t + q;
        if ((int64_t)idx >= len) break;
        const uint64_t g = first + idx;
        double x;
        if (g <= (1u << 20)) {
            x = (double)g;
        } else {
            const uint32_t hi = r[q], lo = r[(q + 1) & 3] ^ r[(q + 2) & 3];
            const uint64_t exp = 256u + (hi >> 21) % 1791u;  // [256, 2047): 2^-767 .. below inf
            const uint64_t mant = ((uint64_t)(hi & 0xfffffu) << 32) | lo;
            x = __builtin_bit_cast(double, (exp << 52) | mant);
        }
        const double a = sqrt(x), b = trig::sqrt_unscaled(x);
        bad += __builtin_bit_cast(uint64_t, a) != __builtin_bit_cast(uint64_t, b);
    }
    const uint64_t m = __ballot(bad != 0);
    if (m) {
        int total = bad;
        for (int off = 32; off > 0; off >>= 1) total += __shfl_xor(total, off);
        if ((threadIdx.x & (kWave - 1)) == __ffsll((unsigned long long)m) - 1) atomicAdd(mismatches, (unsigned long long)total);
    }
}

// dd_stamp kernel: one lane stores the GPU's constant-rate wall clock
// (s_memrealtime) with a vector store.  Captured into a hipGraph beside the
// step kernels it marks where the graph reaches that point (bench.py).
__global__ __launch_bounds__(kWave) void stamp_kernel(unsigned long long* slot) {
    const unsigned long long t = (unsigned long long)wall_clock64();
    if (threadIdx.x == 0) *slot = t;
}

// dd_shaped_reset kernel: the notebook reward's history restarts from the
// current state (slot 0 = its distance, slot 1 = none).
template <typename T>
__global__ __launch_bounds__(kBlock) void shaped_reset_kernel(Consts k, Soa<T> a, const uint8_t* mask,
                                                              double* hist, int64_t stride, int32_t n) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= (uint32_t)n) return;
    if (mask && !at(mask, i)) return;
    Lane s;
    load_dynamics(a, i, s);
    measure(s);
    at(hist, i) = trig::div_exact(s.dist, k.c.world_width, k.inv_w);
    at(hist + stride, i) = __builtin_nan("");
}

// dd_reset kernel: masked re-spawn (+ optional reset observation).
template <typename T>
__global__ __launch_bounds__(kBlock) void reset_kernel(Consts k, Soa<T> a, const uint8_t* mask,
                                                       float* obs, int32_t n) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= (uint32_t)n) return;
    if (mask && !at(mask, i)) return;
    Lane s;
    s.episode = at(a.episode, i);
    spawn(k.c, k.c.max_fuel, a.env_id_base + i, s);
    store_spawn(a, i, s);
    if (obs) observe(k, s, obs + (size_t)i * DD_OBS_DIM);
}

// dd_write_obs kernel: observation of the current state, LDS-staged.
template <typename T>
__global__ __launch_bounds__(kBlock) void obs_kernel(Consts k, Soa<T> a, float* obs, int32_t n) {
    __shared__ __attribute__((aligned(16))) float tile[kBlock * DD_OBS_DIM];
    const uint32_t row0 = blockIdx.x * kBlock;
    const uint32_t i = row0 + threadIdx.x;
    if (i < (uint32_t)n) {
        Lane s;
        load_dynamics(a, i, s);
        s.status = at(a.status, i);
        measure(s);
        observe(k, s, tile + threadIdx.x * DD_OBS_DIM);
    }
    __syncthreads();
    const int rows = (int)min((uint32_t)kBlock, (uint32_t)n - row0);
    flush_obs_tile(tile, obs + (size_t)row0 * DD_OBS_DIM, rows);
}

// dd_get_info kernel: pixel distance and speed (game_engine.py:292-296).
template <typename T>
__global__ __launch_bounds__(kBlock) void info_kernel(Soa<T> a, T* distance, T* speed, int32_t n) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= (uint32_t)n) return;
    const double x = at(a.x, i), y = at(a.y, i), vx = at(a.vx, i), vy = at(a.vy, i);
    const double dx = (double)at(a.px, i) - x, dy = (double)at(a.py, i) - y;
    if (distance) at(distance, i) = (T)sqrt(dx * dx + dy * dy);
    if (speed) at(speed, i) = (T)sqrt(vx * vx + vy * vy);
}

// ---------------------------------------------------------------------------
// dd_gae: one lane per env walks its column of the [T][N] rollout backwards.
// The loads of a frame do not depend on the running gae, so the compiler
// keeps several frames' loads in flight (unroll 4).  Float32 throughout, in
// compute_gae's order: torch evaluates `gamma * v` with gamma rounded to
// float32 and `gamma * lambda_` in Python doubles before that rounding.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void gae_kernel(const float* __restrict__ rewards,
                                                     const float* __restrict__ values,
                                                     const uint8_t* __restrict__ dones, float* __restrict__ adv,
                                                     float* __restrict__ ret, int32_t T, int64_t n, float g,
                                                     float gl) {
    // Frames are processed in groups of kG: the group's loads are all issued
    // before its (serial) arithmetic, so kG loads per array are in flight.
    constexpr int kG = 8;
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    float gae = 0.0f;
    float v_next = values[(int64_t)T * n + i];
    int32_t t = T - 1;
    for (; t >= kG - 1; t -= kG) {
        float r[kG], v[kG], d[kG];
#pragma unroll
        for (int j = 0; j < kG; ++j) {
            const int64_t o = (int64_t)(t - j) * n + i;
            r[j] = rewards[o];
            v[j] = values[o];
            d[j] = (float)dones[o];
        }
#pragma unroll
        for (int j = 0; j < kG; ++j) {
            const int64_t o = (int64_t)(t - j) * n + i;
            const float mask = 1.0f - d[j];
            const float delta = (r[j] + (g * v_next) * mask) - v[j];
            gae = delta + (gl * mask) * gae;
            __builtin_nontemporal_store(gae, adv + o);
            if (ret) __builtin_nontemporal_store(gae + v[j], ret + o);
            v_next = v[j];
        }
    }
    for (; t >= 0; --t) {
        const int64_t o = (int64_t)t * n + i;
        const float v = values[o];
        const float mask = 1.0f - (float)dones[o];
        const float delta = (rewards[o] + (g * v_next) * mask) - v;
        gae = delta + (gl * mask) * gae;
        __builtin_nontemporal_store(gae, adv + o);
        if (ret) __builtin_nontemporal_store(gae + v, ret + o);
        v_next = v;
    }
}

// ---------------------------------------------------------------------------
// Ordered compaction (dd_compact): count per tile -> exclusive scan of tile
// counts -> scatter in lane order.  Ballots give each wave its count and each
// lane its rank; LDS combines the block's four waves.
// ---------------------------------------------------------------------------
__device__ __forceinline__ bool want_flag(const uint8_t* flags, int32_t want, int64_t i, int64_t n) {
    return i < n && ((flags[i] != 0) == (want != 0));
}

__global__ __launch_bounds__(kBlock) void compact_count_kernel(const uint8_t* flags, int32_t want,
                                                               int32_t* tile_counts, int64_t n) {
    __shared__ int wave_cnt[kBlock / kWave];
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    const uint64_t m = __ballot(want_flag(flags, want, i, n));
    if ((threadIdx.x & (kWave - 1)) == 0) wave_cnt[threadIdx.x / kWave] = __popcll(m);
    __syncthreads();
    if (threadIdx.x == 0) {
        int sum = 0;
        for (int w = 0; w < kBlock / kWave; ++w) sum += wave_cnt[w];
        tile_counts[blockIdx.x] = sum;
    }
}

// Single-block exclusive scan over `m` tile counts; total goes to *count.
__global__ __launch_bounds__(1024) void compact_scan_kernel(int32_t* tile_counts, int64_t m, int32_t* count) {
    __shared__ int32_t part[1024];
    __shared__ int32_t carry;
    if (threadIdx.x == 0) carry = 0;
    __syncthreads();
    for (int64_t base = 0; base < m; base += 1024) {
        const int64_t j = base + threadIdx.x;
        const int32_t v = j < m ? tile_counts[j] : 0;
        part[threadIdx.x] = v;
        __syncthreads();
        for (int off = 1; off < 1024; off <<= 1) {  // Hillis-Steele inclusive scan
            const int32_t add = threadIdx.x >= (unsigned)off ? part[threadIdx.x - off] : 0;
            __syncthreads();
            part[threadIdx.x] += add;
            __syncthreads();
        }
        if (j < m) tile_counts[j] = carry + part[threadIdx.x] - v;
        __syncthreads();
        if (threadIdx.x == 1023) carry += part[1023];
        __syncthreads();
    }
    if (threadIdx.x == 0) *count = carry;
}

__global__ __launch_bounds__(kBlock) void compact_scatter_kernel(const uint8_t* flags, int32_t want,
                                                                 const int32_t* tile_offsets,
                                                                 int32_t* idx_out, int64_t n) {
    __shared__ int wave_off[kBlock / kWave];
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    const bool keep = want_flag(flags, want, i, n);
    const uint64_t m = __ballot(keep);
    const int w = threadIdx.x / kWave;
    if ((threadIdx.x & (kWave - 1)) == 0) wave_off[w] = __popcll(m);
    __syncthreads();
    if (threadIdx.x == 0) {
        int run = tile_offsets[blockIdx.x];
        for (int k = 0; k < kBlock / kWave; ++k) { const int c = wave_off[k]; wave_off[k] = run; run += c; }
    }
    __syncthreads();
    if (keep) {
        const int rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
        idx_out[wave_off[w] + rank] = (int32_t)i;
    }
}

#ifdef DD_ISA_PROBE
// tools/lab/isa_probe.sh: one kernel instantiation alone (device assembly in
// seconds instead of the whole library's minutes), for reading its ISA.
#define DD_PROBE_KERNEL_(k) template __global__ void k;
DD_PROBE_KERNEL_(DD_ISA_PROBE)
}  // namespace dd
#else
// ---------------------------------------------------------------------------
// Host side: argument checks, chunking and launches.
// ---------------------------------------------------------------------------
inline int64_t tiles_of(int64_t n) { return (n + kBlock - 1) / kBlock; }

// The notebook reward a call asks for (frame.h kShape*): REINFORCE's by its
// mode, PPO's when the history pointer is set, else none.
inline int shape_of(int32_t shaped_mode, const void* shaped_hist, const void* shaped_reward) {
    if (shaped_mode == DD_SHAPED_REINFORCE) return kShapeReinforce;
    return shaped_hist || shaped_reward ? kShapePpo : kShapeNone;
}

template <typename T, int AFMT, bool kRef, int kShape>
void launch_step(const StepArgs& p, const Soa<T>& a, const Soa<T>* o, hipStream_t s) {
    const unsigned blocks = (unsigned)((p.n + kStepBlock - 1) / kStepBlock);
    if (o)
        hipLaunchKernelGGL((step_pp_kernel<T, AFMT, kRef, kShape>), dim3(blocks), dim3(kStepBlock), 0, s, p, a, *o);
    else
        hipLaunchKernelGGL((step_kernel<T, AFMT, kRef, kShape>), dim3(blocks), dim3(kStepBlock), 0, s, p, a);
}

template <typename T, bool kRef, int kShape>
void launch_step_fmt(const StepArgs& p, int afmt, const Soa<T>& a, const Soa<T>* o, hipStream_t s) {
    switch (afmt) {
        case DD_ACT_BITMASK: launch_step<T, DD_ACT_BITMASK, kRef, kShape>(p, a, o, s); break;
        case DD_ACT_F32X3: launch_step<T, DD_ACT_F32X3, kRef, kShape>(p, a, o, s); break;
        default: launch_step<T, DD_ACT_U8X3, kRef, kShape>(p, a, o, s); break;
    }
}

template <typename T, bool kRef>
void launch_step_shape(const StepArgs& p, int shape, int afmt, const Soa<T>& a, const Soa<T>* o, hipStream_t s) {
    switch (shape) {
        case kShapeNone: launch_step_fmt<T, kRef, kShapeNone>(p, afmt, a, o, s); break;
        case kShapePpo: launch_step_fmt<T, kRef, kShapePpo>(p, afmt, a, o, s); break;
        default: launch_step_fmt<T, kRef, kShapeReinforce>(p, afmt, a, o, s); break;
    }
}

template <typename T>
void step_chunks(StepArgs p, const DDState& st, const DDStepIO& io, int64_t n, hipStream_t s) {
    const bool ref = uses_reference_physics(p.k.c);
    const int shape = shape_of(io.shaped_mode, io.shaped_hist, io.shaped_reward);
    const int64_t act_w = io.action_format == DD_ACT_F32X3 ? 12 : io.action_format == DD_ACT_U8X3 ? 3 : 1;
    for (int64_t first = 0; first < n; first += kChunk) {
        const int64_t len = n - first < kChunk ? n - first : kChunk;
        p.actions = static_cast<const char*>(io.actions) + first * act_w;
        p.reward = static_cast<T*>(io.reward) + first;
        p.done = io.done + first;
        p.obs = io.obs ? io.obs + first * DD_OBS_DIM : nullptr;
        p.n = (int32_t)len;
        p.idx_base = (int32_t)first;
        p.shaped_hist = shape == kShapePpo ? io.shaped_hist + first : nullptr;
        p.hist_stride = n;
        p.shaped_reward = shape != kShapeNone ? static_cast<void*>(static_cast<T*>(io.shaped_reward) + first) : nullptr;
        p.shaped_done = shape != kShapeNone ? io.shaped_done + first : nullptr;
        p.max_steps = io.max_steps;
        const Soa<T> a = soa_of<T>(st, first);
        Soa<T> o;
        if (io.state_out) o = soa_of<T>(*io.state_out, first);
        if (ref) launch_step_shape<T, true>(p, shape, io.action_format, a, io.state_out ? &o : nullptr, s);
        else launch_step_shape<T, false>(p, shape, io.action_format, a, io.state_out ? &o : nullptr, s);
    }
}

// The split rollout (rollout_kernel's kSplit) when the launch is one block per
// CU or fewer: its block takes 8 waves of ~256 registers, all of a CU's
// register file for 256 drones, where the single-role kernel fits two blocks
// (262,144 drones: 4 rounds of split blocks against 2 of single-role ones).
inline bool split_rollout_fits(unsigned blocks) {
    static int cus[64] = {};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return false;
    if (cus[dev] == 0 && hipDeviceGetAttribute(&cus[dev], hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        return false;
    return blocks <= (unsigned)cus[dev];
}

// Which rollout kernel a launch of n lanes takes (DD_ROLLOUT_*): the held
// observation path needs every frame row start 16-byte aligned and (bitmask
// actions) a 4-byte aligned action buffer for its dword loads; the split
// kernel covers the reference world's held path with the engine reward.
inline int rollout_kernel_for(bool ref, int shape, int afmt, const void* actions, const float* obs, int64_t n_total,
                              int64_t n, int32_t choice) {
    const bool held = (reinterpret_cast<uintptr_t>(obs) & 15u) == 0 && (n_total & 3) == 0 &&
                      (afmt != DD_ACT_BITMASK || (reinterpret_cast<uintptr_t>(actions) & 3u) == 0);
    if (ref && shape == kShapeNone && held && obs && choice != DD_ROLLOUT_SINGLE &&
        split_rollout_fits((unsigned)tiles_of(n)))
        return DD_ROLLOUT_SPLIT;
    return held ? DD_ROLLOUT_HELD : DD_ROLLOUT_FLUSHED;
}

template <typename T, int AFMT, bool kRef, int kShape>
void launch_rollout(const RolloutArgs& p, int kind, const Soa<T>& a, hipStream_t s) {
    const unsigned blocks = (unsigned)tiles_of(p.n);
    if constexpr (kRef && kShape == kShapeNone) {
        if (kind == DD_ROLLOUT_SPLIT) {
            hipLaunchKernelGGL((rollout_kernel<T, AFMT, true, true, kShapeNone, true>), dim3(blocks), dim3(2 * kBlock),
                               0, s, p, a);
            return;
        }
    }
    if (kind != DD_ROLLOUT_FLUSHED)
        hipLaunchKernelGGL((rollout_kernel<T, AFMT, kRef, true, kShape>), dim3(blocks), dim3(kBlock), 0, s, p, a);
    else
        hipLaunchKernelGGL((rollout_kernel<T, AFMT, kRef, false, kShape>), dim3(blocks), dim3(kBlock), 0, s, p, a);
}

template <typename T, bool kRef, int kShape>
void launch_rollout_fmt(const RolloutArgs& p, int kind, int afmt, const Soa<T>& a, hipStream_t s) {
    switch (afmt) {
        case DD_ACT_BITMASK: launch_rollout<T, DD_ACT_BITMASK, kRef, kShape>(p, kind, a, s); break;
        case DD_ACT_F32X3: launch_rollout<T, DD_ACT_F32X3, kRef, kShape>(p, kind, a, s); break;
        case DD_ACT_U8X3: launch_rollout<T, DD_ACT_U8X3, kRef, kShape>(p, kind, a, s); break;
        default: launch_rollout<T, DD_ACT_PHILOX, kRef, kShape>(p, kind, a, s); break;
    }
}

template <typename T, bool kRef>
void launch_rollout_shape(const RolloutArgs& p, int kind, int shape, int afmt, const Soa<T>& a, hipStream_t s) {
    switch (shape) {
        case kShapeNone: launch_rollout_fmt<T, kRef, kShapeNone>(p, kind, afmt, a, s); break;
        case kShapePpo: launch_rollout_fmt<T, kRef, kShapePpo>(p, kind, afmt, a, s); break;
        default: launch_rollout_fmt<T, kRef, kShapeReinforce>(p, kind, afmt, a, s); break;
    }
}

template <typename T>
void rollout_chunks(RolloutArgs p, const DDState& st, const DDRolloutIO& io, int64_t n, hipStream_t s) {
    const bool ref = uses_reference_physics(p.k.c);
    const int shape = shape_of(io.shaped_mode, io.shaped_hist, nullptr);
    const int64_t act_w = io.action_format == DD_ACT_F32X3 ? 12 : io.action_format == DD_ACT_U8X3 ? 3
                        : io.action_format == DD_ACT_BITMASK ? 1 : 0;
    p.act_stride = n * act_w;
    p.reward_stride = n * (int64_t)sizeof(T);
    p.n_total = n;
    p.spin_cap = io.kernel == DD_ROLLOUT_SPLIT_NO_WAIT ? 0 : kSpinCap;
    const int32_t frames = p.frames;
    const int64_t step0 = p.action_step;
    for (int64_t first = 0; first < n; first += kChunk) {
        const int64_t len = n - first < kChunk ? n - first : kChunk;
        // The kernel reads actions by raw buffer loads with 32-bit offsets
        // (buffer_action): a launch covers as many frames as keep every
        // consumed offset, (frames - 1) x stride + len x width, below 2^32,
        // and the state goes through memory between such launches (the same
        // frames either way: the rollout equals its frames' dd_step calls).
        int64_t fg = frames;
        if (act_w > 0 && (fg - 1) * p.act_stride + len * act_w > (int64_t)UINT32_MAX)
            fg = 1 + (((int64_t)UINT32_MAX - len * act_w) / p.act_stride);
        for (int64_t g0 = 0; g0 < frames; g0 += fg) {
            const int64_t ng = frames - g0 < fg ? frames - g0 : fg;
            p.frames = (int32_t)ng;
            p.action_step = step0 + g0;
            p.actions = io.actions ? static_cast<const char*>(io.actions) + g0 * p.act_stride + first * act_w : nullptr;
            // every byte the range check admits lies in the caller's buffer
            const int64_t extent = (ng - 1) * p.act_stride + (n - first) * act_w;
            p.act_bytes = (uint32_t)(extent < (int64_t)UINT32_MAX ? extent : (int64_t)UINT32_MAX);
            p.reward = reinterpret_cast<char*>(static_cast<T*>(io.reward) + g0 * n + first);
            p.done = io.done + g0 * n + first;
            p.obs = io.obs ? io.obs + (g0 * n + first) * DD_OBS_DIM : nullptr;
            p.n = (int32_t)len;
            p.shaped_hist = shape == kShapePpo ? io.shaped_hist + first : nullptr;
            p.engine_reward = shape != kShapeNone && io.engine_reward
                                  ? reinterpret_cast<char*>(static_cast<T*>(io.engine_reward) + g0 * n + first) : nullptr;
            p.engine_done = shape != kShapeNone && io.engine_reward ? io.engine_done + g0 * n + first : nullptr;
            p.max_steps = io.max_steps;
            const Soa<T> a = soa_of<T>(st, first);
            const int kind = rollout_kernel_for(ref, shape, io.action_format, p.actions, p.obs, n, len, io.kernel);
            if (ref) launch_rollout_shape<T, true>(p, kind, shape, io.action_format, a, s);
            else launch_rollout_shape<T, false>(p, kind, shape, io.action_format, a, s);
        }
    }
}

int finish() { return (int)hipGetLastError(); }

}  // namespace dd

extern "C" {

void dd_config_default(DDConfig* c) {
    if (c) *c = dd::reference_config();
}

int dd_step(const DDConfig* cfg, const DDState* st, const DDStepIO* io, int64_t n, void* stream) {
    if (!cfg || !io || !st || n < 0 || n > INT32_MAX) return hipErrorInvalidValue;
    if (io->action_format < DD_ACT_BITMASK || io->action_format > DD_ACT_U8X3) return hipErrorInvalidValue;
    if (st->precision != DD_F32 && st->precision != DD_F64) return hipErrorInvalidValue;
    if (io->done_idx && !io->done_count) return hipErrorInvalidValue;
    if (io->shaped_mode == DD_SHAPED_REINFORCE) {  // no history: shaped_hist is not read
        if (!io->shaped_reward || !io->shaped_done) return hipErrorInvalidValue;
    } else if (io->shaped_mode == DD_SHAPED_PPO) {
        const int ptrs = (io->shaped_hist != nullptr) + (io->shaped_reward != nullptr) + (io->shaped_done != nullptr);
        if (ptrs != 0 && ptrs != 3) return hipErrorInvalidValue;
    } else {
        return hipErrorInvalidValue;
    }
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (io->done_count) {
        const hipError_t e = hipMemsetAsync(io->done_count, 0, sizeof(int32_t), s);
        if (e != hipSuccess) return (int)e;
    }
    if (n == 0) return 0;  // empty batch: pointers may be null
    if (!dd::state_ok(st) || !io->actions || !io->reward || !io->done) return hipErrorInvalidValue;
    if (const DDState* so = io->state_out) {  // ping-pong: the shared fields, distinct per-frame arrays
        if (!dd::state_ok(so) || so->precision != st->precision || so->env_id_base != st->env_id_base ||
            so->px != st->px || so->py != st->py || so->status != st->status || so->episode != st->episode)
            return hipErrorInvalidValue;
        const void* in[9] = {st->x, st->y, st->vx, st->vy, st->angle, st->omega, st->fuel, st->total_reward,
                             st->steps};
        const void* out[9] = {so->x, so->y, so->vx, so->vy, so->angle, so->omega, so->fuel, so->total_reward,
                              so->steps};
        for (int q = 0; q < 9; ++q)
            if (in[q] == out[q]) return hipErrorInvalidValue;
    }
    dd::StepArgs p{};
    p.k = dd::make_consts(*cfg);
    p.done_idx = io->done_idx;
    p.done_count = io->done_count;
    if (st->precision == DD_F32) dd::step_chunks<float>(p, *st, *io, n, s);
    else dd::step_chunks<double>(p, *st, *io, n, s);
    return dd::finish();
}

int dd_rollout(const DDConfig* cfg, const DDState* st, const DDRolloutIO* io, int64_t n, void* stream) {
    if (!cfg || !io || !st || n < 0 || n > INT32_MAX || io->frames < 0) return hipErrorInvalidValue;
    if (io->action_format < DD_ACT_BITMASK || io->action_format > DD_ACT_PHILOX) return hipErrorInvalidValue;
    if (st->precision != DD_F32 && st->precision != DD_F64) return hipErrorInvalidValue;
    if (n == 0 || io->frames == 0) return 0;
    if (!dd::state_ok(st) || !io->reward || !io->done) return hipErrorInvalidValue;
    if (io->action_format != DD_ACT_PHILOX && !io->actions) return hipErrorInvalidValue;
    if ((io->engine_reward != nullptr) != (io->engine_done != nullptr)) return hipErrorInvalidValue;
    if (io->shaped_mode != DD_SHAPED_PPO && io->shaped_mode != DD_SHAPED_REINFORCE) return hipErrorInvalidValue;
    if (io->engine_reward && dd::shape_of(io->shaped_mode, io->shaped_hist, nullptr) == dd::kShapeNone)
        return hipErrorInvalidValue;
    if (io->kernel < DD_ROLLOUT_AUTO || io->kernel > DD_ROLLOUT_SPLIT_NO_WAIT) return hipErrorInvalidValue;
    hipStream_t s = static_cast<hipStream_t>(stream);
    dd::RolloutArgs p{};
    p.k = dd::make_consts(*cfg);
    p.frames = io->frames;
    p.action_seed = io->action_seed;
    p.action_step = io->action_step;
    if (st->precision == DD_F32) dd::rollout_chunks<float>(p, *st, *io, n, s);
    else dd::rollout_chunks<double>(p, *st, *io, n, s);
    return dd::finish();
}

int dd_rollout_kernel(const DDConfig* cfg, const DDState* st, const DDRolloutIO* io, int64_t n) {
    if (!cfg || !io || !st || n <= 0 || n > INT32_MAX) return -1;
    const int64_t len = n < dd::kChunk ? n : dd::kChunk;
    return dd::rollout_kernel_for(dd::uses_reference_physics(*cfg), dd::shape_of(io->shaped_mode, io->shaped_hist, nullptr),
                                  io->action_format, io->actions, io->obs, n, len, io->kernel);
}

int dd_device_errors(uint32_t* bits, int32_t clear) {
    if (!bits) return hipErrorInvalidValue;
    // every stream's work first: torch's side streams do not synchronise with
    // the null stream, so a launch still running there could set its bit
    // after this read and be blamed on a later check
    hipError_t e = hipDeviceSynchronize();
    if (e != hipSuccess) return (int)e;
    e = hipMemcpyFromSymbol(bits, HIP_SYMBOL(dd::dd_error_bits), sizeof(uint32_t), 0, hipMemcpyDeviceToHost);
    if (e == hipSuccess && clear) {
        static const uint32_t zero = 0;
        e = hipMemcpyToSymbol(HIP_SYMBOL(dd::dd_error_bits), &zero, sizeof(uint32_t), 0, hipMemcpyHostToDevice);
    }
    return (int)e;
}

int dd_reset(const DDConfig* cfg, const DDState* st, const uint8_t* mask, float* obs, int64_t n, void* stream) {
    if (!cfg || !st || n < 0 || n > INT32_MAX) return hipErrorInvalidValue;
    if (n == 0) return 0;
    if (!dd::state_ok(st)) return hipErrorInvalidValue;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const dd::Consts k = dd::make_consts(*cfg);
    for (int64_t first = 0; first < n; first += dd::kChunk) {
        const int32_t len = (int32_t)(n - first < dd::kChunk ? n - first : dd::kChunk);
        const dim3 g((unsigned)dd::tiles_of(len)), b(dd::kBlock);
        const uint8_t* m = mask ? mask + first : nullptr;
        float* o = obs ? obs + first * DD_OBS_DIM : nullptr;
        if (st->precision == DD_F32)
            hipLaunchKernelGGL(dd::reset_kernel<float>, g, b, 0, s, k, dd::soa_of<float>(*st, first), m, o, len);
        else
            hipLaunchKernelGGL(dd::reset_kernel<double>, g, b, 0, s, k, dd::soa_of<double>(*st, first), m, o, len);
    }
    return dd::finish();
}

int dd_shaped_reset(const DDConfig* cfg, const DDState* st, const uint8_t* mask, double* hist, int64_t n,
                    void* stream) {
    if (!cfg || !st || n < 0 || n > INT32_MAX) return hipErrorInvalidValue;
    if (n == 0) return 0;
    if (!hist || !dd::state_ok(st)) return hipErrorInvalidValue;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const dd::Consts k = dd::make_consts(*cfg);
    for (int64_t first = 0; first < n; first += dd::kChunk) {
        const int32_t len = (int32_t)(n - first < dd::kChunk ? n - first : dd::kChunk);
        const dim3 g((unsigned)dd::tiles_of(len)), b(dd::kBlock);
        const uint8_t* m = mask ? mask + first : nullptr;
        if (st->precision == DD_F32)
            hipLaunchKernelGGL(dd::shaped_reset_kernel<float>, g, b, 0, s, k, dd::soa_of<float>(*st, first), m,
                               hist + first, n, len);
        else
            hipLaunchKernelGGL(dd::shaped_reset_kernel<double>, g, b, 0, s, k, dd::soa_of<double>(*st, first), m,
                               hist + first, n, len);
    }
    return dd::finish();
}

int dd_write_obs(const DDConfig* cfg, const DDState* st, float* obs, int64_t n, void* stream) {
    if (!cfg || !st || n < 0 || n > INT32_MAX) return hipErrorInvalidValue;
    if (n == 0) return 0;
    if (!obs || !dd::state_ok(st)) return hipErrorInvalidValue;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const dd::Consts k = dd::make_consts(*cfg);
    for (int64_t first = 0; first < n; first += dd::kChunk) {
        const int32_t len = (int32_t)(n - first < dd::kChunk ? n - first : dd::kChunk);
        const dim3 g((unsigned)dd::tiles_of(len)), b(dd::kBlock);
        float* o = obs + first * DD_OBS_DIM;
        if (st->precision == DD_F32)
            hipLaunchKernelGGL(dd::obs_kernel<float>, g, b, 0, s, k, dd::soa_of<float>(*st, first), o, len);
        else
            hipLaunchKernelGGL(dd::obs_kernel<double>, g, b, 0, s, k, dd::soa_of<double>(*st, first), o, len);
    }
    return dd::finish();
}

int dd_get_info(const DDConfig* cfg, const DDState* st, void* distance, void* speed, int64_t n, void* stream) {
    if (!cfg || !st || n < 0 || n > INT32_MAX) return hipErrorInvalidValue;
    if (n == 0 || (!distance && !speed)) return 0;
    if (!dd::state_ok(st)) return hipErrorInvalidValue;
    hipStream_t s = static_cast<hipStream_t>(stream);
    for (int64_t first = 0; first < n; first += dd::kChunk) {
        const int32_t len = (int32_t)(n - first < dd::kChunk ? n - first : dd::kChunk);
        const dim3 g((unsigned)dd::tiles_of(len)), b(dd::kBlock);
        if (st->precision == DD_F32)
            hipLaunchKernelGGL(dd::info_kernel<float>, g, b, 0, s, dd::soa_of<float>(*st, first),
                               distance ? (float*)distance + first : nullptr,
                               speed ? (float*)speed + first : nullptr, len);
        else
            hipLaunchKernelGGL(dd::info_kernel<double>, g, b, 0, s, dd::soa_of<double>(*st, first),
                               distance ? (double*)distance + first : nullptr,
                               speed ? (double*)speed + first : nullptr, len);
    }
    return dd::finish();
}

int dd_gae(const float* rewards, const float* values, const uint8_t* dones, float* advantages, float* returns,
           int64_t T, int64_t n, double gamma, double lambda, void* stream) {
    if (T < 0 || n < 0 || T > INT32_MAX) return hipErrorInvalidValue;
    if (T == 0 || n == 0) return 0;
    if (!rewards || !values || !dones || !advantages) return hipErrorInvalidValue;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const float g = (float)gamma;
    const float gl = (float)(gamma * lambda);
    hipLaunchKernelGGL(dd::gae_kernel, dim3((unsigned)dd::tiles_of(n)), dim3(dd::kBlock), 0, s, rewards, values,
                       dones, advantages, returns, (int32_t)T, n, g, gl);
    return dd::finish();
}

int dd_selftest_sqrt(uint64_t seed, int64_t n, unsigned long long* mismatches, void* stream) {
    if (n < 0 || n > ((int64_t)1 << 40) || !mismatches) return hipErrorInvalidValue;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const int64_t per = (int64_t)dd::kBlock * 4096;  // lanes per launch; 4 draws per lane
    for (int64_t first = 0; first < n; first += per * 4) {
        const int64_t len = n - first < per * 4 ? n - first : per * 4;
        const unsigned blocks = (unsigned)dd::tiles_of((len + 3) / 4);
        hipLaunchKernelGGL(dd::sqrt_selftest_kernel, dim3(blocks), dim3(dd::kBlock), 0, s, seed,
                           (uint64_t)first, len, mismatches);
    }
    return dd::finish();
}

int dd_stamp(unsigned long long* slot, void* stream) {
    if (!slot) return hipErrorInvalidValue;
    hipLaunchKernelGGL(dd::stamp_kernel, dim3(1), dim3(dd::kWave), 0, static_cast<hipStream_t>(stream), slot);
    return dd::finish();
}

int dd_wall_clock_khz(int* khz) {
    if (!khz) return hipErrorInvalidValue;
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e == hipSuccess) e = hipDeviceGetAttribute(khz, hipDeviceAttributeWallClockRate, dev);
    return (int)e;
}

int64_t dd_compact_workspace(int64_t n) { return n <= 0 ? 1 : dd::tiles_of(n); }

int dd_compact(const uint8_t* flags, int32_t want, int32_t* idx_out, int32_t* count, int32_t* workspace,
               int64_t n, void* stream) {
    if (n < 0 || n > INT32_MAX || !count || (n > 0 && (!flags || !idx_out || !workspace)))
        return hipErrorInvalidValue;
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (n == 0) return (int)hipMemsetAsync(count, 0, sizeof(int32_t), s);
    const int64_t m = dd::tiles_of(n);
    hipLaunchKernelGGL(dd::compact_count_kernel, dim3((unsigned)m), dim3(dd::kBlock), 0, s, flags, want,
                       workspace, n);
    hipLaunchKernelGGL(dd::compact_scan_kernel, dim3(1), dim3(1024), 0, s, workspace, m, count);
    hipLaunchKernelGGL(dd::compact_scatter_kernel, dim3((unsigned)m), dim3(dd::kBlock), 0, s, flags, want,
                       (const int32_t*)workspace, idx_out, n);
    return dd::finish();
}

int64_t dd_step_bytes_per_env(int32_t precision, int32_t action_format, int32_t with_obs) {
    const int64_t f = precision == DD_F64 ? 8 : 4;
    const int64_t act = action_format == DD_ACT_F32X3 ? 12 : action_format == DD_ACT_U8X3 ? 3 : 1;
    // reads: x y vx vy angle omega fuel px py total (10 f) + status 1 + steps 4 + action
    const int64_t rd = 10 * f + 1 + 4 + act;
    // writes: x y vx vy angle omega fuel total reward (9 f) + steps 4 + done 1
    // (status is rewritten only on the frame an episode ends)
    const int64_t wr = 9 * f + 4 + 1;
    return rd + wr + (with_obs ? DD_OBS_DIM * 4 : 0);
}

const char* dd_error_string(int code) { return hipGetErrorString((hipError_t)code); }

int dd_abi_version(void) { return DD_ABI_VERSION; }

}  // extern "C"
#endif  // DD_ISA_PROBE
