/*
 * dronestep.h — C-ABI of the MI355X-native vectorised delivery-drone step.
 *
 * This is the drop-in boundary for the reference's per-frame hot path
 * (vedant-jumle/reinforcement-learning-101, delivery_drone/game/):
 *
 *   DroneGame.step     game_engine.py:95-138   -> dd_step
 *   DroneGame.reset    game_engine.py:59-93    -> dd_reset
 *   DroneGame.get_state game_engine.py:140-177 -> dd_write_obs
 *   DroneGame._get_info game_engine.py:281-298 -> dd_get_info
 *   DroneGame.render    game_engine.py:300-337 -> dd_render ('rgb_array' frames)
 *   config.py:17-68 module constants           -> DDConfig (dd_config_default)
 *
 * and for the notebooks' side of the loop:
 *
 *   calc_reward + max_steps  Actor_Critic_PPO.ipynb:164-263, :886-888 -> dd_step (shaped_*)
 *   calc_reward + max_steps  Policy_Gradients.ipynb:162-238, :590-593 (REINFORCE)
 *                                                       -> dd_step (shaped_mode)
 *   the collection loop       Actor_Critic_PPO.ipynb:797-917          -> dd_rollout
 *   DroneGamerBoi / DroneTeacherBoi + Bernoulli.sample / log_prob
 *                             Actor_Critic_PPO.ipynb:376-424, :851-859 -> dd_mlp_forward
 *   compute_gae               Actor_Critic_PPO.ipynb:733-787          -> dd_gae
 *   collect_episodes_ppo with the actor in the loop
 *                             Actor_Critic_PPO.ipynb:797-917          -> dd_policy_rollout
 *
 * One call processes a batch of N independent drones stored as a
 * struct-of-arrays (SoA) in device memory.  The reference has no FFI of its
 * own (it is 100 % Python and its only cross-process surface is the JSON
 * socket protocol of game/socket_server.py:126-263); these entry points are
 * what a ctypes / cffi binding of that path binds.
 *
 * Conventions
 *  - The caller owns every buffer.  Nothing here allocates, frees or keeps a
 *    pointer past the call.  All work is enqueued on `stream` (a hipStream_t
 *    passed as void*; NULL = the legacy default stream) and is asynchronous.
 *  - Return value: 0 on success, otherwise a hipError_t code
 *    (1 = hipErrorInvalidValue for argument errors).  No exceptions cross the
 *    ABI.  dd_error_string() turns a code into text.
 *  - Floating-point fields are either all float (DD_F32) or all double
 *    (DD_F64); the arithmetic is always IEEE double, matching the reference's
 *    Python floats, and results are rounded once on store.
 */
#ifndef DRONESTEP_H
#define DRONESTEP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DD_ABI_VERSION 12 /* 12: spawns drawn from Philox4x32-7; 11: shaped_mode (REINFORCE reward), DDRolloutIO.kernel, dd_rollout_kernel,
                              dd_device_errors; 10: DDStepIO.state_out (ping-pong state) */

/* Storage precision of the SoA floating-point fields. */
enum { DD_F32 = 0, DD_F64 = 1 };

/* Action encodings accepted by dd_step (DDStepIO.action_format).
 * The reference takes a dict {main_thrust, left_thrust, right_thrust} and
 * casts each with bool() (game_engine.py:114-118). */
enum {
    DD_ACT_BITMASK = 0, /* uint8[N], bit0 = main, bit1 = left, bit2 = right  */
    DD_ACT_F32X3 = 1,   /* float[N][3] (main, left, right), nonzero = on;     */
                        /* the notebooks' Bernoulli(probs).sample() layout     */
    DD_ACT_U8X3 = 2,    /* uint8/bool[N][3] (main, left, right), nonzero = on */
    DD_ACT_PHILOX = 3   /* dd_rollout only: no action buffer; step s's
                           bitmask is nibble s & 31 of Philox4x32-10(key =
                           action_seed, ctr = {env, s >> 5}) & 7 — a uniform
                           random policy, one block per 32 steps            */
};

/* Status byte bits (DDState.status). */
enum {
    DD_ST_DONE = 1u << 0,    /* DroneGame.done                    */
    DD_ST_LANDED = 1u << 1,  /* Drone.landed                      */
    DD_ST_CRASHED = 1u << 2, /* Drone.crashed                     */
    DD_ST_PLAT_LEFT = 1u << 3 /* Platform.direction == -1 (moving) */
};

/* The notebooks' shaped reward (DDStepIO / DDRolloutIO / DDPolicyRolloutIO
 * shaped_mode), each with its collection loop's max_steps timeout (done, -500
 * unless landed):
 *   DD_SHAPED_PPO        calc_reward(state, prev_state) of Actor_Critic_PPO.ipynb:
 *                        164-263 (also Actor_Critic_Basic), prev_state two frames
 *                        back as collect_episodes_ppo passes it; needs shaped_hist.
 *   DD_SHAPED_REINFORCE  calc_reward(state) of Policy_Gradients.ipynb:162-238
 *                        (distance-scaled time penalty, terminal 500 + fuel * 100
 *                        or -200 / -300), timeout :590-593; no history. */
enum { DD_SHAPED_PPO = 0, DD_SHAPED_REINFORCE = 1 };

/* Width of one observation row: state_to_array order of
 * Actor_Critic_PPO.ipynb:346-366 (x, y, vx, vy, angle, omega, fuel, px, py,
 * distance, dx, dy, speed, landed, crashed), each normalised exactly as
 * DroneGame.get_state (game_engine.py:151-175). */
#define DD_OBS_DIM 15

/* World constants.  dd_config_default() fills the values of config.py. */
typedef struct DDConfig {
    /* physics — config.py:18-29, drone.py:44-103 */
    double gravity;           /* GRAVITY 0.3                  */
    double drag;              /* DRAG 0.99                    */
    double angular_drag;      /* ANGULAR_DRAG 0.95            */
    double main_thrust_power; /* MAIN_THRUST_POWER 0.6        */
    double side_thrust_power; /* SIDE_THRUST_POWER 0.3        */
    double fuel_main;         /* FUEL_CONSUMPTION_MAIN 2.0    */
    double fuel_side;         /* FUEL_CONSUMPTION_SIDE 1.0    */
    double max_fuel;          /* MAX_FUEL 1000.0              */
    double drone_half_height; /* DRONE_HEIGHT / 2 = 10.0 (get_bottom_center) */
    double dt;                /* update(dt=1.0)               */
    /* platform — config.py:32-36, platform.py:11-62 */
    double platform_half_width;  /* PLATFORM_WIDTH / 2 = 50.0  */
    double platform_half_height; /* PLATFORM_HEIGHT / 2 = 10.0 */
    double platform_speed;       /* PLATFORM_SPEED 1.0         */
    double platform_min_x;       /* width // 2 = 50            */
    double platform_max_x;       /* WINDOW_WIDTH - width // 2 = 750 */
    /* landing — config.py:39-40 */
    double max_landing_velocity; /* 3.0  */
    double max_landing_angle;    /* 20.0 */
    /* bounds — config.py:3-4, 45; game_engine.py:254 */
    double world_width;  /* 800 */
    double world_height; /* 600 */
    double oob_margin;   /* 50  */
    double ground_level; /* WINDOW_HEIGHT - 50 = 550 */
    /* wind — config.py:48-49, game_engine.py:121-123 */
    double wind_x, wind_y;
    /* rewards — config.py:54-58, game_engine.py:185-214 */
    double reward_step;          /* -0.1   */
    double reward_landing;       /* 100.0  */
    double reward_crash;         /* -100.0 */
    double reward_out_of_fuel;   /* -50.0  */
    double reward_out_of_bounds; /* -50.0  */
    double shaping_offset;       /* 500  in (500 - dist) / 5000 */
    double shaping_scale;        /* 5000 */
    /* observation scales — game_engine.py:155-171 */
    double vel_scale;   /* 10.0  */
    double angle_scale; /* 180.0 */
    /* spawn — config.py:61-68, game_engine.py:66-85 (integer ranges) */
    int32_t drone_start_x, drone_start_y;         /* fixed spawn 400, 100 */
    int32_t drone_x_min, drone_x_max;             /* inclusive 100..700   */
    int32_t drone_y_min, drone_y_max;             /* inclusive 50..250    */
    int32_t platform_start_x, platform_start_y;   /* fixed 400, 500       */
    int32_t platform_x_lo, platform_x_hi;         /* half-open [100, 700) */
    int32_t platform_y_lo, platform_y_hi;         /* half-open [100, 550) */
    /* switches */
    int32_t wind_enabled;       /* WIND_ENABLED False      */
    int32_t platform_moving;    /* PLATFORM_MOVING False   */
    int32_t randomize_drone;    /* DroneGame(randomize_drone=False)   */
    int32_t randomize_platform; /* DroneGame(randomize_platform=True) */
    int32_t auto_reset;         /* 0: sticky done (game_engine.py:107-111);
                                   1: a lane that is done when dd_step starts is
                                   re-spawned and returns its reset observation
                                   with reward 0 and done 0 (next-step reset). */
    int32_t _pad;
    uint64_t seed; /* key of the spawn draws: Philox4x32-7 of (env id, episode) (ABI 12; 10 rounds before) */
} DDConfig;

/* The SoA.  Every pointer addresses N elements in device memory.  The ten
 * floating-point arrays are float* (DD_F32) or double* (DD_F64). */
typedef struct DDState {
    void *x, *y, *vx, *vy, *angle, *omega, *fuel; /* Drone: drone.py:19-33      */
    void *px, *py;                                /* Platform.x / .y            */
    void *total_reward;                           /* DroneGame.total_reward     */
    uint8_t *status;                              /* DD_ST_* bits               */
    int32_t *steps;                               /* DroneGame.steps            */
    int32_t *episode;                             /* DroneGame.episode          */
    int64_t env_id_base; /* global id of element 0 (sharding-invariant RNG)    */
    int32_t precision;   /* DD_F32 or DD_F64                                   */
    int32_t _pad;
} DDState;

/* Per-call inputs and outputs of dd_step. */
typedef struct DDStepIO {
    const void *actions;  /* see action_format (required)                      */
    int32_t action_format;
    int32_t _pad;
    void *reward;         /* float or double [N] by precision (required)        */
    uint8_t *done;        /* uint8 [N], 1 = done after this call (required)     */
    float *obs;           /* float [N][15] (nullable)                           */
    int32_t *done_idx;    /* lanes whose episode ended in this call, in any
                             order (nullable; wave-ballot compaction)            */
    int32_t *done_count;  /* number of entries written to done_idx (zeroed by
                             dd_step; required iff done_idx != NULL)             */
    /* The notebooks' shaped reward, fused (all three pointers set, or none):
     * calc_reward(state, prev_state) of Actor_Critic_PPO.ipynb:164-263 on the
     * frame's double-precision observation, with prev_state the state two
     * frames back as collect_episodes_ppo passes it (:797-917), plus its
     * max_steps truncation (:886-888: steps >= max_steps ends the episode,
     * -500 unless landed; the lane's done bit is set so it stops / re-spawns). */
    double *shaped_hist;  /* [2][N] per-lane distance history, slot = steps & 1;
                             NaN = no previous state (dd_shaped_reset fills it) */
    void *shaped_reward;  /* float or double [N] by precision                   */
    uint8_t *shaped_done; /* uint8 [N]: done or truncated                        */
    int32_t max_steps;    /* <= 0: no truncation                                 */
    int32_t shaped_mode;  /* DD_SHAPED_PPO (the three pointers above, or none) or
                             DD_SHAPED_REINFORCE (shaped_reward and shaped_done
                             required, shaped_hist not read)                     */
    /* Ping-pong state (nullable = in place): the step reads the nine fields
     * that change every frame (x y vx vy angle omega fuel total_reward steps)
     * from `st` and writes them to *state_out's arrays, which must not alias
     * st's; px, py, status and episode change only on a terminal frame or a
     * re-spawn and stay in place (state_out's pointers for them must equal
     * st's, and so must precision and env_id_base).  Separate in / out arrays
     * spare the kernel the in-place update's end-of-launch write-back of lines
     * it also read.  A sticky-done lane copies its fields. */
    const struct DDState *state_out;
} DDStepIO;

/* Inputs and outputs of dd_rollout: `frames` consecutive frames, frame-major.
 * Buffers are [frames][N] (actions in action_format, reward, done) and
 * [frames][N][15] (obs).  The rollout equals `frames` dd_step calls with
 * actions[k], bit for bit; the state stays in registers between frames. */
typedef struct DDRolloutIO {
    const void *actions;  /* [frames][N] per action_format; NULL for DD_ACT_PHILOX */
    int32_t action_format;
    int32_t frames;
    void *reward;         /* float or double [frames][N] (required)             */
    uint8_t *done;        /* uint8 [frames][N] (required)                       */
    float *obs;           /* float [frames][N][15] (nullable)                   */
    uint64_t action_seed; /* DD_ACT_PHILOX key                                  */
    int64_t action_step;  /* DD_ACT_PHILOX counter of frame 0 (frame k: +k)     */
    /* Notebook reward mode (as DDStepIO's shaped_*): with shaped_mode
     * DD_SHAPED_PPO and shaped_hist set, or DD_SHAPED_REINFORCE, reward / done
     * receive the notebook's calc_reward and done with the max_steps timeout,
     * and the PPO [2][N] history is read at launch and written back at its end.
     * DD_SHAPED_PPO with shaped_hist NULL = the engine reward.              */
    double *shaped_hist;  /* double [2][N] (nullable)                           */
    void *engine_reward;  /* shaped mode: the engine's reward [frames][N] (nullable) */
    uint8_t *engine_done; /* and done; both or neither                          */
    int32_t max_steps;    /* shaped mode: episode cap, <= 0 = none              */
    int32_t shaped_mode;  /* DD_SHAPED_*                                        */
    int32_t kernel;       /* DD_ROLLOUT_AUTO / _SINGLE / _SPLIT_NO_WAIT          */
    int32_t _pad;
} DDRolloutIO;

/* DDRolloutIO.kernel.  AUTO: the split kernel (frame waves + writer waves,
 * DESIGN.md §4) where it applies (reference world, engine reward, obs rows,
 * one block per CU or fewer), the single-role kernel elsewhere.  SINGLE: never
 * the split kernel.  SPLIT_NO_WAIT (diagnostic): as AUTO with the split
 * kernel's hand-over waits capped at zero polls, which reports DD_ERR_HANDOVER
 * through dd_device_errors — the check that a broken hand-over is not silent. */
enum { DD_ROLLOUT_AUTO = 0, DD_ROLLOUT_SINGLE = 1, DD_ROLLOUT_SPLIT_NO_WAIT = 2 };
/* dd_rollout_kernel(): the kernel a dd_rollout call launches (its first chunk). */
enum { DD_ROLLOUT_FLUSHED = 16, DD_ROLLOUT_HELD = 17, DD_ROLLOUT_SPLIT = 18 };

/* Fills *cfg with config.py's values (randomize_platform = 1, others 0). */
void dd_config_default(DDConfig *cfg);

/* One frame for every lane: DroneGame.step (game_engine.py:95-138). */
int dd_step(const DDConfig *cfg, const DDState *st, const DDStepIO *io,
            int64_t n, void *stream);

/* `frames` consecutive frames in one launch (open-loop action sequences,
 * random-policy collection, PPO-shaped rollouts with known actions): the
 * same frame as dd_step, game_engine.py:95-138, applied frames times. */
int dd_rollout(const DDConfig *cfg, const DDState *st, const DDRolloutIO *io,
               int64_t n, void *stream);

/* Which kernel dd_rollout takes for these arguments (DD_ROLLOUT_FLUSHED /
 * _HELD / _SPLIT), -1 for invalid ones.  No GPU work. */
int dd_rollout_kernel(const DDConfig *cfg, const DDState *st, const DDRolloutIO *io,
                      int64_t n);

/* Sticky error bits the kernels set on the device (DD_ERR_*), read after a
 * hipDeviceSynchronize (work on every stream, non-blocking ones included, has
 * finished) and cleared if `clear`. */
enum { DD_ERR_HANDOVER = 1 }; /* a split-rollout hand-over wait ran out: rows of
                                 that launch are not to be trusted */
int dd_device_errors(uint32_t *bits, int32_t clear);

/* Re-spawn lanes (DroneGame.reset, game_engine.py:59-93).  mask: uint8 [N],
 * nonzero = reset that lane; NULL = all lanes.  obs (nullable) receives the
 * reset observation of the reset lanes; other rows are left untouched. */
int dd_reset(const DDConfig *cfg, const DDState *st, const uint8_t *mask,
             float *obs, int64_t n, void *stream);

/* (Re)start the shaped-reward history of the masked lanes (NULL = all) from
 * their current state: slot 0 = this state's distance, slot 1 = none.  Call
 * after dd_reset; auto-reset inside dd_step restarts it by itself. */
int dd_shaped_reset(const DDConfig *cfg, const DDState *st, const uint8_t *mask,
                    double *shaped_hist, int64_t n, void *stream);

/* Observation rows from the current state (DroneGame.get_state). */
int dd_write_obs(const DDConfig *cfg, const DDState *st, float *obs,
                 int64_t n, void *stream);

/* Pixel-unit distance to the platform and speed (DroneGame._get_info,
 * game_engine.py:292-296); float or double [N] by precision. */
int dd_get_info(const DDConfig *cfg, const DDState *st, void *distance,
                void *speed, int64_t n, void *stream);

/* Ordered compaction: idx_out receives, in ascending order, every i with
 * (flags[i] != 0) == (want != 0); *count its length.  Builds the notebooks'
 * active-game list (Actor_Critic_PPO.ipynb:840-850) on device.
 * workspace: int32 [dd_compact_workspace(n)] scratch. */
int64_t dd_compact_workspace(int64_t n);
int dd_compact(const uint8_t *flags, int32_t want, int32_t *idx_out,
               int32_t *count, int32_t *workspace, int64_t n, void *stream);

/* Generalised advantage estimation over a [T][N] rollout (compute_gae of
 * Actor_Critic_PPO.ipynb:733-787, per lane; a done at t cuts the recursion):
 *   delta = r[t] + gamma * v[t+1] * (1 - d[t]) - v[t]
 *   gae   = delta + gamma * lambda * (1 - d[t]) * gae
 * in float32 with the notebook's operation order (torch float32 tensors,
 * Python-float gamma / lambda).  values is [T+1][N] (row T = bootstrap).
 * returns (nullable) = advantages + values[t], as the notebook forms them. */
int dd_gae(const float *rewards, const float *values, const uint8_t *dones,
           float *advantages, float *returns, int64_t T, int64_t n,
           double gamma, double lambda, void *stream);

/* ---- Policy and value networks ------------------
 * The notebooks' DroneGamerBoi (actor) and DroneTeacherBoi (critic),
 * Actor_Critic_PPO.ipynb:376-424:
 *   Linear(15,128) LayerNorm(128) ReLU  Linear(128,128) LayerNorm(128) ReLU
 *   Linear(128,64) LayerNorm(64) ReLU   Linear(64,K)  [+ Sigmoid, actor]
 * with K = 3 (main, left, right) for the actor and K = 1 for the critic, in
 * float32.  The parameters are the state_dict tensors (torch layout: weight
 * [out][in] row-major, device pointers), repacked once by dd_mlp_pack into
 * the kernel's MFMA operand order. */
typedef struct DDMlpParams {
    const float *w0, *b0, *ln1_w, *ln1_b; /* network.0 (Linear), network.1 (LayerNorm) */
    const float *w3, *b3, *ln4_w, *ln4_b; /* network.3, network.4 */
    const float *w6, *b6, *ln7_w, *ln7_b; /* network.6, network.7 */
    const float *w9, *b9;                 /* network.9: [K][64], [K] */
    int32_t out_dim;                      /* K: 3 (actor) or 1 (critic) */
    float ln_eps;                         /* nn.LayerNorm eps (1e-5) */
} DDMlpParams;

/* One forward pass over N observation rows.  The actor (K = 3) writes the
 * Sigmoid probabilities, and optionally samples actions as
 * Bernoulli(probs).sample() (Actor_Critic_PPO.ipynb:857-858: bit j set iff
 * u_j < p_j, u_j uniform in [0,1) from Philox4x32-10 keyed by
 * (seed; env_id_base + i, step, 0x5A5A5A5A)) packed as the dd_step bitmask,
 * with Bernoulli.log_prob(actions).sum(-1) (:859).  The critic (K = 1)
 * writes the value. */
typedef struct DDMlpIO {
    const float *obs;    /* [N][15] f32, dd_step / dd_write_obs rows */
    float *out;          /* nullable: [N][3] probabilities (actor) or [N] values (critic) */
    uint8_t *actions;    /* actor, nullable: uint8 [N] sampled bitmask */
    float *log_prob;     /* actor, nullable: [N] summed log-probability of `actions` */
    uint64_t seed;
    int64_t step;
    int64_t env_id_base;
} DDMlpIO;

/* Arithmetic of the three hidden GEMMs.  DD_MLP_F32: the f32 MFMA, the
 * notebook's float32 model as is.  DD_MLP_F16X3 (opt-in, ~2.7x faster:
 * 65,536 rows 33 -> 12-13 us on MI355X): each operand split into two f16
 * halves, a = hi + lo, three f16 MFMAs per product with f32 accumulation
 * (~21-22 bits per product, about the f32 path's end-to-end error).  Its
 * operands must fit the f16 halves at the packing's powers of two: hidden
 * weights |w| < 2047, observations |obs| < 1023, each LayerNorm's output
 * below 128 (max|weight| sqrt(rows) + max|bias| < 128); beyond, results are
 * wrong or NaN (MlpNet checks the parameters before packing).  LayerNorm,
 * the last layer and sampling are f32 either way. */
enum { DD_MLP_F32 = 0, DD_MLP_F16X3 = 1 };

/* Floats of a packed parameter buffer (same for K = 1 and 3, either compute).
 * The buffer ends in a layout tag: the compute and K it was packed for.  A
 * consumer launched with another compute or K (or, for dd_policy_rollout, a
 * critic's buffer) does not misread it: its probabilities, log-probabilities
 * and values come out NaN. */
int64_t dd_mlp_packed_floats(void);
/* Repack state_dict tensors into `packed` (device, dd_mlp_packed_floats()
 * floats, 16-byte aligned: every consumer reads it in 16-byte fragments;
 * a misaligned pointer is hipErrorInvalidValue) for `compute` (DD_MLP_*). */
int dd_mlp_pack(const DDMlpParams *params, int32_t compute, float *packed, void *stream);
/* Forward pass; out_dim and compute must match the packed parameters. */
int dd_mlp_forward(const float *packed, int32_t compute, int32_t out_dim,
                   const DDMlpIO *io, int64_t n, void *stream);

/* ---- The collection loop with the actor in it --
 * collect_episodes_ppo (Actor_Critic_PPO.ipynb:797-917) for N drones and
 * `frames` frames in one launch: per frame, the actor on the current
 * observation (dd_mlp_forward's network and sampling, :851-859), then the
 * drone frame (dd_step) with the sampled action.  Frame k writes
 *   obs[k]      the policy input (the observation before the frame; frame 0's
 *               is obs0, later ones are the previous frame's dd_step obs)
 *   actions[k], log_prob[k]   as dd_mlp_forward with step = step + k
 *   reward[k], done[k]        as dd_step (reward_mode as DDRolloutIO)
 * and obs_final receives the observation after the last frame.  Equal, bit
 * for bit, to `frames` x (dd_mlp_forward(obs) ; dd_step(actions)) with the
 * state's env ids as the sampling ids.  The actor's packed parameters
 * (dd_mlp_pack, out_dim 3) are read into LDS once per launch. */
typedef struct DDPolicyRolloutIO {
    const float *obs0;    /* [N][15] observation before frame 0 (required)      */
    float *obs_final;     /* [N][15] observation after the last frame (nullable;
                             may be obs0)                                        */
    float *obs;           /* [frames][N][15] policy inputs (nullable)           */
    uint8_t *actions;     /* [frames][N] sampled bitmask (nullable)             */
    float *log_prob;      /* [frames][N] summed log-probability (nullable)      */
    void *reward;         /* float or double [frames][N] by precision (required) */
    uint8_t *done;        /* uint8 [frames][N] (required)                       */
    uint64_t seed;        /* Bernoulli draws: Philox4x32-10 key                 */
    int64_t step;         /* sampling step of frame 0 (frame k: step + k)       */
    int32_t frames;
    int32_t max_steps;    /* notebook mode: episode cap, <= 0 = none            */
    double *shaped_hist;  /* notebook reward mode, as DDRolloutIO (nullable)    */
    void *engine_reward;  /* notebook mode: the engine's reward / done          */
    uint8_t *engine_done; /* [frames][N] (both or neither, nullable)            */
    int32_t shaped_mode;  /* DD_SHAPED_* as DDRolloutIO                         */
    int32_t _pad;
} DDPolicyRolloutIO;

int dd_policy_rollout(const DDConfig *cfg, const DDState *st, const float *packed,
                      int32_t compute, const DDPolicyRolloutIO *io, int64_t n,
                      void *stream);

/* ---- Rendering -------------------------------------
 * DroneGame.render() in 'rgb_array' mode (game_engine.py:300-337): the scene
 * of platform.py:76-102, drone.py:155-218, _render_hud (game_engine.py:339-384)
 * and, for a lane that is done, _render_game_over (:386-412), as
 * surfarray.array3d(screen).transpose(1, 0, 2) gives it: uint8 [H][W][3] with
 * W x H = world_width x world_height (800 x 600; width a multiple of 4).
 * pygame's primitives are restated (render.hip's header), not pixel-verified:
 * pygame is absent here, and the text uses DejaVu Sans Bold for pygame's
 * bundled font. */
enum { DD_RENDER_HUD = 1, DD_RENDER_GAME_OVER = 2 };

/* Renders `count` frames into rgb: uint8 [count][H][W][3].  The SoA holds n
 * lanes.  lanes: int32 [count] device indices into it, or NULL for lanes
 * 0..count-1 (count <= n); a frame whose index is outside [0, n) is left
 * all zero.  actions (nullable): the uint8 [n] bitmask of the last step, which
 * _render_thrust draws as flames (drone.py:189-218, where fuel > 0); NULL
 * draws none, and so does a lane whose steps is 0 (Drone.reset clears the
 * thrusters).  flags: DD_RENDER_*. */
int dd_render(const DDConfig *cfg, const DDState *st, const uint8_t *actions,
              const int32_t *lanes, int64_t count, int64_t n, uint8_t *rgb,
              int32_t flags, void *stream);

/* Algorithmic HBM bytes of one dd_step lane (the roofline byte model,
 * DESIGN.md §4): precision, action format, obs on/off. */
int64_t dd_step_bytes_per_env(int32_t precision, int32_t action_format,
                              int32_t with_obs);

const char *dd_error_string(int code);
int dd_abi_version(void);
/* "abi=<n>;step_isa=<sha256/16>;policy_rollout_isa=<sha256/16>": the ABI version
 * and hashes of the device ISA this library was built with (tools/build_info.py);
 * bench.py reports PMC traffic only for the build it was measured on. */
const char *dd_build_info(void);

/* Self-check of the frame's square root (not a reference interface): the
 * kernels take sqrt through an unscaled form of the compiler's sequence
 * (trig.h sqrt_unscaled) for operands >= 2^-767.  Evaluates both on n
 * doubles (the integers 0..2^20, then Philox-drawn values with exponents
 * spread over the whole range) and adds the number whose results differ in
 * any bit to *mismatches (device memory). */
int dd_selftest_sqrt(uint64_t seed, int64_t n, unsigned long long *mismatches, void *stream);

/* Measurement helpers for bench.py (not reference interfaces).  dd_stamp
 * launches a one-lane kernel on `stream` that writes the GPU's constant-rate
 * wall clock to *slot (device memory) when it runs; captured into a hipGraph
 * between step launches it stamps that point of the graph.  dd_wall_clock_khz
 * gives the clock's rate (hipDeviceAttributeWallClockRate, current device). */
int dd_stamp(unsigned long long *slot, void *stream);
int dd_wall_clock_khz(int *khz);

/* Device memory for an env's arrays (not a reference interface;
 * VecDroneEnv(memory=...) carves its SoA fields and per-step outputs from
 * one range).  DD_MEM_DEFAULT: hipMalloc.  DD_MEM_CONTIGUOUS:
 * hipExtMallocWithFlags(hipDeviceMallocContiguous), one physically
 * contiguous range: an HBM-resident batch (16.8M drones) steps at the same
 * speed from every such allocation (within ~1 %) where hipMalloc'd ones vary
 * ~10 % with the driver's placement, but a cache-resident
 * batch (262,144 drones) steps ~35 % slower from it (profiles/r06/lab/).
 * dd_device_free(NULL) is a no-op. */
#define DD_MEM_DEFAULT 0
#define DD_MEM_CONTIGUOUS 1
int dd_device_alloc(void **ptr, uint64_t bytes, int32_t flags);
int dd_device_free(void *ptr);

#ifdef __cplusplus
}
#endif

#endif /* DRONESTEP_H */
