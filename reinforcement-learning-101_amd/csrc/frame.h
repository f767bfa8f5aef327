// frame.h — one drone's frame of DroneGame.step in IEEE double: world
// constants, the lane state, Drone.apply_thrust / update, the reward cascade,
// get_state's observation row and the notebooks' calc_reward.  Shared by the
// step / rollout kernels (drone_step.hip) and the fused policy rollout
// (policy_rollout.hip), so every path evaluates the same frame bit for bit.
// Compiled with -ffp-contract=off (see drone_step.hip).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <type_traits>

#include "dronestep.h"
#include "philox.h"
#include "trig.h"

// The reference's sin, cos and squares, bit for bit: libm_ref.h restates
// glibc's (the reference calls np.sin / np.cos and `v ** 2` = glibc pow), with
// their tables (csrc/libm_tables.h: glibc 2.35's, committed) in device
// memory, for the rare frames near a predicate boundary (frame).
#include "libm_tables.h"
__device__ const double dd_libm_pow_tab[384] = DD_LIBM_POW_TAB;
__device__ const uint64_t dd_libm_exp_tab[256] = DD_LIBM_EXP_TAB;
__device__ const double dd_libm_sincos_tab[440] = DD_LIBM_SINCOS_TAB;
#define DD_LIBM_FN __device__ __forceinline__
#define DD_LIBM_OPAQUE
#define DD_LIBM_ENTRY __device__ __forceinline__
#include "libm_ref.h"
#undef DD_LIBM_FN
#undef DD_LIBM_ENTRY
#undef DD_LIBM_SINCOS_FN
#undef DD_LIBM_OPAQUE

namespace dd {

// numpy's deg2rad: x * (NPY_PI / 180.0)   (physics.py:16, np.radians)
constexpr double kDeg2Rad = 3.14159265358979323846 / 180.0;

// sin and cos of an angle in degrees, as rotate_point computes them
// (physics.py:16-18: np.radians, then np.cos and np.sin).  Fast: trig.h's
// (within an ulp of glibc's; glibc's everywhere measured +9 % step, +26 %
// rollout; OCML's sincos equal within noise); kExact: glibc's, bit for bit
// (libm_ref.h), for the rare frames where an ulp could flip a flag (frame).
// kSgpr: the polynomial coefficients as SGPR operands (trig::hstep_c), for
// the step kernel, whose four waves per SIMD overlap one wave's scalar moves
// with another's VALU; the loops (one wave per SIMD) keep the vector form.
template <bool kExact = false, bool kSgpr = false>
__device__ __forceinline__ void sincos_deg(double deg, double* s, double* c) {
    if constexpr (kExact) {
        libm::sincos(deg * kDeg2Rad, s, c);
        return;
    }
    trig::sincos<kSgpr>(deg * kDeg2Rad, s, c);
}

// ---------------------------------------------------------------------------
// World constants
// ---------------------------------------------------------------------------
// config.py:17-68 as a DDConfig (also what dd_config_default returns).
constexpr DDConfig reference_config() {
    DDConfig c{};
    c.gravity = 0.3;
    c.drag = 0.99;
    c.angular_drag = 0.95;
    c.main_thrust_power = 0.6;
    c.side_thrust_power = 0.3;
    c.fuel_main = 2.0;
    c.fuel_side = 1.0;
    c.max_fuel = 1000.0;
    c.drone_half_height = 20 / 2.0;
    c.dt = 1.0;
    c.platform_half_width = 100 / 2.0;
    c.platform_half_height = 20 / 2.0;
    c.platform_speed = 1.0;
    c.platform_min_x = 100 / 2;
    c.platform_max_x = 800 - 100 / 2;
    c.max_landing_velocity = 3.0;
    c.max_landing_angle = 20.0;
    c.world_width = 800;
    c.world_height = 600;
    c.oob_margin = 50;
    c.ground_level = 600 - 50;
    c.wind_x = 0.0;
    c.wind_y = 0.0;
    c.reward_step = -0.1;
    c.reward_landing = 100.0;
    c.reward_crash = -100.0;
    c.reward_out_of_fuel = -50.0;
    c.reward_out_of_bounds = -50.0;
    c.shaping_offset = 500;
    c.shaping_scale = 5000;
    c.vel_scale = 10.0;
    c.angle_scale = 180.0;
    c.drone_start_x = 800 / 2;
    c.drone_start_y = 100;
    c.drone_x_min = 100;
    c.drone_x_max = 700;
    c.drone_y_min = 50;
    c.drone_y_max = 250;
    c.platform_start_x = 800 / 2;
    c.platform_start_y = 600 - 100;
    c.platform_x_lo = 100 / 2 + 50;
    c.platform_x_hi = 800 - 100 / 2 - 50;
    c.platform_y_lo = 100;
    c.platform_y_hi = 550;
    c.wind_enabled = 0;
    c.platform_moving = 0;
    c.randomize_drone = 0;
    c.randomize_platform = 1;
    c.auto_reset = 0;
    c.seed = 0;
    return c;
}

// The constants the frame reads: the config plus the correctly rounded
// reciprocals of its divisors (for trig::div_exact).
struct Consts {
    DDConfig c;
    double inv_w, inv_h, inv_vel, inv_angle, inv_fuel, inv_shaping;
};

constexpr Consts make_consts(const DDConfig& c) {
    Consts k{};
    k.c = c;
    k.inv_w = 1.0 / c.world_width;
    k.inv_h = 1.0 / c.world_height;
    k.inv_vel = 1.0 / c.vel_scale;
    k.inv_angle = 1.0 / c.angle_scale;
    k.inv_fuel = 1.0 / c.max_fuel;
    k.inv_shaping = 1.0 / c.shaping_scale;
    return k;
}

// The reference's physics, reward and observation constants as compile-time
// data: kernels instantiated with kRef = true read them from here and the
// compiler folds them into the instruction stream (no kernarg SGPRs, no SGPR
// spills).  Switches, spawn ranges, wind and seed always come from the call.
__device__ constexpr Consts kRefConsts = make_consts(reference_config());

// True when every double the frame reads (wind aside) equals config.py's
// and the run has neither wind nor a moving platform: the kernels' kRef
// instantiation, whose frame compiles neither in.
inline bool uses_reference_physics(const DDConfig& c) {
    if (c.wind_enabled || c.platform_moving) return false;
    const DDConfig r = reference_config();
    const double* a = &c.gravity;
    const double* b = &r.gravity;
    const int n = (int)((&c.vel_scale - &c.gravity) + 1);
    for (int j = 0; j < n; ++j) {
        if (a + j == &c.wind_x || a + j == &c.wind_y) continue;
        if (memcmp(a + j, b + j, sizeof(double)) != 0) return false;
    }
    return true;
}

// Uniform integer in [lo, lo + span) from one 32-bit draw (multiply-high).
__device__ __forceinline__ int32_t draw_range(uint32_t r, int32_t lo, uint32_t span) {
    return lo + (int32_t)(((uint64_t)r * span) >> 32);
}

// ---------------------------------------------------------------------------
// One drone
// ---------------------------------------------------------------------------
// The per-lane state, widened to double for the frame's arithmetic.
struct Lane {
    double x, y, vx, vy, angle, omega, fuel, px, py, total;
    double speed, dist;  // derived: Drone.get_speed, physics.distance to the pad
    uint32_t status;
    int32_t steps, episode;
};

// Drone.get_speed (drone.py:139-145) and physics.distance (physics.py:42-44)
// of the current state; both the reward and get_state use them.  Returns the
// speed's sum of squares.  The reference squares with `v ** 2`, glibc pow,
// which differs from v*v by an ulp on ~0.09 % of inputs: speed and distance
// may differ from the reference's by an ulp (the observation and the shaping
// reward's tolerance); the one flag they decide, slow, is made exact in
// frame().
// kUnscaled (the step kernel): the two square roots go through
// trig::sqrt_unscaled unless a lane of the wave has an operand below 2^-767
// (zero included: a wave-uniform rare branch to sqrt()); bit-identical to
// sqrt() either way (dd_selftest_sqrt).  Config 3: 8.13 -> 8.02 us per step
// (lab medians, with the SGPR coefficients and the kRef thrust).  The loops
// keep sqrt(): their frame is one basic block, and the branch splitting it
// cost more than the four VALU it saves per root (65,536 x 256 rollout
// 0.362 -> 0.371 ms, profiles/r03/lab/valu_trims_ab.jsonl).
template <bool kUnscaled = false>
__device__ __forceinline__ double measure(Lane& s) {
    const double dx = s.px - s.x, dy = s.py - s.y;
    const double ss = s.vx * s.vx + s.vy * s.vy;
    const double dd = dx * dx + dy * dy;
    if (!kUnscaled) {
        s.speed = sqrt(ss);
        s.dist = sqrt(dd);
        return ss;
    }
    if (__builtin_expect(__ballot(!(ss >= 0x1p-767) | !(dd >= 0x1p-767)) != 0, 0)) {
        s.speed = sqrt(ss);
        s.dist = sqrt(dd);
    } else {
        s.speed = trig::sqrt_unscaled(ss);
        s.dist = trig::sqrt_unscaled(dd);
    }
    return ss;
}

// DroneGame.reset (game_engine.py:59-93) + Drone.reset (drone.py:221-238) +
// Platform.reset (platform.py:104-114).  `c` is the call's config (switches,
// spawn ranges, seed), `max_fuel` the physics' (compile-time under kRef, so
// a rollout's frame loop issues no scalar load that a join's lgkmcnt wait
// would couple to its LDS reads); s.episode becomes the value after
// `episode += 1`.
// The Philox block of (seed; env, episode) that a re-spawn draws from:
// Philox4x32-7 (philox.h; 10 rounds until round 5 — the step kernel's re-spawn
// branch runs in ~35 % of its waves at config 3, and the three rounds were
// 1.8 % of the step, lab A/B profiles/r06/lab/).
__device__ __forceinline__ void spawn_words(const DDConfig& c, int64_t env, int32_t episode, uint32_t (&r)[4]) {
    philox4x32_7((uint32_t)env, (uint32_t)((uint64_t)env >> 32), (uint32_t)episode, 0u, (uint32_t)c.seed,
                  (uint32_t)(c.seed >> 32), r);
}

// The re-spawn of a lane whose episode counter is already the new episode's,
// from that episode's Philox block r (spawn_words).
__device__ __forceinline__ void spawn_from(const DDConfig& c, double max_fuel, const uint32_t (&r)[4], Lane& s) {
    if (c.randomize_drone) {
        s.x = draw_range(r[0], c.drone_x_min, (uint32_t)(c.drone_x_max - c.drone_x_min + 1));
        s.y = draw_range(r[1], c.drone_y_min, (uint32_t)(c.drone_y_max - c.drone_y_min + 1));
    } else {
        s.x = c.drone_start_x;
        s.y = c.drone_start_y;
    }
    if (c.randomize_platform) {
        s.px = draw_range(r[2], c.platform_x_lo, (uint32_t)(c.platform_x_hi - c.platform_x_lo));
        s.py = draw_range(r[3], c.platform_y_lo, (uint32_t)(c.platform_y_hi - c.platform_y_lo));
    } else {
        s.px = c.platform_start_x;
        s.py = c.platform_start_y;
    }
    s.vx = 0.0; s.vy = 0.0; s.angle = 0.0; s.omega = 0.0;
    s.fuel = max_fuel;
    s.status = 0u;  // not done / landed / crashed; platform direction +1
    s.steps = 0;
    s.total = 0.0;
    // measure() of this state: the speed is sqrt(+0) = +0; the positions are
    // integers (DDConfig's spawn fields), so the squared distance is 0 or at
    // least 1, inside trig::sqrt_unscaled's exact range
    const double dx = s.px - s.x, dy = s.py - s.y;
    s.speed = 0.0;
    s.dist = trig::sqrt_unscaled(dx * dx + dy * dy);
}

__device__ __forceinline__ void spawn(const DDConfig& c, double max_fuel, int64_t env, Lane& s) {
    s.episode += 1;
    uint32_t r[4];
    spawn_words(c, env, s.episode, r);
    spawn_from(c, max_fuel, r, s);
}

// A rollout loop's re-spawns with the Philox block drawn ahead.  Under
// auto-reset most waves have a lane to re-spawn in most frames (a wave of 64
// drones, episodes of tens to hundreds of frames), and the wave runs the
// re-spawn's Philox block (~60 VALU) for it.  Here each lane keeps the block
// of its NEXT episode (r, drawn for episode `ep`); a re-spawn takes it, and
// every kRefill-th frame (32) the lanes whose block is spent draw the next one
// together: one Philox per wave per kRefill frames instead of one per frame.
// A lane ending two episodes within kRefill frames draws in-frame (the old
// path).  Same blocks, same spawns: the results are bit for bit spawn()'s.
struct SpawnAhead {
    uint32_t r[4];
    int32_t ep;  // the episode r was drawn for
    // frames between refills (a power of two): 4 / 8 / 16 / 32 frames measured
    // 0.303 / 0.295 / 0.293 / 0.288 ms (config 5; 64 no better), DESIGN.md §4
    static constexpr int kRefill = 32;

    __device__ __forceinline__ void init(const DDConfig& c, int64_t env, int32_t episode) {
        ep = episode + 1;
        spawn_words(c, env, ep, r);
    }
    // frame f's end (wave-uniform f): refill the spent blocks
    __device__ __forceinline__ void refill(const DDConfig& c, int64_t env, int32_t episode, int f) {
        if ((f & (kRefill - 1)) == kRefill - 1) {
            const bool spent = ep != episode + 1;
            if (__ballot(spent)) {
                if (spent) init(c, env, episode);
            }
        }
    }
    // the auto-reset re-spawn of a done lane (called by that lane only)
    __device__ __forceinline__ void respawn(const DDConfig& c, double max_fuel, int64_t env, Lane& s) {
        s.episode += 1;
        uint32_t w[4] = {r[0], r[1], r[2], r[3]};
        if (ep != s.episode) spawn_words(c, env, s.episode, w);  // spent: draw now
        spawn_from(c, max_fuel, w, s);
    }
};

// physics.normalize_angle after one frame's turn.  |omega| stays near
// 0.3 / (1 - 0.95) = 6 degrees per frame, so the angle leaves (-540, 540]
// only if the caller wrote such an angle; then the loop form runs (a rare,
// separate branch).  One exact +-360 equals the reference's while-loops
// inside that range (NaN passes through both unchanged).
__device__ __forceinline__ double wrap_angle(double a) {
    double w = a > 180.0 ? a - 360.0 : a;
    w = a < -180.0 ? a + 360.0 : w;
    if (__builtin_expect(fabs(a) > 540.0, 0)) {
        w = trig::normalize_angle(a);
    }
    return w;
}

// One frame of a live lane: Drone.apply_thrust (drone.py:44-76), wind
// (game_engine.py:121-123), Drone.update (drone.py:78-103), Platform.update
// (platform.py:31-49), _calculate_reward with _check_landing / _check_crash /
// _check_out_of_bounds (game_engine.py:179-279).  `k` holds the physics
// (compile-time under kRef), `sw` the call's switches; kRef also means no
// wind and a static platform (their code is not compiled in).  Returns the
// reward.
//
// kFlat (the rollout kernel, one wave per SIMD at its usual size): the
// common path is one basic block.  The thrusters are applied through
// selects (the thrust vector's sincos runs for every lane; a wave almost
// always has a lane firing its main engine anyway) and the angle wrap is a
// select with a rare fallback, so the scheduler can interleave the frame's
// independent chains (sincos, fuel and spin, the two square roots) where
// no other wave fills the stalls: 65,536 x 256 frames 0.424 -> 0.403 ms.
// The step kernel (four waves per SIMD) keeps the branches: selects cost it
// VALU slots the other waves would use.  Only the bottom-centre test near
// the pad (rare) branches in both.
// kDefer (the split rollout's frame waves, reference world, kFlat): the
// frame stops at the flags and the step count.  Speed, distance, the reward
// and the running total are left to the writer wave (finish_deferred), which
// derives them from the frame's state exactly as this function would; the
// landing test's speed limit compares the squared speed (9 = 3^2: for every
// squared speed outside the risky edge band, sqrt(ss) > 3 iff ss > 9; NaN
// fails both).  s.speed, s.dist and s.total are stale on return.
// The thrust's sin and cos of a lane's angle, computed ahead (kPipe).  In a
// loop that keeps the state in registers the thrust of frame f + 1 rotates by
// the angle frame f stored (rounded to the storage width), which is known
// halfway through frame f: the sincos for frame f + 1 (next_trig) then runs
// beside the rest of frame f, off the chain from the angle to vx', x' and the
// flags.  Same function of the same angle: the frame's values are bit for bit
// those of the sincos taken inside it.
struct ThrustTrig {
    double s, c;
};
__device__ __forceinline__ void next_trig(const Lane& s, ThrustTrig& t) { sincos_deg<false>(s.angle, &t.s, &t.c); }

template <bool kRef, bool kFlat, bool kExact = false, bool kDefer = false, bool kPipe = false>
__device__ __forceinline__ double frame(const Consts& k, const DDConfig& sw, uint32_t act, Lane& s, bool* risky_out,
                                        const ThrustTrig* tt = nullptr) {
    static_assert(!kPipe || (kFlat && !kExact), "the pipelined thrust trig is the loops' fast frame");
    static_assert(!kDefer || (kRef && kFlat && !kExact), "deferred frames: reference world, rollout form");
    const DDConfig& c = k.c;

    // apply_thrust: each thruster gated on fuel > 0 at that moment, in order.
    // rotate_point(0, ty, angle) = (0 * ca - ty * sa, 0 * sa + ty * ca)
    // (physics.py:6-23).  Under kRef (ty = -0.6) the zero products drop out
    // exactly: ca and ty * ca are finite and nonzero (cos has no double
    // zero), so 0 * sa + ty * ca = ty * ca; 0 * ca is +0 whenever ty * sa
    // can be zero (sa = +-0 only at angle +-0, where ca = 1), so
    // 0 * ca - ty * sa = 0.6 * sa + 0.0 (the +0.0 turns sa = -0's -0 into
    // the reference's +0; a NaN angle gives NaN both ways).  3 f64 ops fewer.
    const double ty = -c.main_thrust_power;
    constexpr bool kSgpr = !kFlat;  // the step kernel (trig::hstep_c)
    const auto thrust = [&](double sa, double ca, double* dvx, double* dvy) __attribute__((always_inline)) {
        if constexpr (kRef) {
            *dvx = c.main_thrust_power * sa + 0.0;
            *dvy = ty * ca;
        } else {
            *dvx = 0.0 * ca - ty * sa;
            *dvy = 0.0 * sa + ty * ca;
        }
    };
    const bool main_on = (act & 1u) && s.fuel > 0.0;
    if constexpr (kFlat) {
        double sa, ca, dvx, dvy;
        if constexpr (kPipe) {
            sa = tt->s;
            ca = tt->c;
        } else {
            sincos_deg<kExact>(s.angle, &sa, &ca);  // rotate_point(0, -MAIN_THRUST_POWER, angle)   physics.py:6-23
        }
        thrust(sa, ca, &dvx, &dvy);
        s.vx = main_on ? s.vx + dvx : s.vx;
        s.vy = main_on ? s.vy + dvy : s.vy;
        s.fuel = main_on ? s.fuel - c.fuel_main : s.fuel;
        const bool left_on = (act & 2u) && s.fuel > 0.0;
        s.omega = left_on ? s.omega - c.side_thrust_power : s.omega;
        s.fuel = left_on ? s.fuel - c.fuel_side : s.fuel;
        const bool right_on = (act & 4u) && s.fuel > 0.0;
        s.omega = right_on ? s.omega + c.side_thrust_power : s.omega;
        s.fuel = right_on ? s.fuel - c.fuel_side : s.fuel;
    } else {
        if (main_on) {
            double sa, ca, dvx, dvy;
            sincos_deg<kExact, kSgpr>(s.angle, &sa, &ca);  // rotate_point(0, -MAIN_THRUST_POWER, angle)
            thrust(sa, ca, &dvx, &dvy);
            s.vx += dvx;
            s.vy += dvy;
            s.fuel -= c.fuel_main;
        }
        if ((act & 2u) && s.fuel > 0.0) { s.omega -= c.side_thrust_power; s.fuel -= c.fuel_side; }
        if ((act & 4u) && s.fuel > 0.0) { s.omega += c.side_thrust_power; s.fuel -= c.fuel_side; }
    }
    s.fuel = s.fuel > 0.0 ? s.fuel : 0.0;  // max(0, fuel)

    if (!kRef && sw.wind_enabled) { s.vx += sw.wind_x; s.vy += sw.wind_y; }

    s.vy += c.gravity * c.dt;
    s.vx *= c.drag;
    s.vy *= c.drag;
    s.x += s.vx * c.dt;
    s.y += s.vy * c.dt;
    s.angle += s.omega * c.dt;
    s.omega *= c.angular_drag;
    s.angle = kFlat ? wrap_angle(s.angle) : trig::normalize_angle(s.angle);  // (the select form: step +-1 %)

    if (!kRef && sw.platform_moving) {
        const double dir = (s.status & DD_ST_PLAT_LEFT) ? -1.0 : 1.0;
        s.px += c.platform_speed * dir * c.dt;
        if (s.px <= c.platform_min_x) { s.px = c.platform_min_x; s.status &= ~DD_ST_PLAT_LEFT; }
        else if (s.px >= c.platform_max_x) { s.px = c.platform_max_x; s.status |= DD_ST_PLAT_LEFT; }
    }

    // Exactness.  The cascade's predicates are the reference's bit for bit
    // when their inputs are: every operation here is the reference's, but the
    // fast sincos (trig.h) may differ from glibc's by an ulp, and the speed's
    // squares (v*v here, glibc pow there) too.  Those can only flip a flag
    // when a compared quantity lies within a few ulps of its boundary, so the
    // fast frame reports such a lane in *risky_out and the kernel runs its
    // frame again with kExact (glibc's sin, cos and pow: libm_ref.h) out of
    // its hot loop:
    // * x' or y' (thrust-dependent) near an out-of-bounds or ground boundary:
    //   under kRef x', y' rounded to float equal to -50 / 850 / -50 / 550
    //   (within half a float ulp, >= 1.9e-6; four f32 compares on the
    //   conversions the f32 store makes anyway);
    // * on the landing test's lanes (upright, within reach of the pad): the
    //   speed or the bottom centre within 2^-20 of its limit / a pad edge.
    // Under kRef y' = 650 never decides a flag (past 550 the drone has crashed
    // or landed first); fuel, spin and angle involve no transcendental.
    const auto close = [](double q, double b) { return fabs(q - b) <= 0x1p-20 * (1.0 + fabs(b)); };
    bool risky = false;
    if constexpr (!kExact) {
        if constexpr (kRef) {
            constexpr DDConfig r = reference_config();
            static_assert(-r.oob_margin == -50 && r.world_width + r.oob_margin == 850 && r.ground_level == 550,
                          "float boundary constants");
            // |xf - 400| == 450 holds for xf = -50 and 850 (both subtractions
            // exact), and for the few floats within 2^-15 of them that round
            // onto it (harmless: a redo); likewise |yf - 250| == 300.  One
            // compare instead of four compares and three mask ORs: the
            // rollout loop is at its SGPR limit, and every lane mask costs one.
            const float xf = (float)s.x, yf = (float)s.y;
            const float qx = fabsf(fabsf(xf - 400.0f) - 450.0f), qy = fabsf(fabsf(yf - 250.0f) - 300.0f);
            risky = fminf(qx, qy) == 0.0f;
        } else {
            // (y' = world_height + margin too: with a ground level at or past
            // that edge the out-of-bounds test can decide there)
            const bool q0 = close(s.y, c.ground_level), q1 = close(s.x, -c.oob_margin),
                       q2 = close(s.x, c.world_width + c.oob_margin), q3 = close(s.y, -c.oob_margin),
                       q4 = close(s.y, c.world_height + c.oob_margin);
            risky = q0 | q1 | q2 | q3 | q4;
        }
    }

    // speed (get_speed), distance (physics.distance), shared with get_state
    const double ss = kDefer ? s.vx * s.vx + s.vy * s.vy : measure<!kFlat>(s);
    const bool upright = fabs(s.angle) <= c.max_landing_angle;
    bool on_pad = false;  // _check_landing: bottom centre on the platform, slow and upright
    const double rx = c.platform_half_width + fabs(c.drone_half_height);
    const double ry = c.platform_half_height + fabs(c.drone_half_height);
    // |bx - x| <= |half_height| + the rounding of bx, and the rounding of bx,
    // px and their difference stays below 2^-50 (|x| + |px| + |bx - px|) + 1
    // ulp-scale terms: with |px| <= |x| + rx + 1 that is far inside the
    // 2^-30 |x| + 1 of slack taken here (x - px: one rounding; NaN or an
    // infinite x fails the test, as the reference's comparisons fail)
    const bool near_pad = upright && fma(-fabs(s.x), 0x1p-30, fabs(s.x - s.px)) <= rx + 1.0 &&
                          fma(-fabs(s.y), 0x1p-30, fabs(s.y - s.py)) <= ry + 1.0;
    if constexpr (kRef && !kExact) {
        // The fast frame, reference world: one branch, taken by the lanes that
        // are near the pad AND slow.  The speed's edge band is tested on every
        // lane (two VALU) rather than inside a branch of its own.
        const bool edge = fabs(ss - 9.0) <= 0x1p-20;
        static_assert(reference_config().max_landing_velocity == 3.0, "the squared speed limit");
        const bool slow = kDefer ? !(ss > 9.0) : !(s.speed > c.max_landing_velocity);
        risky |= near_pad & edge;
        // Where the branch pays depends on the kernel (profiles/r06/lab/
        // rollout_nearpad_respawn_variants.jsonl, rollout_trigearly.jsonl):
        // the step kernel and the split rollout's frame waves (kDefer) keep it
        // (config 5: 0.2252 / 0.2120 ms with it against 0.2300 / 0.2165
        // without); the single-role loops (kFlat, not kDefer: 262,144 x 256,
        // and the fused policy rollout) form the bottom centre on every lane
        // and mask the tests (0.8548 against 0.8751 ms)
        const bool pad_test = near_pad & slow;
        if ((kFlat && !kDefer) || pad_test) {  // get_bottom_center: rotate_point(0, height / 2, angle), updated angle
            // upright (|angle| <= 20): the small-angle sin / cos, within 3e-13
            // (trig.h); bx, by then lie within 1e-11 of the reference's, far
            // inside the risky band below
            static_assert(reference_config().max_landing_angle == 20.0 &&
                              reference_config().drone_half_height == 10.0 &&
                              reference_config().platform_half_width == 50.0 &&
                              reference_config().platform_half_height == 10.0,
                          "sincos_upright_deg's range; the pad's half extents");
            double sb, cb;
            trig::sincos_upright_deg<kSgpr>(s.angle, &sb, &cb);
            const double bx = s.x - c.drone_half_height * sb;
            const double by = s.y + c.drone_half_height * cb;
            // px - 50 <= bx <= px + 50 as |bx - px| <= 50 (likewise y): the two
            // forms can only disagree where bx lies within a few ulps of an
            // edge, and such a lane is inside the risky band (2^-19 relative,
            // as before) and redone with the reference's own comparisons
            const double dxp = bx - s.px, dyp = by - s.py;
            const bool in_x = fabs(dxp) <= c.platform_half_width, in_y = fabs(dyp) <= c.platform_half_height;
            const bool in_box = in_x & in_y;
            const double m = fmin(fabs(fabs(dxp) - c.platform_half_width), fabs(fabs(dyp) - c.platform_half_height));
            const bool band = m <= 0x1p-19 * (1.0 + fabs(bx) + fabs(by));
            on_pad = pad_test && in_box;
            risky |= pad_test && band;
        }
    } else if (near_pad) {
        // (lanes out of this reach of the pad: on_pad = false exactly as the
        // reference's comparisons give, the bottom centre lying within
        // |half_height| (+ rounding) of (x, y); NaN fails both tests alike)
        const bool edge = kRef ? fabs(ss - 9.0) <= 0x1p-20 : close(s.speed, c.max_landing_velocity);
        bool slow = !(s.speed > c.max_landing_velocity);
        if constexpr (kExact) {
            if (edge) {  // the reference's speed: sqrt(pow(vx, 2) + pow(vy, 2))
                double sq = 0.0, v = s.vx;
#pragma unroll 1
                for (int q = 0; q < 2; ++q) {
                    sq += libm::pow2(v);
                    v = s.vy;
                }
                slow = !(sqrt(sq) > c.max_landing_velocity);
            }
        } else {
            risky |= edge;
        }
        if (slow) {  // get_bottom_center: rotate_point(0, height / 2, angle) on the updated angle
            double sb, cb;
            sincos_deg<kExact, kSgpr>(s.angle, &sb, &cb);
            const double bx = s.x + (0.0 * cb - c.drone_half_height * sb);
            const double by = s.y + (0.0 * sb + c.drone_half_height * cb);
            on_pad = (s.px - c.platform_half_width <= bx) & (bx <= s.px + c.platform_half_width) &
                     (s.py - c.platform_half_height <= by) & (by <= s.py + c.platform_half_height);
            if constexpr (!kExact) {
                // bx or by within 2^-20 (relative) of a pad edge: the nearest
                // edge's distance against one bound that covers close() for
                // every edge (|edge| <= |bx| + |by| + its distance), one compare
                const double m = fmin(fmin(fabs(bx - (s.px - c.platform_half_width)),
                                           fabs(bx - (s.px + c.platform_half_width))),
                                      fmin(fabs(by - (s.py - c.platform_half_height)),
                                           fabs(by - (s.py + c.platform_half_height))));
                risky |= m <= 0x1p-19 * (1.0 + fabs(bx) + fabs(by));
            }
        }
    }
    if constexpr (!kExact) *risky_out = risky;

    // _calculate_reward's cascade, evaluated branch-free: every predicate is
    // formed, then the first that holds picks the term.  (The nested
    // else-if form miscompiled on ROCm 7.2 / gfx950: the divergent-branch phi
    // register of the out-of-bounds term was reused as a temporary, giving
    // 649.9 instead of -50.1; tests/test_gpu_parity.py pins every branch.)
    const bool landing = on_pad;  // _check_landing: on the pad, slow (the reference's speed) and upright
    const bool crash = s.y > c.ground_level;                              // _check_crash, landing ruled out
    const bool no_fuel = s.fuel <= 0.0;
    const bool oob = (s.x < -c.oob_margin) | (s.x > c.world_width + c.oob_margin) |
                     (s.y < -c.oob_margin) | (s.y > c.world_height + c.oob_margin);
    double term = trig::div_exact(c.shaping_offset - s.dist, c.shaping_scale, k.inv_shaping);
    const bool terminal = landing | crash | no_fuel | oob;
    if constexpr (kRef) {
        // config.py's terminal rewards are integers: pick one as an int (one
        // literal per select) and widen it once, instead of selecting doubles
        // (two literal moves and two selects each): dd_rollout 65,536 x 256
        // 0.372 -> 0.365 ms, 262,144 x 256 0.952 -> 0.928 ms
        constexpr DDConfig r = reference_config();
        static_assert(r.reward_landing == 100.0 && r.reward_crash == -100.0 && r.reward_out_of_fuel == -50.0 &&
                      r.reward_out_of_bounds == -50.0, "integer terminal rewards");
        const int32_t ti = landing ? 100 : crash ? -100 : -50;
        term = terminal ? (double)ti : term;
    } else {
        term = oob ? c.reward_out_of_bounds : term;
        term = no_fuel ? c.reward_out_of_fuel : term;
        term = crash ? c.reward_crash : term;
        term = landing ? c.reward_landing : term;
    }
    s.status |= landing ? (DD_ST_LANDED | DD_ST_DONE) : terminal ? (DD_ST_CRASHED | DD_ST_DONE) : 0u;
    if constexpr (kDefer) {  // (the term above is dead code here)
        s.steps += 1;
        return 0.0;
    }
    const double reward = c.reward_step + term;
    s.total += reward;
    s.steps += 1;
    return reward;
}



// The writer wave's half of a kDefer frame: speed and distance of the
// frame's state (measure()'s arithmetic), then _calculate_reward's value and
// the running total as frame() + quantize give them (reference world).
// was_done: the lane started the frame done (auto-reset: re-spawned, reward 0
// and total 0; sticky: reward 0, total kept).
template <typename T>
__device__ __forceinline__ double finish_deferred(Lane& s, bool was_done, bool auto_reset, double& total) {
    constexpr DDConfig r = reference_config();
    const double dx = s.px - s.x, dy = s.py - s.y;
    s.speed = sqrt(s.vx * s.vx + s.vy * s.vy);
    s.dist = sqrt(dx * dx + dy * dy);
    if (was_done) {
        total = auto_reset ? 0.0 : total;
        return 0.0;
    }
    const bool terminal = (s.status & DD_ST_DONE) != 0;
    const int32_t ti = (s.status & DD_ST_LANDED) ? 100 : s.y > r.ground_level ? -100 : -50;
    double term = trig::div_exact(r.shaping_offset - s.dist, r.shaping_scale, kRefConsts.inv_shaping);
    term = terminal ? (double)ti : term;
    const double reward = r.reward_step + term;
    total = (double)(T)(total + reward);
    return reward;
}

// A frame for kernels that keep the lane's state in registers (the rollout
// loops): the fast frame, and for a lane it reports risky the frame again
// from the kept state with glibc's functions (a wave-uniform rare branch; as
// an out-of-line call, or through an LDS slot, it measured slower or equal,
// DESIGN.md §3.2).
// kPipe: *tt holds the sin / cos of the frame's starting angle and receives
// those of the next frame's, i.e. of this frame's angle rounded to the
// storage width TQ.  Taken before the redo's branch, beside the frame's flag
// tests: the angle update has no transcendental, so the exact redo ends on
// the same angle.  (A re-spawn after the frame resets it to (+0, 1).)
template <bool kRef, bool kFlat, bool kDefer = false, bool kPipe = false, typename TQ = double>
__device__ __forceinline__ double frame_checked(const Consts& k, const DDConfig& sw, uint32_t act, Lane& s,
                                                ThrustTrig* tt = nullptr) {
    const Lane s0 = s;  // (in an LDS slot instead: config 5 0.215 -> 0.226 ms, profiles/r06/lab/rollout_s0lds.jsonl)
    bool risky = false;
    double reward = frame<kRef, kFlat, false, kDefer, kPipe>(k, sw, act, s, &risky, tt);
    if constexpr (kPipe) sincos_deg<false>((double)(TQ)s.angle, &tt->s, &tt->c);
    if (__builtin_expect(__ballot(risky) != 0, 0)) {
        if (risky) {
            s = s0;
            reward = frame<kRef, false, true>(k, sw, act, s, nullptr);
        }
    }
    return reward;
}

// DroneGame.get_state (game_engine.py:140-177) in state_to_array order, as
// doubles (columns 0-12; 13/14 are the landed / crashed flags); measure() has
// run on `s`.  kExactDiv: the reference's quotients bit for bit (x / d by
// trig::div_exact, 3 ops) — the notebook reward consumes these doubles.
// Otherwise x * RN(1/d), one op per column: within one double ulp of the
// quotient, and identical after the float32 rounding of an observation row
// except when the quotient lies within ~1e-16 relative of a float32 rounding
// boundary (0 of 2e7 random values per divisor, 0 of the integer spawn
// positions: tools/obs_mul_check.py) — inside the rows' 1-ulp contract.
// Saves 26 of the rollout frame's ~360 VALU ops.
template <bool kGuard = false, bool kExactDiv = false>
__device__ __forceinline__ void observe_values(const Consts& k, const Lane& s, double v[13]) {
    const DDConfig& c = k.c;
    const double dx = s.px - s.x, dy = s.py - s.y;
#define DD_Q(x, d, inv) \
    (!kExactDiv ? (x) * (inv) : kGuard ? trig::div_exact_guarded((x), (d), (inv)) : trig::div_exact((x), (d), (inv)))
    v[0] = DD_Q(s.x, c.world_width, k.inv_w);
    v[1] = DD_Q(s.y, c.world_height, k.inv_h);
    v[2] = DD_Q(s.vx, c.vel_scale, k.inv_vel);
    v[3] = DD_Q(s.vy, c.vel_scale, k.inv_vel);
    v[4] = DD_Q(s.angle, c.angle_scale, k.inv_angle);
    v[5] = DD_Q(s.omega, c.vel_scale, k.inv_vel);
    v[6] = DD_Q(s.fuel, c.max_fuel, k.inv_fuel);
    v[7] = DD_Q(s.px, c.world_width, k.inv_w);
    v[8] = DD_Q(s.py, c.world_height, k.inv_h);
    v[9] = DD_Q(s.dist, c.world_width, k.inv_w);
    v[10] = DD_Q(dx, c.world_width, k.inv_w);
    v[11] = DD_Q(dy, c.world_height, k.inv_h);
    v[12] = DD_Q(s.speed, c.vel_scale, k.inv_vel);
#undef DD_Q
}

__device__ __forceinline__ void write_obs_row(const double v[13], uint32_t status, float* o) {
#pragma unroll
    for (int j = 0; j < 13; ++j) o[j] = (float)v[j];
    o[13] = (status & DD_ST_LANDED) ? 1.0f : 0.0f;
    o[14] = (status & DD_ST_CRASHED) ? 1.0f : 0.0f;
}

template <bool kGuard = false>
__device__ __forceinline__ void observe(const Consts& k, const Lane& s, float* o) {
    double v[13];
    observe_values<kGuard>(k, s, v);
    write_obs_row(v, s.status, o);
}

// The notebooks' shaped rewards a kernel fuses (kShape): none (the engine's
// reward only), PPO's calc_reward(state, prev_state) with its two-frame
// history, REINFORCE's calc_reward(state).
enum { kShapeNone = 0, kShapePpo = 1, kShapeReinforce = 2 };

// calc_reward(state, prev_state)['total'] of Actor_Critic_PPO.ipynb:164-263
// (scalers: rl_helpers/scalers.py) on the frame's double observation `v`;
// prev_dist is prev_state.distance_to_platform, NaN for prev_state None.  The
// terms are summed in the notebook's order.  Branch-free (see frame()).
__device__ __forceinline__ double notebook_reward(const double v[13], uint32_t status, double prev_dist) {
    const double vx = v[2], vy = v[3], angle = v[4], fuel = v[6], dist = v[9], dx = v[10], dy = v[11],
                 speed = v[12];
    const bool have_prev = !__builtin_isnan(prev_dist);
    const double delta = prev_dist - dist;
    const double vtp = dist > 1e-6 ? (vx * dx + vy * dy) / dist : 0.0;  // velocity toward platform
    const bool fast_toward = (speed >= 0.15) & (vtp > 0.1) & (dist > 0.065);
    const double clipped = fmin(fmax(delta * 1000 * (1.0 + speed * 2.0), -2.0), 5.0);  // np.clip
    const bool away = !fast_toward & (delta < -0.001);
    double distance = fast_toward ? clipped : away ? -2.0 * fabs(delta) * 1000 : 0.0;
    double hovering = (fast_toward | away) ? 0.0 : speed < 0.05 ? -1.0 : speed < 0.15 ? -0.3 : 0.0;
    distance = have_prev ? distance : 0.0;
    hovering = have_prev ? hovering : 0.0;
    double total = 0.0;
    total += -0.5;
    total += distance;
    total += hovering;
    const double excess = fabs(angle) - (((0.20 - 0.111) * dist) + 0.111);
    total += -(excess > 0.0 ? excess : 0.0);
    const double over = dist < 1 ? speed - 0.1 : speed - 0.6;
    total += (dist < 1 ? -2.0 : -1.0) * (over > 0.0 ? over : 0.0);
    total += dy > 0.0 ? 0.0 : dy * 4.0;
    const bool landed = status & DD_ST_LANDED, crashed = status & DD_ST_CRASHED;
    const double crash_term = dist > 0.3 ? -200.0 - 100.0 : -200.0;
    total += landed ? 800.0 + fuel * 100.0 : crashed ? crash_term : 0.0;
    return total;
}

// calc_reward(state)['total'] of Policy_Gradients.ipynb:162-238 (the REINFORCE
// notebook; velocity alignment :128-153, scalers rl_helpers/scalers.py) on
// the frame's double observation `v`.  No prev_state.  The terms are summed
// in the notebook's order, each formed as the notebook's Python evaluates it
// (`x**2` as x*x: glibc's pow(x, 2) may differ by an ulp; exp is the device
// library's): within a few ulps of the notebook's value, as the PPO reward.
__device__ __forceinline__ double reinforce_reward(const double v[13], uint32_t status) {
    const double vx = v[2], vy = v[3], angle = v[4], fuel = v[6], dist = v[9], dx = v[10], dy = v[11],
                 speed = v[12];
    // time penalty: -inverse_quadratic(dist, decay=50, scaler=1-0.3) - 0.3
    constexpr double kScale = 1.0 - 0.3;  // 0.69999999999999996 = RN(0.7), as Python forms 1 - 0.3
    const double time_penalty = -(kScale * (1.0 / (1.0 + (50.0 * (dist * dist))))) - 0.3;
    // calc_velocity_alignment: only its sign is used
    const double odx0 = -dx, ody0 = -dy;
    const double onorm = sqrt(odx0 * odx0 + ody0 * ody0);
    const double odx = odx0 / onorm, ody = ody0 / onorm;
    const double align_v = (vx / speed) * odx + (vy / speed) * ody;
    const double align = onorm < 1e-6 ? 1.0 : speed < 1e-6 ? 0.0 : align_v;
    // distance and velocity-alignment terms, only above the platform
    const bool above = (dist > 0.065) & (dy > 0.0);
    const double sig = 4.5 * (1.0 / (1.0 + exp(10.0 * (dist - 0.5))));  // scaled_shifted_negative_sigmoid
    const double distance = above ? ((align > 0.0 ? 1.0 : 0.0) * speed) * sig : 0.0;
    const double valign = (above & (align > 0.0)) ? 0.5 : 0.0;
    double total = time_penalty;
    total += distance;
    total += valign;
    const double excess = fabs(angle) - (((0.20 - 0.111) * dist) + 0.111);
    total += -(excess > 0.0 ? excess : 0.0);
    const double over = dist < 1 ? speed - 0.1 : speed - 0.4;
    total += (dist < 1 ? -2.0 : -1.0) * (over > 0.0 ? over : 0.0);
    total += dy > 0.0 ? 0.0 : dy * 4.0;
    const bool landed = status & DD_ST_LANDED, crashed = status & DD_ST_CRASHED;
    const double crash_term = dist > 0.3 ? -200.0 - 100.0 : -200.0;
    total += landed ? 500.0 + fuel * 100.0 : crashed ? crash_term : 0.0;
    return total;
}

// element i of a lane array (i < kChunk)
template <typename E>
__device__ __forceinline__ E& at(E* base, uint32_t i) {
    using B = typename std::conditional<std::is_const<E>::value, const char, char>::type;
    return *reinterpret_cast<E*>(reinterpret_cast<B*>(base) + (uint32_t)(i * (uint32_t)sizeof(E)));
}

// A wave-uniform pointer the compiler cannot prove uniform (it comes from
// threadIdx-derived arithmetic, or is hoisted into a VGPR), moved to SGPRs so
// loads and stores use the SGPR-base + 32-bit lane offset form and its
// arithmetic stays on the scalar unit.
template <typename P>
__device__ __forceinline__ P* uniform_ptr(P* q) {
    const uint64_t v = reinterpret_cast<uint64_t>(q);
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    return reinterpret_cast<P*>(((uint64_t)hi << 32) | lo);
}

// The state between two frames is what dd_step would store: rounded to the
// storage width T (a no-op for double).
// Under kRef the pad is static: px / py only change on a re-spawn, to
// integers, which every storage width holds exactly.
template <typename T, bool kRef = false>
__device__ __forceinline__ void quantize(Lane& s) {
    s.x = (T)s.x; s.y = (T)s.y; s.vx = (T)s.vx; s.vy = (T)s.vy; s.angle = (T)s.angle;
    s.omega = (T)s.omega; s.fuel = (T)s.fuel; s.total = (T)s.total;
    if constexpr (!kRef) { s.px = (T)s.px; s.py = (T)s.py; }
}

// The SoA of one batch (DDState) with typed pointers, offset to lane `first`.
template <typename T>
struct Soa {
    T *x, *y, *vx, *vy, *angle, *omega, *fuel, *px, *py, *total;
    uint8_t* status;
    int32_t *steps, *episode;
    int64_t env_id_base;
};

template <typename T>
Soa<T> soa_of(const DDState& st, int64_t first) {
    Soa<T> s;
    s.x = (T*)st.x + first; s.y = (T*)st.y + first; s.vx = (T*)st.vx + first; s.vy = (T*)st.vy + first;
    s.angle = (T*)st.angle + first; s.omega = (T*)st.omega + first; s.fuel = (T*)st.fuel + first;
    s.px = (T*)st.px + first; s.py = (T*)st.py + first; s.total = (T*)st.total_reward + first;
    s.status = st.status + first; s.steps = st.steps + first; s.episode = st.episode + first;
    s.env_id_base = st.env_id_base + first;
    return s;
}

inline bool state_ok(const DDState* st) {
    return st && st->x && st->y && st->vx && st->vy && st->angle && st->omega && st->fuel && st->px &&
           st->py && st->total_reward && st->status && st->steps && st->episode &&
           (st->precision == DD_F32 || st->precision == DD_F64);
}
}  // namespace dd
