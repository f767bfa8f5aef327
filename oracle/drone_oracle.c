/*
 * drone_oracle.c — TEST INFRASTRUCTURE ONLY.  CPU restatement of the
 * reference's delivery-drone frame, used as the parity checker for the HIP
 * path (tests/, __graft_entry__.smoke(), bench.py's cpu_baseline leg).
 * Nothing in the product package links, loads or calls this file.
 *
 * Restated from vedant-jumle/reinforcement-learning-101 (read, not copied):
 *   delivery_drone/game/config.py:17-68      constants (DDConfig defaults)
 *   delivery_drone/game/physics.py:6-44      rotate_point, normalize_angle, distance
 *   delivery_drone/game/drone.py:44-153      apply_thrust, update, bottom centre, speed, upright
 *   delivery_drone/game/platform.py:31-74    update, bounds, point-on-platform
 *   delivery_drone/game/game_engine.py:59-298 reset, step, get_state, reward, checks, info
 *
 * Every quantity is an IEEE double, in the reference's operation order, so
 * that on this image's glibc the results equal the Python reference bit for
 * bit (pinned by tests/golden/, generated from the reference itself):
 *   - np.radians(a) is a * (pi / 180)           (numpy deg2rad)
 *   - np.cos / np.sin are libm cos / sin         (numpy float64 loops)
 *   - v ** 2 is libm pow(v, 2.0)                 (CPython float_pow and numpy
 *     scalar power both call pow(); it differs from v * v in ~0.09 % of cases,
 *     so it is called through a pointer the compiler cannot fold)
 *   - np.sqrt is the correctly rounded sqrt.
 * Spawn positions use Philox4x32-10 keyed by (seed; env id, episode), the
 * product's documented RNG contract; the reference draws them from numpy's
 * global MT19937, which no batched engine can reproduce.
 *
 * Build (oracle/Makefile): gcc -O2 -fno-builtin -ffp-contract=off -fPIC -shared
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/dronestep.h"

static double (*volatile ora_pow)(double, double) = pow;
static double (*volatile ora_sin)(double) = sin;
static double (*volatile ora_cos)(double) = cos;
static double (*volatile ora_exp)(double) = exp;

#define ORA_PI 3.141592653589793238462643383279502884

typedef struct OraLane {
    double x, y, vx, vy, angle, omega, fuel, px, py, total;
    uint32_t status;
    int32_t steps, episode;
} OraLane;

/* ---- Philox4x32-R: 10 rounds (actions, policy samples), 7 (spawns) -------*/
static void philox4x32_r(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4], int rounds) {
    uint32_t c0 = ctr[0], c1 = ctr[1], c2 = ctr[2], c3 = ctr[3];
    uint32_t k0 = key[0], k1 = key[1];
    for (int round = 0; round < rounds; ++round) {
        uint64_t a = (uint64_t)0xD2511F53u * c0;
        uint64_t b = (uint64_t)0xCD9E8D57u * c2;
        uint32_t n0 = (uint32_t)(b >> 32) ^ c1 ^ k0;
        uint32_t n2 = (uint32_t)(a >> 32) ^ c3 ^ k1;
        c1 = (uint32_t)b;
        c3 = (uint32_t)a;
        c0 = n0;
        c2 = n2;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

void ora_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) {
    philox4x32_r(ctr, key, out, 10);
}

/* The spawn stream (frame.h spawn_words): Philox4x32-7 since round 6. */
void ora_philox4x32_7(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) {
    philox4x32_r(ctr, key, out, 7);
}

static int32_t pick(uint32_t r, int32_t lo, uint32_t span) {
    return lo + (int32_t)(((uint64_t)r * span) >> 32);
}

/* ---- physics.py ----------------------------------------------------------*/
/* rotate_point(x, y, angle_deg) with x == 0 (the only form step() uses). */
static void rotate_y(double y, double angle_deg, double *ox, double *oy) {
    double rad = angle_deg * (ORA_PI / 180.0);
    double ca = ora_cos(rad), sa = ora_sin(rad);
    *ox = 0.0 * ca - y * sa;
    *oy = 0.0 * sa + y * ca;
}

static double wrap_degrees(double a) {
    /* physics.normalize_angle's loops.  Past |a| = 2^55, a - 360 == a and the
     * reference never returns; the oracle reports NaN there instead of hanging. */
    if (!(fabs(a) < 36028797018963968.0)) return fabs(a) < INFINITY ? NAN : a;
    while (a > 180.0) a -= 360.0;
    while (a < -180.0) a += 360.0;
    return a;
}

static double dist2d(double x1, double y1, double x2, double y2) {
    return sqrt(ora_pow(x2 - x1, 2.0) + ora_pow(y2 - y1, 2.0));
}

static double speed_of(const OraLane *s) { return sqrt(ora_pow(s->vx, 2.0) + ora_pow(s->vy, 2.0)); }

/* ---- game_engine.py reset ------------------------------------------------*/
void ora_spawn(const DDConfig *c, int64_t env, OraLane *s) {
    s->episode += 1;
    uint32_t ctr[4] = {(uint32_t)env, (uint32_t)((uint64_t)env >> 32), (uint32_t)s->episode, 0u};
    uint32_t key[2] = {(uint32_t)c->seed, (uint32_t)(c->seed >> 32)};
    uint32_t r[4];
    ora_philox4x32_7(ctr, key, r);
    if (c->randomize_drone) {
        s->x = pick(r[0], c->drone_x_min, (uint32_t)(c->drone_x_max - c->drone_x_min + 1));
        s->y = pick(r[1], c->drone_y_min, (uint32_t)(c->drone_y_max - c->drone_y_min + 1));
    } else {
        s->x = c->drone_start_x;
        s->y = c->drone_start_y;
    }
    if (c->randomize_platform) {
        s->px = pick(r[2], c->platform_x_lo, (uint32_t)(c->platform_x_hi - c->platform_x_lo));
        s->py = pick(r[3], c->platform_y_lo, (uint32_t)(c->platform_y_hi - c->platform_y_lo));
    } else {
        s->px = c->platform_start_x;
        s->py = c->platform_start_y;
    }
    s->vx = s->vy = s->angle = s->omega = 0.0;
    s->fuel = c->max_fuel;
    s->status = 0;
    s->steps = 0;
    s->total = 0.0;
}

/* ---- game_engine.py step (live lane) ------------------------------------*/
static int on_platform(const DDConfig *c, const OraLane *s, double bx, double by) {
    double left = s->px - c->platform_half_width, right = s->px + c->platform_half_width;
    double top = s->py - c->platform_half_height, bottom = s->py + c->platform_half_height;
    return (left <= bx && bx <= right) && (top <= by && by <= bottom);
}

double ora_frame(const DDConfig *c, uint32_t act, OraLane *s) {
    /* Drone.apply_thrust */
    if ((act & 1u) && s->fuel > 0) {
        double tx, ty;
        rotate_y(-c->main_thrust_power, s->angle, &tx, &ty);
        s->vx += tx;
        s->vy += ty;
        s->fuel -= c->fuel_main;
    }
    if ((act & 2u) && s->fuel > 0) { s->omega -= c->side_thrust_power; s->fuel -= c->fuel_side; }
    if ((act & 4u) && s->fuel > 0) { s->omega += c->side_thrust_power; s->fuel -= c->fuel_side; }
    if (!(s->fuel > 0)) s->fuel = 0.0;
    /* wind */
    if (c->wind_enabled) { s->vx += c->wind_x; s->vy += c->wind_y; }
    /* Drone.update */
    s->vy += c->gravity * c->dt;
    s->vx *= c->drag;
    s->vy *= c->drag;
    s->x += s->vx * c->dt;
    s->y += s->vy * c->dt;
    s->angle += s->omega * c->dt;
    s->omega *= c->angular_drag;
    s->angle = wrap_degrees(s->angle);
    /* Platform.update */
    if (c->platform_moving) {
        double dir = (s->status & DD_ST_PLAT_LEFT) ? -1.0 : 1.0;
        s->px += c->platform_speed * dir * c->dt;
        if (s->px <= c->platform_min_x) { s->px = c->platform_min_x; s->status &= ~(uint32_t)DD_ST_PLAT_LEFT; }
        else if (s->px >= c->platform_max_x) { s->px = c->platform_max_x; s->status |= DD_ST_PLAT_LEFT; }
    }
    /* _calculate_reward */
    double reward = c->reward_step;
    double ox, oy;
    rotate_y(c->drone_half_height, s->angle, &ox, &oy);
    double bx = s->x + ox, by = s->y + oy;
    int landing = on_platform(c, s, bx, by) && !(speed_of(s) > c->max_landing_velocity) &&
                  fabs(s->angle) <= c->max_landing_angle;
    int crash = 0;
    if (!landing && s->y > c->ground_level) {
        crash = !on_platform(c, s, bx, by) || speed_of(s) > c->max_landing_velocity ||
                !(fabs(s->angle) <= c->max_landing_angle);
    }
    if (landing) {
        s->status |= DD_ST_LANDED | DD_ST_DONE;
        reward += c->reward_landing;
    } else if (crash) {
        s->status |= DD_ST_CRASHED | DD_ST_DONE;
        reward += c->reward_crash;
    } else if (s->fuel <= 0) {
        s->status |= DD_ST_CRASHED | DD_ST_DONE;
        reward += c->reward_out_of_fuel;
    } else if (s->x < -c->oob_margin || s->x > c->world_width + c->oob_margin || s->y < -c->oob_margin ||
               s->y > c->world_height + c->oob_margin) {
        s->status |= DD_ST_CRASHED | DD_ST_DONE;
        reward += c->reward_out_of_bounds;
    } else {
        double d = dist2d(s->x, s->y, s->px, s->py);
        reward += (c->shaping_offset - d) / c->shaping_scale;
    }
    s->total += reward;
    s->steps += 1;
    return reward;
}

/* ---- get_state / _get_info ------------------------------------------------*/
void ora_observe(const DDConfig *c, const OraLane *s, double o[DD_OBS_DIM]) {
    double dx = s->px - s->x, dy = s->py - s->y;
    double d = dist2d(s->x, s->y, s->px, s->py);
    o[0] = s->x / c->world_width;
    o[1] = s->y / c->world_height;
    o[2] = s->vx / c->vel_scale;
    o[3] = s->vy / c->vel_scale;
    o[4] = s->angle / c->angle_scale;
    o[5] = s->omega / c->vel_scale;
    o[6] = s->fuel / c->max_fuel;
    o[7] = s->px / c->world_width;
    o[8] = s->py / c->world_height;
    o[9] = d / c->world_width;
    o[10] = dx / c->world_width;
    o[11] = dy / c->world_height;
    o[12] = speed_of(s) / c->vel_scale;
    o[13] = (s->status & DD_ST_LANDED) ? 1.0 : 0.0;
    o[14] = (s->status & DD_ST_CRASHED) ? 1.0 : 0.0;
}

/* ---- the notebooks' shaped reward ----------------------------------------*/
/* calc_reward(state, prev_state)['total'], Actor_Critic_PPO.ipynb:164-263;
 * o = get_state's doubles (state_to_array order), prev_dist NaN = None. */
double ora_notebook_reward(const double o[DD_OBS_DIM], double prev_dist) {
    double vx = o[2], vy = o[3], angle = o[4], fuel = o[6], dist = o[9], dx = o[10], dy = o[11], speed = o[12];
    int landed = o[13] != 0.0, crashed = o[14] != 0.0;
    double total = 0;
    total += -0.5;
    double distance = 0, hovering = 0;
    if (!isnan(prev_dist)) {
        double delta = prev_dist - dist;
        double vtp = 0.0;
        if (dist > 1e-6) vtp = (vx * dx + vy * dy) / dist;
        if (speed >= 0.15 && vtp > 0.1 && dist > 0.065) {
            double mult = 1.0 + speed * 2.0;
            double v = delta * 1000 * mult;
            distance = v < -2 ? -2 : (v > 5 ? 5 : v); /* np.clip */
        } else if (delta < -0.001) {
            distance = -2.0 * fabs(delta) * 1000;
            hovering = 0;
        } else if (speed < 0.05) {
            hovering = -1.0;
        } else if (speed < 0.15) {
            hovering = -0.3;
        } else {
            distance = 0.0;
        }
    }
    total += distance;
    total += hovering;
    double max_permissible = ((0.20 - 0.111) * dist) + 0.111;
    double excess = fabs(angle) - max_permissible;
    total += -(excess > 0 ? excess : 0);
    if (dist < 1) total += -2 * ((speed - 0.1) > 0 ? speed - 0.1 : 0);
    else total += -1 * ((speed - 0.6) > 0 ? speed - 0.6 : 0);
    if (dy > 0) total += 0;
    else total += dy * 4.0;
    double terminal = 0;
    if (landed) {
        terminal = 800.0 + fuel * 100.0;
    } else if (crashed) {
        terminal = -200.0;
        if (dist > 0.3) terminal -= 100.0;
    }
    total += terminal;
    return total;
}

/* calc_reward(state)['total'] of the REINFORCE notebook, Policy_Gradients.ipynb:
 * 162-238, with calc_velocity_alignment (:128-153) and rl_helpers/scalers.py's
 * inverse_quadratic / scaled_shifted_negative_sigmoid, as its Python
 * evaluates them (`x**2` = pow(x, 2), math.exp = exp, int * float products). */
double ora_reinforce_reward(const double o[DD_OBS_DIM]) {
    double vx = o[2], vy = o[3], angle = o[4], fuel = o[6], dist = o[9], dx = o[10], dy = o[11], speed = o[12];
    int landed = o[13] != 0.0, crashed = o[14] != 0.0;
    double total = 0;
    /* -inverse_quadratic(dist, decay=50, scaler=1 - 0.3) - 0.3 */
    double time_penalty = -((1 - 0.3) * (1 / (1 + (50 * ora_pow(dist, 2))))) - 0.3;
    total += time_penalty;
    double odx = -dx, ody = -dy, align;
    double onorm = sqrt(ora_pow(odx, 2) + ora_pow(ody, 2));
    if (onorm < 1e-6) {
        align = 1.0;
    } else {
        odx /= onorm;
        ody /= onorm;
        if (speed < 1e-6) {
            align = 0.0;
        } else {
            double vdx = vx / speed, vdy = vy / speed;
            align = vdx * odx + vdy * ody;
        }
    }
    double distance = 0, valign = 0;
    if (dist > 0.065 && dy > 0) {
        double sig = 4.5 * (1 / (1 + ora_exp(10 * (dist - 0.5))));
        distance = (double)(align > 0) * speed * sig;
        if (align > 0) valign = 0.5;
    }
    total += distance;
    total += valign;
    double excess = fabs(angle) - (((0.20 - 0.111) * dist) + 0.111);
    total += -(excess > 0 ? excess : 0);
    if (dist < 1) total += -2 * ((speed - 0.1) > 0 ? speed - 0.1 : 0);
    else total += -1 * ((speed - 0.4) > 0 ? speed - 0.4 : 0);
    if (!(dy > 0)) total += dy * 4.0;
    double terminal = 0;
    if (landed) {
        terminal = 500.0 + fuel * 100.0;
    } else if (crashed) {
        terminal = -200.0;
        if (dist > 0.3) terminal -= 100.0;
    }
    total += terminal;
    return total;
}

/* ---- SoA batch entry points (host arrays, DDState layout) ----------------*/
#define FLD(name) (st->precision == DD_F64 ? ((double *)st->name)[i] : (double)((float *)st->name)[i])
#define PUT(name, v)                                                \
    do {                                                            \
        if (st->precision == DD_F64) ((double *)st->name)[i] = (v); \
        else ((float *)st->name)[i] = (float)(v);                   \
    } while (0)

static void load_lane(const DDState *st, int64_t i, OraLane *s) {
    s->x = FLD(x); s->y = FLD(y); s->vx = FLD(vx); s->vy = FLD(vy);
    s->angle = FLD(angle); s->omega = FLD(omega); s->fuel = FLD(fuel);
    s->px = FLD(px); s->py = FLD(py); s->total = FLD(total_reward);
    s->status = st->status[i];
    s->steps = st->steps[i];
    s->episode = st->episode[i];
}

static void store_lane(const DDState *st, int64_t i, const OraLane *s) {
    PUT(x, s->x); PUT(y, s->y); PUT(vx, s->vx); PUT(vy, s->vy);
    PUT(angle, s->angle); PUT(omega, s->omega); PUT(fuel, s->fuel);
    PUT(px, s->px); PUT(py, s->py); PUT(total_reward, s->total);
    st->status[i] = (uint8_t)s->status;
    st->steps[i] = s->steps;
    st->episode[i] = s->episode;
}

static void emit_obs(const DDConfig *c, const OraLane *s, int64_t i, float *obs, double *obs64) {
    if (!obs && !obs64) return;
    double o[DD_OBS_DIM];
    ora_observe(c, s, o);
    for (int k = 0; k < DD_OBS_DIM; ++k) {
        if (obs) obs[i * DD_OBS_DIM + k] = (float)o[k];
        if (obs64) obs64[i * DD_OBS_DIM + k] = o[k];
    }
}

/* dd_step semantics over host arrays; actions are DD_ACT_BITMASK bytes.
 * reward is float or double by st->precision.  shaped/shaped_done add the
 * notebooks' reward: mode DD_SHAPED_PPO with hist ([2][n] doubles, slot
 * steps & 1 holds the distance of the state two frames back, NaN = None),
 * DD_SHAPED_REINFORCE without; max_steps > 0 adds the collection loops'
 * timeout. */
int ora_step_shaped(const DDConfig *c, const DDState *st, const uint8_t *actions, void *reward, uint8_t *done,
                    float *obs, double *obs64, double *hist, void *shaped, uint8_t *shaped_done,
                    int32_t max_steps, int32_t mode, int64_t n) {
    for (int64_t i = 0; i < n; ++i) {
        OraLane s;
        load_lane(st, i, &s);
        double r = 0.0, sr = 0.0;
        int sd = 0;
        if (s.status & DD_ST_DONE) {
            if (c->auto_reset) {
                ora_spawn(c, st->env_id_base + i, &s);
                if (hist && mode == DD_SHAPED_PPO) {
                    hist[i] = dist2d(s.x, s.y, s.px, s.py) / c->world_width;
                    hist[n + i] = NAN;
                }
            } else {
                sd = 1;
            }
        } else {
            r = ora_frame(c, actions[i], &s);
            if (shaped) {
                double o[DD_OBS_DIM];
                ora_observe(c, &s, o);
                if (mode == DD_SHAPED_REINFORCE) {
                    sr = ora_reinforce_reward(o);
                } else {
                    double *slot = hist + (s.steps & 1) * n;
                    sr = ora_notebook_reward(o, slot[i]);
                    slot[i] = o[9];
                }
                sd = (s.status & DD_ST_DONE) != 0;
                if (max_steps > 0 && s.steps >= max_steps) {
                    if (!(s.status & DD_ST_LANDED)) sr -= 500;
                    sd = 1;
                    s.status |= DD_ST_DONE;
                }
            }
        }
        store_lane(st, i, &s);
        if (st->precision == DD_F64) ((double *)reward)[i] = r;
        else ((float *)reward)[i] = (float)r;
        done[i] = (s.status & DD_ST_DONE) ? 1 : 0;
        if (shaped) {
            if (st->precision == DD_F64) ((double *)shaped)[i] = sr;
            else ((float *)shaped)[i] = (float)sr;
            shaped_done[i] = (uint8_t)sd;
        }
        emit_obs(c, &s, i, obs, obs64);
    }
    return 0;
}

int ora_step(const DDConfig *c, const DDState *st, const uint8_t *actions, void *reward, uint8_t *done,
             float *obs, double *obs64, int64_t n) {
    return ora_step_shaped(c, st, actions, reward, done, obs, obs64, NULL, NULL, NULL, 0, DD_SHAPED_PPO, n);
}

/* Threshold probing (tests/threshold_states.py): the post-update quantities
 * the reward cascade compares, for a live lane stepped with `actions` — x', y',
 * speed', angle', the bottom centre (bx', by') and vx', vy' — as q[i*8 + 0..7].  The
 * lanes' state is not modified. */
int ora_probe(const DDConfig *c, const DDState *st, const uint8_t *actions, double *q, int64_t n) {
    for (int64_t i = 0; i < n; ++i) {
        OraLane s;
        load_lane(st, i, &s);
        s.status = 0;
        ora_frame(c, actions[i], &s);
        double ox, oy;
        rotate_y(c->drone_half_height, s.angle, &ox, &oy);
        q[i * 8 + 0] = s.x;
        q[i * 8 + 1] = s.y;
        q[i * 8 + 2] = speed_of(&s);
        q[i * 8 + 3] = s.angle;
        q[i * 8 + 4] = s.x + ox;
        q[i * 8 + 5] = s.y + oy;
        q[i * 8 + 6] = s.vx;
        q[i * 8 + 7] = s.vy;
    }
    return 0;
}

int ora_reset(const DDConfig *c, const DDState *st, const uint8_t *mask, float *obs, double *obs64, int64_t n) {
    for (int64_t i = 0; i < n; ++i) {
        if (mask && !mask[i]) continue;
        OraLane s;
        load_lane(st, i, &s);
        ora_spawn(c, st->env_id_base + i, &s);
        store_lane(st, i, &s);
        emit_obs(c, &s, i, obs, obs64);
    }
    return 0;
}

int ora_write_obs(const DDConfig *c, const DDState *st, float *obs, double *obs64, int64_t n) {
    for (int64_t i = 0; i < n; ++i) {
        OraLane s;
        load_lane(st, i, &s);
        emit_obs(c, &s, i, obs, obs64);
    }
    return 0;
}

int ora_get_info(const DDConfig *c, const DDState *st, double *distance, double *speed, int64_t n) {
    (void)c;
    for (int64_t i = 0; i < n; ++i) {
        OraLane s;
        load_lane(st, i, &s);
        if (distance) distance[i] = dist2d(s.x, s.y, s.px, s.py);
        if (speed) speed[i] = speed_of(&s);
    }
    return 0;
}

/* CPU baseline: `n` lanes x `steps` frames of the config-3 workload
 * (randomised spawn, auto-reset, uniform 3-bit actions from Philox keyed by
 * (seed ^ 0xA5, env, step)).  Lanes [lane0, lane0 + n) of the global batch.
 * Returns a checksum of rewards so the loop cannot be elided. */
double ora_bench(const DDConfig *c, int64_t lane0, int64_t n, int64_t steps) {
    OraLane *lanes = (OraLane *)calloc((size_t)(n > 0 ? n : 1), sizeof(OraLane));
    if (!lanes) return NAN;
    double sum = 0.0;
    double o[DD_OBS_DIM];
    for (int64_t i = 0; i < n; ++i) ora_spawn(c, lane0 + i, &lanes[i]);
    const uint32_t key[2] = {(uint32_t)c->seed ^ 0xA5u, (uint32_t)(c->seed >> 32)};
    for (int64_t t = 0; t < steps; ++t) {
        for (int64_t i = 0; i < n; ++i) {
            OraLane *s = &lanes[i];
            uint32_t ctr[4] = {(uint32_t)(lane0 + i), (uint32_t)((uint64_t)(lane0 + i) >> 32), (uint32_t)t, 1u};
            uint32_t r[4];
            ora_philox4x32_10(ctr, key, r);
            double rew = 0.0;
            if (s->status & DD_ST_DONE) ora_spawn(c, lane0 + i, s);
            else rew = ora_frame(c, r[0] & 7u, s);
            ora_observe(c, s, o);
            sum += rew + o[9];
        }
    }
    free(lanes);
    return sum;
}

/* compute_gae (Actor_Critic_PPO.ipynb:733-787) for every column of a
 * [T][n] float32 rollout; torch float32 semantics: Python-float gamma is
 * rounded to float32 where it meets a tensor, gamma * lambda_ is formed in
 * double first. */
void ora_gae(const float *rewards, const float *values, const uint8_t *dones, float *adv, int64_t T, int64_t n,
             double gamma, double lambda) {
    const float g = (float)gamma, gl = (float)(gamma * lambda);
    for (int64_t i = 0; i < n; ++i) {
        float gae = 0.0f;
        for (int64_t t = T - 1; t >= 0; --t) {
            float mask = 1.0f - (dones[t * n + i] ? 1.0f : 0.0f);
            float a = g * values[(t + 1) * n + i];
            a = a * mask;
            float delta = rewards[t * n + i] + a;
            delta = delta - values[t * n + i];
            float b = gl * mask;
            b = b * gae;
            gae = delta + b;
            adv[t * n + i] = gae;
        }
    }
}
