"""TEST INFRASTRUCTURE ONLY (CPU baseline, parity checker) — never the product path.

A scalar, one-object-per-drone Python restatement of the reference engine's
step, shaped like ``DroneGame.step`` so that timing it gives the reference's
own per-core speed on a host the reference cannot travel to (SURVEY.md
§8(d), BASELINE.md "CPU baseline"): one game object per drone, a drone and a
pad object, method calls per frame, numpy scalar ufuncs for the trigonometry
and square roots and ``v ** 2`` (glibc ``pow``) for the squares, the ordered
reward cascade, and a fresh observation dict and info dict every frame.

Restated from (file:line in the reference repository):
  physics.rotate_point / normalize_angle / distance  delivery_drone/game/physics.py:6-44
  Drone.apply_thrust / update                        delivery_drone/game/drone.py:44-103
  Drone.get_bottom_center / get_speed / is_upright   delivery_drone/game/drone.py:130-153
  Platform.update / get_bounds / is_point_on_platform delivery_drone/game/platform.py:31-74
  DroneGame.step / get_state / _calculate_reward     delivery_drone/game/game_engine.py:95-216
  _check_landing / _check_crash / _check_out_of_bounds / _get_info  :218-298
  DroneGame.reset                                    :59-93 (draws: Philox, as oracle/drone_oracle.c)

Pinned bit for bit to the reference's own outputs by tests/test_pyloop.py
(tests/golden/single_step.npz, edge_cases.json) and to the C oracle over
multi-frame random-spawn runs.  The reference's defaults only (config.py);
no wind, static pad unless ``platform_moving``.
"""
from __future__ import annotations

import numpy as np

# config.py:17-68
GRAVITY, DRAG, ANGULAR_DRAG = 0.3, 0.99, 0.95
MAIN_THRUST_POWER, SIDE_THRUST_POWER = 0.6, 0.3
MAX_FUEL, FUEL_MAIN, FUEL_SIDE = 1000.0, 2.0, 1.0
DRONE_HEIGHT = 20
PLATFORM_WIDTH, PLATFORM_HEIGHT, PLATFORM_SPEED = 100, 20, 1.0
WIDTH, HEIGHT = 800, 600
MAX_LANDING_VELOCITY, MAX_LANDING_ANGLE = 3.0, 20.0
MARGIN = 50
R_STEP, R_LAND, R_CRASH, R_FUEL, R_OOB = -0.1, 100.0, -100.0, -50.0, -50.0

_M32 = 0xFFFFFFFF


def philox4x32_10(c0, c1, c2, c3, k0, k1, rounds=10):
    """Philox4x32-10 (Salmon et al., SC'11) on Python ints (oracle/drone_oracle.c);
    rounds=7: the spawn stream."""
    for _ in range(rounds):
        p0 = 0xD2511F53 * c0
        p1 = 0xCD9E8D57 * c2
        c0, c1, c2, c3 = ((p1 >> 32) ^ c1 ^ k0) & _M32, p1 & _M32, ((p0 >> 32) ^ c3 ^ k1) & _M32, p0 & _M32
        k0 = (k0 + 0x9E3779B9) & _M32
        k1 = (k1 + 0xBB67AE85) & _M32
    return c0, c1, c2, c3


def _rotate(x, y, angle_deg):
    # physics.rotate_point: np.radians, np.cos, np.sin on a scalar
    rad = np.radians(angle_deg)
    c = np.cos(rad)
    s = np.sin(rad)
    return x * c - y * s, x * s + y * c


def _wrap(angle):
    while angle > 180:
        angle -= 360
    while angle < -180:
        angle += 360
    return angle


def _distance(x1, y1, x2, y2):
    return np.sqrt((x2 - x1) ** 2 + (y2 - y1) ** 2)


class Pad:
    def __init__(self, x=WIDTH // 2, y=HEIGHT - 100, moving=False):
        self.x, self.y = x, y
        self.moving = moving
        self.direction = 1

    def advance(self):
        if not self.moving:
            return
        self.x += PLATFORM_SPEED * self.direction * 1.0
        lo, hi = PLATFORM_WIDTH // 2, WIDTH - PLATFORM_WIDTH // 2
        if self.x <= lo:
            self.x, self.direction = lo, 1
        elif self.x >= hi:
            self.x, self.direction = hi, -1

    def holds(self, px, py):
        hw, hh = PLATFORM_WIDTH / 2, PLATFORM_HEIGHT / 2
        return (self.x - hw <= px <= self.x + hw) and (self.y - hh <= py <= self.y + hh)


class Craft:
    def __init__(self, x=WIDTH / 2, y=100):
        self.x, self.y = x, y
        self.vx = self.vy = 0.0
        self.angle = self.omega = 0.0
        self.fuel = MAX_FUEL
        self.landed = self.crashed = False

    def fire(self, main, left, right):
        if main and self.fuel > 0:
            tx, ty = _rotate(0, -MAIN_THRUST_POWER, self.angle)
            self.vx += tx
            self.vy += ty
            self.fuel -= FUEL_MAIN
        if left and self.fuel > 0:
            self.omega -= SIDE_THRUST_POWER
            self.fuel -= FUEL_SIDE
        if right and self.fuel > 0:
            self.omega += SIDE_THRUST_POWER
            self.fuel -= FUEL_SIDE
        self.fuel = max(0, self.fuel)

    def advance(self):
        if self.crashed or self.landed:
            return
        self.vy += GRAVITY * 1.0
        self.vx *= DRAG
        self.vy *= DRAG
        self.x += self.vx * 1.0
        self.y += self.vy * 1.0
        self.angle += self.omega * 1.0
        self.omega *= ANGULAR_DRAG
        self.angle = _wrap(self.angle)

    def bottom(self):
        ox, oy = _rotate(0, DRONE_HEIGHT / 2, self.angle)
        return self.x + ox, self.y + oy

    def speed(self):
        return np.sqrt(self.vx ** 2 + self.vy ** 2)

    def upright(self):
        return abs(self.angle) <= MAX_LANDING_ANGLE


class Game:
    """One drone game (DroneGame with render_mode=None)."""

    def __init__(self, env_id=0, seed=0, randomize_drone=False, randomize_platform=True, moving=False):
        self.env_id, self.seed = env_id, seed
        self.randomize_drone, self.randomize_platform = randomize_drone, randomize_platform
        self.craft = Craft()
        self.pad = Pad(moving=moving)
        self.steps = 0
        self.total_reward = 0
        self.done = False
        self.episode = 0

    def reset(self):
        self.episode += 1
        e, s = self.env_id, self.seed
        r = philox4x32_10(e & _M32, (e >> 32) & _M32, self.episode & _M32, 0, s & _M32, (s >> 32) & _M32,
                          rounds=7)
        if self.randomize_drone:
            self.craft = Craft(100 + ((r[0] * 601) >> 32), 50 + ((r[1] * 201) >> 32))
        else:
            self.craft = Craft(WIDTH / 2, 100)
        if self.randomize_platform:
            self.pad.x, self.pad.y = 100 + ((r[2] * 600) >> 32), 100 + ((r[3] * 450) >> 32)
        else:
            self.pad.x, self.pad.y = WIDTH // 2, HEIGHT - 100
        self.pad.direction = 1
        self.steps = 0
        self.total_reward = 0
        self.done = False
        return self.observe()

    def step(self, action: dict):
        if self.done:
            info = self.info()
            info["needs_reset"] = True
            return self.observe(), 0, True, info
        self.craft.fire(bool(action.get("main_thrust", 0)), bool(action.get("left_thrust", 0)),
                        bool(action.get("right_thrust", 0)))
        self.craft.advance()
        self.pad.advance()
        reward = self._reward()
        self.total_reward += reward
        self.steps += 1
        return self.observe(), reward, self.done, self.info()

    def _landing(self):
        c = self.craft
        if c.crashed or c.landed:
            return False
        bx, by = c.bottom()
        return self.pad.holds(bx, by) and not c.speed() > MAX_LANDING_VELOCITY and c.upright()

    def _crash(self):
        c = self.craft
        if c.crashed:
            return True
        if c.y > HEIGHT - 50:
            bx, by = c.bottom()
            return not self.pad.holds(bx, by) or c.speed() > MAX_LANDING_VELOCITY or not c.upright()
        return False

    def _reward(self):
        c = self.craft
        r = R_STEP
        if self._landing():
            c.landed = True
            self.done = True
            return r + R_LAND
        if self._crash():
            c.crashed = self.done = True
            return r + R_CRASH
        if c.fuel <= 0:
            c.crashed = self.done = True
            return r + R_FUEL
        if c.x < -MARGIN or c.x > WIDTH + MARGIN or c.y < -MARGIN or c.y > HEIGHT + MARGIN:
            c.crashed = self.done = True
            return r + R_OOB
        return r + (500 - _distance(c.x, c.y, self.pad.x, self.pad.y)) / 5000

    def observe(self):
        c, p = self.craft, self.pad
        dx, dy = p.x - c.x, p.y - c.y
        dist = _distance(c.x, c.y, p.x, p.y)
        return {"drone_x": c.x / WIDTH, "drone_y": c.y / HEIGHT, "drone_vx": c.vx / 10.0,
                "drone_vy": c.vy / 10.0, "drone_angle": c.angle / 180.0, "drone_angular_vel": c.omega / 10.0,
                "drone_fuel": c.fuel / MAX_FUEL, "platform_x": p.x / WIDTH, "platform_y": p.y / HEIGHT,
                "distance_to_platform": dist / WIDTH, "dx_to_platform": dx / WIDTH, "dy_to_platform": dy / HEIGHT,
                "speed": c.speed() / 10.0, "landed": c.landed, "crashed": c.crashed, "steps": self.steps}

    def info(self):
        c, p = self.craft, self.pad
        return {"steps": self.steps, "total_reward": self.total_reward, "episode": self.episode,
                "fuel_remaining": c.fuel, "distance_to_platform": _distance(c.x, c.y, p.x, p.y),
                "speed": c.speed(), "angle": c.angle}


OBS_KEYS = ("drone_x", "drone_y", "drone_vx", "drone_vy", "drone_angle", "drone_angular_vel", "drone_fuel",
            "platform_x", "platform_y", "distance_to_platform", "dx_to_platform", "dy_to_platform", "speed",
            "landed", "crashed")
_ACTION_DICTS = tuple({"main_thrust": a & 1, "left_thrust": (a >> 1) & 1, "right_thrust": (a >> 2) & 1}
                      for a in range(8))


def action_dict(bits: int) -> dict:
    return _ACTION_DICTS[bits & 7]


def bench(lane0: int, lanes: int, steps: int, seed: int = 0) -> tuple:
    """Config-3 workload on `lanes` game objects for `steps` frames: random
    spawn, auto-reset on the frame after done, uniform random 3-bit actions
    (a fixed LCG, drawn outside the games).  Returns (drone-steps, checksum)."""
    games = [Game(lane0 + i, seed, randomize_drone=True, randomize_platform=True) for i in range(lanes)]
    for g in games:
        g.reset()
    state = (seed * 2654435761 + lane0) & _M32
    chk = 0.0
    for _ in range(steps):
        for g in games:
            if g.done:
                g.reset()
            state = (state * 1664525 + 1013904223) & _M32
            obs, reward, done, info = g.step(_ACTION_DICTS[state >> 29])
            chk += reward
    return lanes * steps, float(chk)
