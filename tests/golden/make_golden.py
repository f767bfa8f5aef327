#!/usr/bin/env python
"""Generate the golden fixtures in tests/golden/ by running the REFERENCE.

Runs only where the reference checkout exists (/root/reference, or
$RL101_REFERENCE): it imports ``delivery_drone.game.game_engine.DroneGame``
read-only (``python -B``; an empty ``pygame`` module is injected because
``render_mode=None`` never touches it — game_engine.py:27, 306), pokes the
engine's attributes to the fixture inputs and records what ``step()`` /
``reset()`` return.  The outputs are data (inputs + expected outputs); no
reference source is copied.  The GPU box never runs this script: it only
reads the .npz / .json files written here.

    python -B tests/golden/make_golden.py                  # every fixture
    python -B tests/golden/make_golden.py --only policy    # policy.npz alone
"""
from __future__ import annotations

import json
import os
import sys
import types

sys.dont_write_bytecode = True

import numpy as np  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
REF = os.environ.get("RL101_REFERENCE", "/root/reference")

ACTION_KEYS = ("main_thrust", "left_thrust", "right_thrust")
OBS_KEYS = ("drone_x", "drone_y", "drone_vx", "drone_vy", "drone_angle", "drone_angular_vel",
            "drone_fuel", "platform_x", "platform_y", "distance_to_platform", "dx_to_platform",
            "dy_to_platform", "speed", "landed", "crashed")


def import_reference():
    if not os.path.isdir(os.path.join(REF, "delivery_drone", "game")):
        raise SystemExit(f"reference not found at {REF}; fixtures are committed, nothing to do")
    sys.modules.setdefault("pygame", types.ModuleType("pygame"))
    sys.path.insert(0, REF)
    from delivery_drone.game import config as ref_config  # noqa: E402
    from delivery_drone.game.game_engine import DroneGame  # noqa: E402
    return DroneGame, ref_config


DroneGame, ref_config = import_reference()


def act_dict(bits: int) -> dict:
    return {k: (bits >> i) & 1 for i, k in enumerate(ACTION_KEYS)}


def obs_vec(state: dict) -> list:
    return [float(state[k]) for k in OBS_KEYS]


def new_game(randomize_drone=False, randomize_platform=False, moving=False):
    g = DroneGame(render_mode=None, randomize_drone=randomize_drone, randomize_platform=randomize_platform)
    g.platform.moving = moving
    return g


def poke(g, s: dict):
    d = g.drone
    d.x, d.y, d.vx, d.vy = s["x"], s["y"], s["vx"], s["vy"]
    d.angle, d.angular_velocity, d.fuel = s["angle"], s["omega"], s["fuel"]
    d.crashed = bool(s.get("crashed", False))
    d.landed = bool(s.get("landed", False))
    g.platform.x, g.platform.y = s["px"], s["py"]
    g.platform.direction = int(s.get("direction", 1))
    g.steps = int(s.get("steps", 0))
    g.total_reward = s.get("total", 0.0)
    g.done = bool(s.get("done", False))


def record_step(g, s: dict, bits: int) -> dict:
    poke(g, s)
    state, reward, done, info = g.step(act_dict(bits))
    d = g.drone
    return dict(
        x=float(d.x), y=float(d.y), vx=float(d.vx), vy=float(d.vy), angle=float(d.angle),
        omega=float(d.angular_velocity), fuel=float(d.fuel), px=float(g.platform.x), py=float(g.platform.y),
        direction=int(g.platform.direction), reward=float(reward), done=bool(done), landed=bool(d.landed),
        crashed=bool(d.crashed), steps=int(g.steps), total=float(g.total_reward), obs=obs_vec(state),
        info_distance=float(info["distance_to_platform"]), info_speed=float(info["speed"]),
        needs_reset=bool(info.get("needs_reset", False)))


# --------------------------------------------------------------------------
# Random single-step records
# --------------------------------------------------------------------------
def f32(a):
    return np.asarray(a, dtype=np.float32).astype(np.float64)


def draw_states(rng, m: int, kind: str) -> dict:
    """Fixture input states, every float exactly representable in float32."""
    px = rng.integers(100, 700, m).astype(np.float64)
    py = rng.integers(100, 550, m).astype(np.float64)
    if kind == "broad":
        s = dict(x=f32(rng.uniform(-60, 860, m)), y=f32(rng.uniform(-60, 660, m)),
                 vx=f32(rng.uniform(-8, 8, m)), vy=f32(rng.uniform(-8, 12, m)),
                 angle=f32(rng.uniform(-180, 180, m)), omega=f32(rng.uniform(-6, 6, m)))
    elif kind == "pad":  # bottom centre within +-12 px of the pad box, slow, near upright
        ang = rng.uniform(-25, 25, m)
        bx = px + rng.uniform(-62, 62, m)
        by = py + rng.uniform(-22, 22, m)
        rad = np.radians(ang)
        sp = rng.uniform(0, 3.4, m)
        th = rng.uniform(0, 2 * np.pi, m)
        s = dict(x=f32(bx + 10 * np.sin(rad)), y=f32(by - 10 * np.cos(rad)),
                 vx=f32(sp * np.cos(th)), vy=f32(sp * np.sin(th) - 0.3),
                 angle=f32(ang), omega=f32(rng.uniform(-1.5, 1.5, m)))
    elif kind == "ground":  # around the y > 550 ground line, on and off the pad
        py = rng.integers(530, 550, m).astype(np.float64)
        s = dict(x=f32(px + rng.uniform(-80, 80, m)), y=f32(rng.uniform(540, 560, m)),
                 vx=f32(rng.uniform(-4, 4, m)), vy=f32(rng.uniform(-2, 5, m)),
                 angle=f32(rng.uniform(-30, 30, m)), omega=f32(rng.uniform(-3, 3, m)))
    elif kind == "bounds":  # around the +-50 px out-of-bounds margins
        edge = rng.integers(0, 4, m)
        x = np.where(edge == 0, rng.uniform(-53, -47, m), np.where(edge == 1, rng.uniform(847, 853, m),
                                                                   rng.uniform(0, 800, m)))
        y = np.where(edge == 2, rng.uniform(-53, -47, m), np.where(edge == 3, rng.uniform(546, 553, m),
                                                                   rng.uniform(0, 540, m)))
        s = dict(x=f32(x), y=f32(y), vx=f32(rng.uniform(-4, 4, m)), vy=f32(rng.uniform(-4, 4, m)),
                 angle=f32(rng.uniform(-180, 180, m)), omega=f32(rng.uniform(-6, 6, m)))
    elif kind == "wrap":  # angle crossing +-180
        ang = rng.choice([-1.0, 1.0], m) * rng.uniform(174, 180, m)
        s = dict(x=f32(rng.uniform(0, 800, m)), y=f32(rng.uniform(0, 500, m)),
                 vx=f32(rng.uniform(-3, 3, m)), vy=f32(rng.uniform(-3, 3, m)),
                 angle=f32(ang), omega=f32(-np.sign(ang) * rng.uniform(0, 6, m)))
    else:
        raise ValueError(kind)
    s["px"], s["py"] = px, py
    fuel = rng.integers(0, 1001, m).astype(np.float64)
    low = rng.random(m) < 0.15
    fuel[low] = rng.integers(0, 4, int(low.sum()))
    s["fuel"] = fuel
    s["steps"] = rng.integers(0, 600, m).astype(np.int32)
    s["total"] = f32(rng.uniform(-60, 10, m))
    s["done"] = rng.random(m) < 0.04
    s["direction"] = rng.choice([-1, 1], m)
    s["action"] = rng.integers(0, 8, m).astype(np.uint8)
    return s


def single_step_set(rng, counts: dict, moving=False) -> dict:
    ins = {}
    for kind, m in counts.items():
        for k, v in draw_states(rng, m, kind).items():
            ins.setdefault(k, []).append(v)
    ins = {k: np.concatenate(v) for k, v in ins.items()}
    if moving:  # platform near the bounce points too
        sel = rng.random(ins["px"].shape[0]) < 0.3
        ins["px"][sel] = rng.choice([49.0, 50.0, 51.0, 749.0, 750.0, 751.0], int(sel.sum()))
    n = ins["x"].shape[0]
    g = new_game(moving=moving)
    outs = {}
    for i in range(n):
        s = {k: (v[i].item() if hasattr(v[i], "item") else v[i]) for k, v in ins.items()}
        r = record_step(g, s, int(ins["action"][i]))
        for k, v in r.items():
            outs.setdefault(k, []).append(v)
    rec = {f"in_{k}": np.asarray(v) for k, v in ins.items()}
    rec.update({f"out_{k}": np.asarray(v) for k, v in outs.items()})
    return rec


# --------------------------------------------------------------------------
# Edge cases and exact-threshold probes
# --------------------------------------------------------------------------
def base_state(**kw) -> dict:
    s = dict(x=400.0, y=100.0, vx=0.0, vy=0.0, angle=0.0, omega=0.0, fuel=1000.0, px=400.0, py=500.0,
             steps=0, total=0.0, done=False, direction=1)
    s.update(kw)
    return s


def search_double(f, target, lo, hi):
    """Smallest double v in [lo, hi] with f(v) >= target (f monotone)."""
    lo, hi = float(lo), float(hi)
    for _ in range(200):
        mid = (lo + hi) / 2
        if mid in (lo, hi):
            break
        if f(mid) >= target:
            hi = mid
        else:
            lo = mid
    return hi


def edge_cases() -> list:
    cases = []

    def add(name, s, bits, f64_only=False):
        g = new_game()
        cases.append(dict(name=name, state=s, action=bits, f64_only=f64_only, expect=record_step(g, dict(s), bits)))

    add("spawn_over_pad_lands", base_state(x=400.0, y=480.0, px=400.0, py=500.0), 0)
    add("fuel1_main_left", base_state(fuel=1.0), 0b011)
    add("fuel1_main_only", base_state(fuel=1.0), 0b001)
    add("fuel2_main_right", base_state(fuel=2.0), 0b101)
    add("fuel0_no_thrust", base_state(fuel=0.0), 0b111)
    add("angle_wrap_pos", base_state(angle=179.0, omega=3.0), 0)
    add("angle_wrap_neg", base_state(angle=-179.0, omega=-3.0), 0)
    add("angle_exactly_180", base_state(angle=177.0, omega=3.0), 0)
    add("ground_off_pad", base_state(x=100.0, y=552.0, vy=1.0, px=600.0, py=540.0), 0)
    add("oob_left", base_state(x=-49.5, vx=-1.0), 0)
    add("oob_right", base_state(x=849.5, vx=1.0), 0)
    add("oob_top", base_state(y=-49.0, vy=-1.5), 0)
    add("on_pad_fast_above_ground", base_state(x=300.0, y=380.0, vy=3.5, px=300.0, py=400.0), 0)
    add("on_pad_fast_below_ground", base_state(x=300.0, y=548.0, vy=3.5, px=300.0, py=560.0), 0)
    add("on_pad_tilted", base_state(x=300.0, y=380.0, vy=0.5, angle=25.0, px=300.0, py=400.0), 0)
    add("landing_beats_fuel_out", base_state(x=300.0, y=380.0, vy=0.5, fuel=1.0, px=300.0, py=400.0), 0b001)
    add("sticky_done", base_state(done=True, steps=17, total=-3.5), 0b111)
    add("far_shaping_negative", base_state(x=-40.0, y=-40.0, px=699.0, py=549.0), 0)
    add("main_thrust_at_angle", base_state(angle=33.0, omega=0.7), 0b001)
    add("all_thrusters", base_state(angle=-12.5, omega=-0.4, vx=1.25, vy=-0.75), 0b111)
    # exact thresholds, reachable only with double inputs
    g = new_game()

    def post_speed(vx):
        return float(np.sqrt((vx * 0.99) ** 2 + ((0.0 + 0.3) * 0.99) ** 2))

    vx3 = search_double(post_speed, 3.0, 2.9, 3.1)
    add("speed_at_3_plus", base_state(x=300.0, y=380.0, vx=vx3, px=300.0, py=400.0), 0, f64_only=True)
    vx3m = np.nextafter(vx3, 0.0)
    add("speed_at_3_minus", base_state(x=300.0, y=380.0, vx=float(vx3m), px=300.0, py=400.0), 0, f64_only=True)
    # bottom exactly on the pad's left edge after the update (angle 0 -> bx = x)
    x_edge = search_double(lambda x: x + 0.0 * 0.99, 250.0, 249.0, 251.0)
    add("pad_left_edge", base_state(x=x_edge, y=380.0, px=300.0, py=400.0), 0, f64_only=True)
    add("pad_left_edge_minus", base_state(x=float(np.nextafter(x_edge, 0.0)), y=380.0, px=300.0, py=400.0), 0,
        f64_only=True)
    return cases


# --------------------------------------------------------------------------
# Trajectories
# --------------------------------------------------------------------------
def traj_fixed(frames=1000) -> dict:
    """Config 1: one drone, fixed spawn, actions rng(0).integers(0, 8, 1000),
    reset as soon as an episode ends (game_engine.py:59-138)."""
    acts = np.random.default_rng(0).integers(0, 8, frames).astype(np.uint8)
    g = new_game(randomize_drone=False, randomize_platform=False)
    g.reset()
    obs, rew, done, reset_obs, state = [], [], [], [], []
    for t in range(frames):
        st, r, d, info = g.step(act_dict(int(acts[t])))
        obs.append(obs_vec(st))
        rew.append(float(r))
        done.append(bool(d))
        dr = g.drone
        state.append([dr.x, dr.y, dr.vx, dr.vy, dr.angle, dr.angular_velocity, dr.fuel])
        if d:
            reset_obs.append(obs_vec(g.reset()))
        else:
            reset_obs.append([np.nan] * 15)
    return dict(actions=acts, obs=np.array(obs), reward=np.array(rew), done=np.array(done),
                reset_obs=np.array(reset_obs), state=np.array(state, dtype=np.float64))


def traj_batch(games=32, frames=400, seed=1234, randomize_drone=True, moving=False) -> dict:
    """`games` reference engines with random spawns; every reset's spawn is
    recorded so the batched engine can be replayed on the same episodes."""
    np.random.seed(seed)  # the reference draws spawns from numpy's global RNG
    acts = np.random.default_rng(seed + 1).integers(0, 8, (frames, games)).astype(np.uint8)
    gs = [new_game(randomize_drone=randomize_drone, randomize_platform=True, moving=moving) for _ in range(games)]
    spawn0 = []
    for g in gs:
        g.reset()
        spawn0.append([g.drone.x, g.drone.y, g.platform.x, g.platform.y])
    obs = np.zeros((frames, games, 15))
    rew = np.zeros((frames, games))
    done = np.zeros((frames, games), dtype=bool)
    events = []  # (t, game, x, y, px, py): spawn used from frame t + 1 on
    for t in range(frames):
        for b, g in enumerate(gs):
            st, r, d, _ = g.step(act_dict(int(acts[t, b])))
            obs[t, b] = obs_vec(st)
            rew[t, b] = r
            done[t, b] = d
            if d:
                g.reset()
                events.append([t, b, g.drone.x, g.drone.y, g.platform.x, g.platform.y])
    return dict(actions=acts, spawn0=np.array(spawn0, dtype=np.float64), obs=obs, reward=rew, done=done,
                events=np.array(events, dtype=np.float64).reshape(-1, 6))


def reset_facts(draws=20000, seed=7) -> dict:
    np.random.seed(seed)
    g = new_game(randomize_drone=True, randomize_platform=True)
    xs, ys, pxs, pys = [], [], [], []
    for _ in range(draws):
        g.reset()
        xs.append(g.drone.x); ys.append(g.drone.y); pxs.append(g.platform.x); pys.append(g.platform.y)
    st = g.reset()
    facts = {
        "draws": draws,
        "drone_x": [int(min(xs)), int(max(xs))], "drone_y": [int(min(ys)), int(max(ys))],
        "platform_x": [int(min(pxs)), int(max(pxs))], "platform_y": [int(min(pys)), int(max(pys))],
        "all_integer": bool(all(float(v).is_integer() for v in xs + ys + pxs + pys)),
        "fixed_drone": [ref_config.DRONE_START_X, ref_config.DRONE_START_Y],
        "fixed_platform": [ref_config.WINDOW_WIDTH // 2, ref_config.PLATFORM_Y],
        "reset_obs_tail": obs_vec(st)[2:7] + obs_vec(st)[12:],
        "episode_after_20001_resets": g.episode,
    }
    return facts


def notebook_kats() -> dict:
    """The two known-answer tests recorded in the reference's notebooks.

    Inputs reconstructed from the recorded reset states; expected values are
    the printed outputs (data), re-derived here by the reference itself."""
    out = {}
    # Policy_Gradients_inference.ipynb:52-79: reset to drone (507, 185), platform
    # (210, 128), then {main:1, left:1, right:0} twelve times (steps=12, fuel 964).
    g = new_game()
    poke(g, base_state(x=507, y=185, px=210, py=128))
    g.episode = 1
    for _ in range(12):
        st, r, d, info = g.step({"main_thrust": 1, "left_thrust": 1, "right_thrust": 0})
    nb1 = {"drone_x": 0.6303063103052077, "drone_y": 0.27143029172515365, "drone_vx": -0.07620077073819269,
           "drone_vy": -0.32998130054135, "drone_angle": -0.10889472218633672,
           "drone_angular_vel": -0.26199475003229683, "drone_fuel": 0.964, "speed": 0.3386653453898928,
           "distance_to_platform": 0.37037827112753247, "dx_to_platform": -0.36780631030520766,
           "dy_to_platform": -0.058096958391820316, "reward": -0.0592605233804052,
           "total_reward": -0.7206733615676174, "info_angle": -19.60104999354061,
           "info_distance": 296.302616902026, "info_speed": 3.3866534538989277, "steps": 12}
    got1 = {k: float(st[k]) for k in OBS_KEYS[:13]}
    got1.update(reward=float(r), total_reward=float(info["total_reward"]), info_angle=float(info["angle"]),
                info_distance=float(info["distance_to_platform"]), info_speed=float(info["speed"]),
                steps=int(info["steps"]))
    for k, v in nb1.items():
        assert got1[k] == v, (k, got1[k], v)
    out["policy_gradients_inference"] = dict(
        source="Policy_Gradients_inference.ipynb:52-79", start=dict(x=507, y=185, px=210, py=128),
        action=0b011, frames=12, expect=nb1)
    # Actor_Critic_PPO.ipynb:286-301: drone (688, 152), platform (631, 113), one
    # step without thrust.
    g = new_game()
    poke(g, base_state(x=688, y=152, px=631, py=113))
    st, r, d, info = g.step({})
    nb2 = {"drone_x": 0.86, "drone_y": 0.2538283333333333, "drone_vy": 0.029699999999999997,
           "platform_x": 0.78875, "platform_y": 0.18833333333333332,
           "distance_to_platform": 0.08654166454120524, "dx_to_platform": -0.07125,
           "dy_to_platform": -0.065495, "speed": 0.029699999999999997, "steps": 1}
    for k, v in nb2.items():
        assert st[k] == v, (k, st[k], v)
    # the same cell prints calc_reward(state) with prev_state None (:309-316)
    shaped = notebook_reward_fn()(st, None)
    nb3 = {"time_penalty": -0.5717729518600626, "vertical_position": -0.26198, "total": -0.76198}
    for k, v in nb3.items():
        assert shaped[k] == v, (k, shaped[k], v)
    out["actor_critic_ppo"] = dict(source="Actor_Critic_PPO.ipynb:286-301",
                                   start=dict(x=688, y=152, px=631, py=113), action=0, frames=1, expect=nb2,
                                   shaped_source="Actor_Critic_PPO.ipynb:309-316", shaped_total=nb3["total"])
    return out


# --------------------------------------------------------------------------
# The notebooks' shaped reward
# --------------------------------------------------------------------------
def notebook_reward_fn():
    """calc_reward from Actor_Critic_PPO.ipynb, executed from the notebook's
    own cell source (read at generation time; nothing is copied)."""
    import json as _json
    import math
    from types import SimpleNamespace
    from delivery_drone.game.socket_client import DroneState
    import rl_helpers.scalers as scalers
    nb = _json.load(open(os.path.join(REF, "Actor_Critic_PPO.ipynb")))
    ns = {"np": np, "math": math, "DroneState": DroneState}
    ns.update({k: getattr(scalers, k) for k in dir(scalers) if not k.startswith("_")})
    for cell in nb["cells"]:
        src = "".join(cell["source"])
        if cell["cell_type"] == "code" and ("def calc_velocity_alignment" in src or "def calc_reward" in src):
            exec(compile(src, "Actor_Critic_PPO.ipynb", "exec"), ns)
    calc = ns["calc_reward"]

    def total(state_dict, prev_dist):
        prev = None if prev_dist is None else SimpleNamespace(distance_to_platform=prev_dist)
        return calc(SimpleNamespace(**state_dict), prev_state=prev)

    return total


def shaped_set(rng, counts: dict, max_steps: int = 300) -> dict:
    """Single steps whose next_state goes through the notebook reward, with
    prev_state None / near / far and step counts around max_steps; the
    timeout rule of collect_episodes_ppo (Actor_Critic_PPO.ipynb:886-888)."""
    reward = notebook_reward_fn()
    ins = {}
    for kind, m in counts.items():
        for k, v in draw_states(rng, m, kind).items():
            ins.setdefault(k, []).append(v)
    ins = {k: np.concatenate(v) for k, v in ins.items()}
    n = ins["x"].shape[0]
    ins["done"][:] = False
    ins["steps"] = np.where(rng.random(n) < 0.3, rng.integers(max_steps - 3, max_steps + 2, n),
                            rng.integers(0, max_steps - 3, n)).astype(np.int32)
    g = new_game()
    prev = np.full(n, np.nan)
    out_total, out_shaped, out_done, parts = [], [], [], []
    for i in range(n):
        s = {k: (v[i].item() if hasattr(v[i], "item") else v[i]) for k, v in ins.items()}
        poke(g, s)
        st, _, done, _ = g.step(act_dict(int(ins["action"][i])))
        d = st["distance_to_platform"]
        mode = rng.integers(0, 4)
        pd = None if mode == 0 else d + rng.uniform(-0.004, 0.004) if mode == 1 else \
            d + rng.choice([-0.001, 0.001, 0.0]) if mode == 2 else float(rng.uniform(0, 1.2))
        prev[i] = np.nan if pd is None else pd
        r = reward(st, pd)
        tot = r["total"]
        shaped, sdone = tot, bool(done)
        if g.steps >= max_steps:
            if not st["landed"]:
                shaped -= 500
            sdone = True
        out_total.append(tot)
        out_shaped.append(shaped)
        out_done.append(sdone)
    rec = {f"in_{k}": np.asarray(v) for k, v in ins.items()}
    rec.update(in_prev=prev, max_steps=np.int32(max_steps), out_total=np.asarray(out_total),
               out_shaped=np.asarray(out_shaped), out_shaped_done=np.asarray(out_done))
    return rec


def gae_set(seed=5, T=257, cols=48, gamma=0.99, lam=0.95) -> dict:
    """compute_gae of Actor_Critic_PPO.ipynb:733-787 (executed from the cell),
    column by column, on CPU float32 torch tensors."""
    import json as _json
    import torch
    nb = _json.load(open(os.path.join(REF, "Actor_Critic_PPO.ipynb")))
    ns = {"torch": torch}
    for cell in nb["cells"]:
        src = "".join(cell["source"])
        if cell["cell_type"] == "code" and "def compute_gae" in src:
            exec(compile(src, "Actor_Critic_PPO.ipynb", "exec"), ns)
    compute_gae = ns["compute_gae"]
    rng = np.random.default_rng(seed)
    rewards = rng.normal(0, 30, (T, cols)).astype(np.float32)
    rewards[rng.random((T, cols)) < 0.05] = -300.0
    values = rng.normal(0, 50, (T + 1, cols)).astype(np.float32)
    dones = rng.random((T, cols)) < 0.02
    dones[-1, ::3] = True
    adv = np.zeros((T, cols), dtype=np.float32)
    for j in range(cols):
        a = compute_gae(rewards[:, j].tolist(), values[:, j], dones[:, j].tolist(), gamma=gamma, lambda_=lam,
                        device=torch.device("cpu"))
        adv[:, j] = a.numpy()
    ret = (torch.from_numpy(adv) + torch.from_numpy(values[:T])).numpy()
    return dict(rewards=rewards, values=values, dones=dones, advantages=adv, returns=ret,
                gamma=np.float64(gamma), lam=np.float64(lam))


# The REINFORCE notebook's reward (the widening of SURVEY §8(f) row 1)
def reinforce_reward_fn():
    """calc_reward from Policy_Gradients.ipynb (REINFORCE), executed from the
    notebook's own cells (calc_velocity_alignment :128-153, calc_reward
    :162-238) with rl_helpers/scalers.py; read at generation time, nothing is
    copied."""
    import json as _json
    import math
    from types import SimpleNamespace
    from delivery_drone.game.socket_client import DroneState
    import rl_helpers.scalers as scalers
    nb = _json.load(open(os.path.join(REF, "Policy_Gradients.ipynb")))
    ns = {"np": np, "math": math, "DroneState": DroneState}
    ns.update({k: getattr(scalers, k) for k in dir(scalers) if not k.startswith("_")})
    for cell in nb["cells"]:
        src = "".join(cell["source"])
        if cell["cell_type"] == "code" and ("def calc_velocity_alignment" in src or "def calc_reward" in src):
            exec(compile(src, "Policy_Gradients.ipynb", "exec"), ns)
    calc = ns["calc_reward"]
    return lambda state_dict: calc(SimpleNamespace(**state_dict))


def reinforce_set(rng, counts: dict, max_steps: int = 300) -> dict:
    """Single steps whose next_state goes through the REINFORCE notebook's
    calc_reward, with step counts around max_steps for collect_episodes'
    timeout (Policy_Gradients.ipynb:590-593: -500 unless landed, done)."""
    reward = reinforce_reward_fn()
    ins = {}
    for kind, m in counts.items():
        for k, v in draw_states(rng, m, kind).items():
            ins.setdefault(k, []).append(v)
    ins = {k: np.concatenate(v) for k, v in ins.items()}
    n = ins["x"].shape[0]
    ins["done"][:] = False
    ins["steps"] = np.where(rng.random(n) < 0.3, rng.integers(max_steps - 3, max_steps + 2, n),
                            rng.integers(0, max_steps - 3, n)).astype(np.int32)
    g = new_game()
    out_total, out_shaped, out_done = [], [], []
    for i in range(n):
        s = {k: (v[i].item() if hasattr(v[i], "item") else v[i]) for k, v in ins.items()}
        poke(g, s)
        st, _, done, _ = g.step(act_dict(int(ins["action"][i])))
        tot = reward(st)["total"]
        shaped, sdone = tot, bool(done)
        if g.steps >= max_steps:
            if not st["landed"]:
                shaped -= 500
            sdone = True
        out_total.append(tot)
        out_shaped.append(shaped)
        out_done.append(sdone)
    rec = {f"in_{k}": np.asarray(v) for k, v in ins.items()}
    rec.update(max_steps=np.int32(max_steps), out_total=np.asarray(out_total),
               out_shaped=np.asarray(out_shaped), out_shaped_done=np.asarray(out_done))
    return rec


# The notebooks' policy / value networks
def policy_set(seed=11, games=24, frames=120) -> dict:
    """DroneGamerBoi / DroneTeacherBoi of Actor_Critic_PPO.ipynb:376-424,
    executed from the notebook's cells, with the trained weights of
    models/actor-critic-ppo/*.pth (state_dicts, loaded weights_only=True).
    Inputs are observations of reference games under random actions plus
    synthetic rows; outputs are the notebook models' float32 CPU results and
    Bernoulli.log_prob of fixed action draws (:857-859).  The weights are
    stored as plain float arrays so the GPU box can rebuild the networks."""
    import json as _json
    import torch
    from torch import nn
    from torch.distributions import Bernoulli
    nb = _json.load(open(os.path.join(REF, "Actor_Critic_PPO.ipynb")))
    ns = {"torch": torch, "nn": nn, "np": np, "device": torch.device("cpu"), "DroneState": type("DroneState", (), {})}
    for cell in nb["cells"]:
        src = "".join(cell["source"])
        if cell["cell_type"] == "code" and ("class DroneGamerBoi" in src or "class DroneTeacherBoi" in src):
            exec(compile(src, "Actor_Critic_PPO.ipynb", "exec"), ns)
    actor, critic = ns["DroneGamerBoi"](), ns["DroneTeacherBoi"]()
    mdir = os.path.join(REF, "models", "actor-critic-ppo")
    actor.load_state_dict(torch.load(os.path.join(mdir, "drone_policy_v1.pth"), map_location="cpu",
                                     weights_only=True))
    critic.load_state_dict(torch.load(os.path.join(mdir, "drone_critic_v1.pth"), map_location="cpu",
                                      weights_only=True))
    rng = np.random.default_rng(seed)
    # DroneGame.reset draws its spawns from numpy's global RNG (game_engine.py:66-85):
    # seeded here so that the fixture regenerates byte for byte
    np.random.seed(seed)
    rows = []
    for g in range(games):
        game = new_game(randomize_drone=True, randomize_platform=True)
        state = game.reset()
        for _ in range(frames):
            rows.append(obs_vec(state))
            state, _, done, _ = game.step(act_dict(int(rng.integers(0, 8))))
            if done:
                rows.append(obs_vec(state))
                state = game.reset()
    obs = np.asarray(rows, dtype=np.float32)
    synth = rng.normal(0, 1.5, (256, 15)).astype(np.float32)
    synth[:, 13:] = (rng.random((256, 2)) < 0.1).astype(np.float32)
    synth[0] = 0.0
    obs = np.concatenate([obs, synth])
    with torch.no_grad():
        x = torch.from_numpy(obs)
        probs = actor(x)
        values = critic(x)
    actions = (rng.random((obs.shape[0], 3)) < 0.5).astype(np.float32)
    log_prob = Bernoulli(probs=probs).log_prob(torch.from_numpy(actions)).sum(dim=1)
    out = dict(obs=obs, probs=probs.numpy(), values=values.numpy(), actions=actions, log_prob=log_prob.numpy())
    for tag, net in (("actor", actor), ("critic", critic)):
        for k, v in net.state_dict().items():
            out[f"{tag}.{k}"] = v.numpy()
    return out


def main():
    out = HERE
    args = sys.argv[1:]
    if args[:1] == ["--out"]:  # regenerate into another directory (tests/test_golden_regen.py)
        out, args = args[1], args[2:]
    only = {"policy": lambda: np.savez_compressed(os.path.join(out, "policy.npz"), **policy_set()),
            "reinforce": lambda: np.savez_compressed(os.path.join(out, "reinforce_reward.npz"),
                                                     **reinforce_set(np.random.default_rng(991),
                                                                     REINFORCE_COUNTS))}
    if args[:1] == ["--only"]:
        only[args[1]]()
        print(f"{args[1]} fixture written to", out)
        return
    write_all(out)


REINFORCE_COUNTS = {"broad": 1200, "pad": 1200, "ground": 400, "bounds": 200}


def write_all(HERE):
    rng = np.random.default_rng(20261015)
    kats = notebook_kats()
    with open(os.path.join(HERE, "kat_notebooks.json"), "w") as f:
        json.dump(kats, f, indent=1)
    np.savez_compressed(os.path.join(HERE, "single_step.npz"),
                        **single_step_set(rng, {"broad": 2400, "pad": 1600, "ground": 800, "bounds": 600,
                                                "wrap": 400}))
    np.savez_compressed(os.path.join(HERE, "single_step_moving.npz"),
                        **single_step_set(rng, {"broad": 600, "pad": 400}, moving=True))
    # wind: dead in the reference (wind_x/y never set); exercised with set values
    ref_config.WIND_ENABLED = True
    try:
        wind = single_step_set_wind(rng)
    finally:
        ref_config.WIND_ENABLED = False
    np.savez_compressed(os.path.join(HERE, "single_step_wind.npz"), **wind)
    with open(os.path.join(HERE, "edge_cases.json"), "w") as f:
        json.dump(edge_cases(), f, indent=1)
    np.savez_compressed(os.path.join(HERE, "traj_fixed.npz"), **traj_fixed())
    np.savez_compressed(os.path.join(HERE, "traj_random.npz"), **traj_batch())
    np.savez_compressed(os.path.join(HERE, "traj_moving.npz"),
                        **traj_batch(games=8, frames=300, seed=99, moving=True))
    with open(os.path.join(HERE, "reset_facts.json"), "w") as f:
        json.dump(reset_facts(), f, indent=1)
    np.savez_compressed(os.path.join(HERE, "shaped_reward.npz"),
                        **shaped_set(np.random.default_rng(777), {"broad": 1200, "pad": 1200, "ground": 400,
                                                                 "bounds": 200}))
    np.savez_compressed(os.path.join(HERE, "reinforce_reward.npz"),
                        **reinforce_set(np.random.default_rng(991), REINFORCE_COUNTS))
    np.savez_compressed(os.path.join(HERE, "gae.npz"), **gae_set())
    np.savez_compressed(os.path.join(HERE, "policy.npz"), **policy_set())
    print("fixtures written to", HERE)


def single_step_set_wind(rng) -> dict:
    """Like single_step_set, with DroneGame.wind_x / wind_y set (fixture keys
    in_wind_x / in_wind_y hold the values)."""
    wx, wy = 0.0625, -0.03125
    orig_new = globals()["new_game"]

    def windy_game(**kw):
        g = orig_new(**kw)
        g.wind_x, g.wind_y = wx, wy
        return g

    globals()["new_game"] = windy_game
    try:
        rec = single_step_set(rng, {"broad": 300, "pad": 200})
    finally:
        globals()["new_game"] = orig_new
    rec["in_wind_x"] = np.float64(wx)
    rec["in_wind_y"] = np.float64(wy)
    return rec


if __name__ == "__main__":
    main()
