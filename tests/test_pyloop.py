"""CPU: oracle/pyloop.py (the scalar Python-object restatement timed as the
CPU baseline's reference-shaped leg) against the reference's own outputs, bit
for bit, and against the C oracle over random-spawn episodes."""
import numpy as np
import pytest

import golden_data as gd
from delivery_drone_amd import EnvConfig
from oracle import oracle as ora
from oracle import pyloop


def _game(rec, i, moving=False):
    g = pyloop.Game(moving=moving)
    c = g.craft
    c.x, c.y, c.vx, c.vy = (float(rec[f"in_{k}"][i]) for k in ("x", "y", "vx", "vy"))
    c.angle, c.omega, c.fuel = float(rec["in_angle"][i]), float(rec["in_omega"][i]), float(rec["in_fuel"][i])
    g.pad.x, g.pad.y, g.pad.direction = float(rec["in_px"][i]), float(rec["in_py"][i]), int(rec["in_direction"][i])
    g.steps, g.total_reward, g.done = int(rec["in_steps"][i]), float(rec["in_total"][i]), bool(rec["in_done"][i])
    return g


@pytest.mark.parametrize("name,moving", [("single_step.npz", False), ("single_step_moving.npz", True)])
def test_pyloop_matches_reference_records(name, moving):
    rec = gd.npz(name)
    for i in range(rec["in_x"].shape[0]):
        g = _game(rec, i, moving)
        obs, reward, done, info = g.step(pyloop.action_dict(int(rec["in_action"][i])))
        c = g.craft
        got = dict(x=c.x, y=c.y, vx=c.vx, vy=c.vy, angle=c.angle, omega=c.omega, fuel=c.fuel, px=g.pad.x,
                   py=g.pad.y, reward=reward, total=g.total_reward)
        for k, v in got.items():
            assert float(v) == float(rec[f"out_{k}"][i]), (i, k, v, rec[f"out_{k}"][i])
        assert done == bool(rec["out_done"][i]) and g.steps == int(rec["out_steps"][i]), i
        assert c.landed == bool(rec["out_landed"][i]) and c.crashed == bool(rec["out_crashed"][i]), i
        assert g.pad.direction == int(rec["out_direction"][i]), i
        row = [float(obs[k]) for k in pyloop.OBS_KEYS]
        assert row == [float(v) for v in rec["out_obs"][i]], i
        assert float(info["distance_to_platform"]) == float(rec["out_info_distance"][i]), i
        assert float(info["speed"]) == float(rec["out_info_speed"][i]), i
        assert info.get("needs_reset", False) == bool(rec["out_needs_reset"][i]), i


def test_pyloop_edge_cases():
    for case in gd.js("edge_cases.json"):
        s = case["state"]
        g = pyloop.Game()
        c = g.craft
        for k, attr in (("x", "x"), ("y", "y"), ("vx", "vx"), ("vy", "vy"), ("angle", "angle"),
                        ("omega", "omega"), ("fuel", "fuel")):
            setattr(c, attr, float(s[k]))
        g.pad.x, g.pad.y, g.pad.direction = float(s["px"]), float(s["py"]), int(s["direction"])
        g.steps, g.total_reward, g.done = int(s["steps"]), float(s["total"]), bool(s["done"])
        obs, reward, done, _ = g.step(pyloop.action_dict(int(case["action"])))
        e = case["expect"]
        assert float(reward) == float(e["reward"]) and done == bool(e["done"]), case["name"]
        assert float(g.craft.fuel) == float(e["fuel"]) and float(g.craft.y) == float(e["y"]), case["name"]
        assert [float(obs[k]) for k in pyloop.OBS_KEYS] == [float(v) for v in e["obs"]], case["name"]


def test_pyloop_matches_c_oracle_over_episodes():
    # random spawn + auto-reset: the Python-object loop and the C oracle (f64)
    # step the same lanes through several episodes, bit for bit
    n, frames, seed = 64, 300, 7
    cfg = EnvConfig(randomize_drone=True, randomize_platform=True, auto_reset=True, seed=seed)
    o = ora.OracleEnv(n, precision="f64", config=cfg)
    o.reset()
    games = [pyloop.Game(i, seed, randomize_drone=True, randomize_platform=True) for i in range(n)]
    for g in games:
        g.reset()
    rng = np.random.default_rng(1)
    episodes = 0
    for t in range(frames):
        a = rng.integers(0, 8, n).astype(np.uint8)
        oobs, oreward, odone, obs64 = o.step(a)
        for i, g in enumerate(games):
            if g.done:
                g.reset()
                episodes += 1
                obs, reward, done = g.observe(), 0.0, False
            else:
                obs, reward, done, _ = g.step(pyloop.action_dict(int(a[i])))
            assert float(reward) == float(oreward[i]) and done == bool(odone[i]), (t, i)
            assert [float(obs[k]) for k in pyloop.OBS_KEYS] == [float(v) for v in obs64[i]], (t, i)
    assert episodes > 20


def test_pyloop_bench_runs():
    steps, chk = pyloop.bench(0, 8, 20, seed=3)
    assert steps == 160 and np.isfinite(chk)
