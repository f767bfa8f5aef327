"""GPU: dd_render (VecDroneEnv.render) against the numpy restatement in
oracle/render.py, pixel for pixel, on lanes chosen to reach every primitive:
rotated sprites (any angle, half off-screen), each flame, the three fuel-bar
colours, landed / crashed game-over frames, and HUD numbers on formatting
edges (ties to even, negative zero, large values).  pygame is absent, so the
rules themselves are unpinned against the reference."""
import numpy as np
import pytest
import torch

from delivery_drone_amd import EnvConfig, VecDroneEnv
from delivery_drone_amd.compat import DroneGame
from oracle import render as R

pytestmark = pytest.mark.gpu

FIELDS = ("x", "y", "vx", "vy", "angle", "fuel", "px", "py", "total_reward", "status", "steps", "episode")


def lanes_for_test(n, seed):
    rng = np.random.default_rng(seed)
    d = {
        "x": rng.uniform(-60, 860, n), "y": rng.uniform(-60, 660, n),
        "vx": rng.uniform(-8, 8, n), "vy": rng.uniform(-8, 12, n),
        "angle": rng.uniform(-180, 180, n), "fuel": rng.integers(0, 1001, n).astype(np.float64),
        "px": rng.integers(100, 700, n).astype(np.float64), "py": rng.integers(100, 550, n).astype(np.float64),
        "total_reward": rng.uniform(-300, 120, n), "status": rng.choice([0, 0, 0, 1 | 2, 1 | 4], n),
        "steps": rng.integers(1, 5000, n), "episode": rng.integers(1, 100000, n),
    }
    # formatting edges: .1f ties (0.25 -> 0.2, 0.75 -> 0.8), -0.0, .0f ties (2.5 -> 2, 3.5 -> 4)
    edge = [dict(angle=0.25, total_reward=0.75, status=1 | 2), dict(angle=-0.04, total_reward=-0.05, status=1 | 4),
            dict(angle=180.0, vx=0.0, vy=0.0, x=397.5, y=300.0, px=400.0, py=300.0),
            dict(angle=-179.95, x=396.5, y=300.0, px=400.0, py=300.0, fuel=0.0),
            dict(angle=90.0, fuel=300.0), dict(angle=-90.0, fuel=100.0, x=10.0, y=590.0),
            dict(x=400.0, y=100.0, angle=0.0, px=400.0, py=500.0, total_reward=1e6, status=1 | 4)]
    for k, e in enumerate(edge):
        for f, v in e.items():
            d[f][k] = v
    return d


def make_env(d, dev, precision):
    n = len(d["x"])
    env = VecDroneEnv(n, device=dev, config=EnvConfig(randomize_drone=True), precision=precision)
    env.reset()
    for f in FIELDS:
        t = getattr(env, f)
        t.copy_(torch.as_tensor(d[f]).to(t.dtype))
    return env


def lane_values(env, i):
    return {f: getattr(env, f)[i].item() for f in FIELDS}


@pytest.mark.parametrize("precision", ["f32", "f64"])
def test_render_matches_oracle(precision, gpu_device):
    n = 48
    d = lanes_for_test(n, 7)
    env = make_env(d, gpu_device, precision)
    acts = torch.as_tensor(np.random.default_rng(1).integers(0, 8, n), dtype=torch.uint8, device=gpu_device)
    frames = env.render(actions=acts).cpu().numpy()
    assert frames.shape == (n, 600, 800, 3)
    for i in range(n):
        ref = R.render(lane_values(env, i), int(acts[i]))
        bad = np.argwhere((frames[i] != ref).any(axis=2))
        assert bad.size == 0, (i, lane_values(env, i), bad[:5].tolist(), frames[i][tuple(bad[0])], ref[tuple(bad[0])])


def test_render_lanes_flags_and_remembered_actions(gpu_device):
    n = 12
    d = lanes_for_test(n, 11)
    env = make_env(d, gpu_device, "f32")
    bits = torch.tensor([7, 1, 2, 4] * 3, dtype=torch.uint8, device=gpu_device)
    three = torch.stack([(bits >> j) & 1 for j in range(3)], dim=1).float()
    env.step(three)  # the flames default to the last step's actions
    sel = [9, 2, 2, 0]
    frames = env.render(lanes=sel, hud=False, game_over=False).cpu().numpy()
    for k, i in enumerate(sel):
        ref = R.render(lane_values(env, i), int(bits[i]) if int(env.steps[i]) > 0 else 0, hud=False, game_over=False)
        assert np.array_equal(frames[k], ref), (k, i)
    out = torch.empty(1, 600, 800, 3, dtype=torch.uint8, device=gpu_device)
    assert env.render(lanes=torch.tensor([5]), out=out) is out
    env.reset()  # a fresh episode shows no flames
    frame = env.render(lanes=3).cpu().numpy()[0]
    assert np.array_equal(frame, R.render(lane_values(env, 3), 0))
    with pytest.raises(IndexError):
        env.render(lanes=[n])
    frames = env.render(lanes=torch.tensor([n, 1, -1], device=gpu_device)).cpu().numpy()
    assert not frames[0].any() and not frames[2].any()  # not a lane: all zero
    assert np.array_equal(frames[1], R.render(lane_values(env, 1), 0))


def test_dronegame_rgb_array(gpu_device):
    g = DroneGame(render_mode="rgb_array", device=gpu_device)
    g.reset()
    g.step({"main_thrust": 1})
    img = g.render()
    assert isinstance(img, np.ndarray) and img.shape == (600, 800, 3) and img.dtype == np.uint8
    ref = R.render(lane_values(g.env, 0), 1)
    assert np.array_equal(img, ref)
    assert DroneGame(render_mode=None, device=gpu_device).render() is None
