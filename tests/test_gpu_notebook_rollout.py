"""GPU: reward_mode="notebook" through dd_rollout, and the env-level
bookkeeping around the notebook reward's history (round-1 advisor items).

calc_reward (Actor_Critic_PPO.ipynb:164-263) needs the state two frames back
and collect_episodes_ppo caps episodes at max_steps (:886-888).  dd_step keeps
that history in a [2][N] ring; dd_rollout keeps it in registers for K frames.
Both must agree bit for bit, and a step() after a rollout must read the
history the rollout left behind.
"""
import pytest
import torch

import golden_data as gd
from delivery_drone_amd import EnvConfig, VecDroneEnv
from delivery_drone_amd.gae import gae

pytestmark = pytest.mark.gpu


def bits_equal(a, b):
    """Bitwise equality (NaN history slots compare equal to themselves)."""
    if a.dtype == torch.float64:
        return torch.equal(a.view(torch.int64), b.view(torch.int64))
    if a.dtype == torch.float32:
        return torch.equal(a.view(torch.int32), b.view(torch.int32))
    return torch.equal(a, b)


def notebook_twins(n, dev, precision, max_steps, mode="notebook", **cfg):
    c = EnvConfig(**cfg)
    a = VecDroneEnv(n, device=dev, config=c, precision=precision, reward_mode=mode, max_steps=max_steps)
    b = VecDroneEnv(n, device=dev, config=c, precision=precision, reward_mode=mode, max_steps=max_steps)
    a.reset()
    b.reset()
    return a, b


def assert_same_env(a, b):
    for f in gd.FLOAT_FIELDS + ("status", "steps", "episode"):
        assert bits_equal(getattr(a, f), getattr(b, f)), f
    if a.shaped_hist is not None:  # PPO's history (REINFORCE's reward has none)
        assert bits_equal(a.shaped_hist, b.shaped_hist)


@pytest.mark.parametrize("mode", ["notebook", "reinforce"])
@pytest.mark.parametrize("precision", ["f32", "f64"])
@pytest.mark.parametrize("auto_reset", [True, False])
@pytest.mark.parametrize("n", [1037, 4100])
def test_notebook_rollout_equals_step_loop(mode, precision, auto_reset, n, gpu_device):
    k, pre = 90, 3
    roll, loop = notebook_twins(n, gpu_device, precision, 40, mode, randomize_drone=True, auto_reset=auto_reset,
                                seed=5)
    g = torch.Generator(device=gpu_device).manual_seed(7)
    acts = torch.randint(0, 8, (pre + k + 1, n), device=gpu_device, generator=g, dtype=torch.uint8)
    for t in range(pre):  # start mid-episode: the history ring holds real distances
        roll.step(acts[t])
        loop.step(acts[t])
    er = torch.empty(k, n, dtype=roll.float_dtype, device=gpu_device)
    ed = torch.empty(k, n, dtype=torch.bool, device=gpu_device)
    obs, reward, done = roll.rollout(acts[pre:pre + k], engine_reward_out=er, engine_done_out=ed)
    timeouts = 0
    for t in range(k):
        o, r, d, info = loop.step(acts[pre + t])
        assert bits_equal(obs[t], o), t
        assert bits_equal(reward[t], r), t
        assert torch.equal(done[t], d), t
        assert bits_equal(er[t], info["engine_reward"]), t
        assert torch.equal(ed[t], info["engine_done"]), t
        timeouts += int((d & (loop.steps == 40)).sum())
    assert_same_env(roll, loop)
    assert timeouts > 0  # the 40-step cap fired inside the rollout
    if auto_reset:
        assert int(roll.episode.max()) > 1
    # the next step() continues from the history the rollout wrote back
    o1, r1, d1, _ = roll.step(acts[-1])
    o2, r2, d2, _ = loop.step(acts[-1])
    assert bits_equal(o1, o2) and bits_equal(r1, r2) and torch.equal(d1, d2)


@pytest.mark.parametrize("mode", ["notebook", "reinforce"])
def test_notebook_rollout_philox_and_no_obs(mode, gpu_device):
    n, k = 2050, 70
    roll, loop = notebook_twins(n, gpu_device, "f32", 25, mode, randomize_drone=True, auto_reset=True, seed=8)
    _, reward, done = roll.rollout(frames=k, write_obs=False, action_seed=11)
    # the same in-kernel actions, one frame per launch
    r_all, d_all = [], []
    for t in range(k):
        _, r, d = loop.rollout(frames=1, write_obs=False, action_seed=11, action_step=t)
        r_all.append(r[0].clone())
        d_all.append(d[0].clone())
    assert bits_equal(reward, torch.stack(r_all)) and torch.equal(done, torch.stack(d_all))
    assert_same_env(roll, loop)


def test_engine_outputs_only_in_notebook_mode(gpu_device):
    env = VecDroneEnv(64, device=gpu_device)
    env.reset()
    buf = torch.empty(3, 64, device=gpu_device)
    with pytest.raises(ValueError):
        env.rollout(frames=3, engine_reward_out=buf, engine_done_out=buf.bool())
    nb = VecDroneEnv(64, device=gpu_device, reward_mode="notebook")
    with pytest.raises(ValueError):
        nb.rollout(frames=3, engine_reward_out=buf)


def test_fresh_env_history_is_seeded(gpu_device):
    """A notebook-mode env stepped without reset(): the history starts from the
    constructed state (prev_state None for the first frame), as after reset()."""
    n = 300
    fresh = VecDroneEnv(n, device=gpu_device, precision="f64", reward_mode="notebook")
    ref = VecDroneEnv(n, device=gpu_device, precision="f64", reward_mode="notebook")
    ref.load_state_dict({k: v for k, v in fresh.state_dict().items() if k != "shaped_hist"})
    assert bits_equal(fresh.shaped_hist, ref.shaped_hist)
    assert torch.isfinite(fresh.shaped_hist[0]).all() and torch.isnan(fresh.shaped_hist[1]).all()
    acts = torch.randint(0, 8, (6, n), device=gpu_device, dtype=torch.uint8)
    for t in range(6):
        _, r1, d1, _ = fresh.step(acts[t])
        _, r2, d2, _ = ref.step(acts[t])
        assert bits_equal(r1, r2) and torch.equal(d1, d2)
        assert torch.isfinite(r1).all()


def test_state_dict_round_trip_keeps_history(gpu_device):
    n = 500
    a = VecDroneEnv(n, device=gpu_device, reward_mode="notebook", randomize_drone=True, auto_reset=True, seed=2)
    a.reset()
    acts = torch.randint(0, 8, (12, n), device=gpu_device, dtype=torch.uint8)
    for t in range(5):
        a.step(acts[t])
    snap = a.state_dict()
    assert "shaped_hist" in snap
    b = VecDroneEnv(n, device=gpu_device, reward_mode="notebook", randomize_drone=True, auto_reset=True, seed=2)
    b.load_state_dict(snap)
    for t in range(5, 12):
        _, r1, d1, _ = a.step(acts[t])
        _, r2, d2, _ = b.step(acts[t])
        assert bits_equal(r1, r2) and torch.equal(d1, d2), t


def test_render_after_rollout_draws_last_frame_actions(gpu_device):
    env = VecDroneEnv(16, device=gpu_device, randomize_drone=True, seed=3)
    env.reset()
    acts = torch.randint(1, 8, (5, 16), device=gpu_device, dtype=torch.uint8)
    env.step(torch.zeros(16, dtype=torch.uint8, device=gpu_device))
    env.rollout(acts)
    assert torch.equal(env.render([0, 5, 9]), env.render([0, 5, 9], actions=acts[-1]))
    env.rollout(frames=2)  # in-kernel actions: no flames drawn
    assert torch.equal(env.render([1, 2]), env.render([1, 2], actions=torch.zeros(16, dtype=torch.uint8,
                                                                                   device=gpu_device)))


def test_gae_out_buffers_checked(gpu_device):
    T, n = 8, 33
    r = torch.randn(T, n, device=gpu_device)
    v = torch.randn(T + 1, n, device=gpu_device)
    d = torch.zeros(T, n, dtype=torch.bool, device=gpu_device)
    adv, ret = gae(r, v, d)
    a2, r2 = torch.empty_like(adv), torch.empty_like(ret)
    out = gae(r, v, d, out=(a2, r2))
    assert out[0] is a2 and torch.equal(a2, adv) and torch.equal(r2, ret)
    for bad in (torch.empty(T, n - 1, device=gpu_device), torch.empty(T, n, dtype=torch.float64, device=gpu_device),
                torch.empty(n, T, device=gpu_device).t(), torch.empty(T, n)):
        with pytest.raises(ValueError):
            gae(r, v, d, out=(bad, r2))
    with pytest.raises(ValueError):
        gae(r, v, d, out=(a2, None))
    only = gae(r, v, d, returns=False, out=(a2, None))
    assert only is a2
